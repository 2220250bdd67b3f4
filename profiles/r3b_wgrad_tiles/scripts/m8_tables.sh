set -o pipefail
cd $GRAFT_REPO_ROOT
MODELS=mlp8 bash scripts/r3b/env_ab.sh m8wtile2 DNN_TUNED_TABLE=bench/tables/m8_w_256_16.json DNN_TUNED_TABLE=bench/tables/m8_w_256_8.json DNN_TUNED_TABLE=bench/tables/m8_w_256_12.json DNN_TUNED_TABLE=bench/tables/m8_w_256_16_w0.json "DNN_TUNED_TABLE=bench/tables/m8_w_256_16.json DNN_SPLIT_FINO=1" || exit 1
