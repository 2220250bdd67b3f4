set -o pipefail
cd $GRAFT_REPO_ROOT
MODELS=mlp8 bash scripts/r3b/env_ab.sh m8wtile3 DNN_TUNED_TABLE=bench/tables/m8_w_256_8.json DNN_TUNED_TABLE=bench/tables/m8_w_256_4.json DNN_TUNED_TABLE=bench/tables/m8_w_256_6.json DNN_TUNED_TABLE=bench/tables/m8_w_128_2.json DNN_TUNED_TABLE=bench/tables/m8_w_256_8_w0_8.json "DNN_TUNED_TABLE=bench/tables/m8_w_256_8.json DNN_SPLIT_FINO=1" || exit 1
MODELS=head bash scripts/r3b/env_ab.sh hw1tile DNN_TUNED=1 DNN_TUNED_TABLE=bench/tables/h_w1_128_16.json DNN_TUNED_TABLE=bench/tables/h_w1_128_32.json DNN_TUNED_TABLE=bench/tables/h_w1_256_32.json DNN_TUNED_TABLE=bench/tables/h_w1_256_16.json || exit 1
