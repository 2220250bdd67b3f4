# wgrad tile A/B through tuned-table overrides (headline W0, mlp8 1024x1024 wgrads)
set -o pipefail
cd $GRAFT_REPO_ROOT
MODELS=head bash scripts/r3b/env_ab.sh w0tile DNN_TUNED=1 DNN_TUNED_TABLE=bench/tables/w0_256_32.json DNN_TUNED_TABLE=bench/tables/w0_256_24.json DNN_TUNED_TABLE=bench/tables/w0_256_16.json || exit 1
MODELS=mlp8 bash scripts/r3b/env_ab.sh m8wtile DNN_TUNED=1 DNN_TUNED_TABLE=bench/tables/m8_w_256_16.json || exit 1
