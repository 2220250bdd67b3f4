R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
TB=$R/bench/tables/r5
step env_splits 900 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh splits "DNN_XSTEP=1" "DNN_TUNED_TABLE=$TB/w1_128_s32.json" "DNN_TUNED_TABLE=$TB/w1_128_s16.json" "DNN_TUNED_TABLE=$TB/w0_128_s24.json" "DNN_TUNED_TABLE=$TB/w0_128_s12.json" "DNN_TUNED_TABLE=$TB/w0_128_s9.json" "DNN_TUNED_TABLE=$TB/w2_64_s16.json" "DNN_TUNED_TABLE=$TB/w1s32_w0s24.json" "DNN_XSTEP=0"
