R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
TB=$R/bench/tables/r5
step env_d1 900 env PREFIX=r5 MODELS=head REPS=5 bash $R/scripts/env_ab.sh d1 "DNN_XSTEP=1" "DNN_TUNED_TABLE=$TB/d1_256x128_c11.json" "DNN_TUNED_TABLE=$TB/d1_256x128_c9.json" "DNN_TUNED_TABLE=$TB/w2_128x64_s64.json" "DNN_TUNED_TABLE=$TB/d1c11_w2.json"
