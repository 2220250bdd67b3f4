R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
T=$R/bench/tables/r5
step env_w0c11 900 env PREFIX=r5 MODELS=head REPS=4 bash $R/scripts/env_ab.sh w0c11 "DNN_BW_OVERLAP=1" "DNN_TUNED_TABLE=$T/w0_128_c11.json" "DNN_TUNED_TABLE=$T/w0_256_c11_s24.json"
