R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
T=$R/bench/tables/r5
step env_m8split 900 env PREFIX=r5 MODELS=mlp8 REPS=4 bash $R/scripts/env_ab.sh m8split "DNN_BW_OVERLAP=1" "DNN_TUNED_TABLE=$T/m8_wgrad_s4.json" "DNN_TUNED_TABLE=$T/m8_wgrad_s6.json" "DNN_TUNED_TABLE=$T/m8_wgrad_s12.json"
