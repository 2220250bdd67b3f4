R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
TB=$R/bench/tables/r5
step env_c11 700 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh c11 "DNN_H0_DOUBLE=1" "DNN_TUNED_TABLE=$TB/f0_c11.json" "DNN_TUNED_TABLE=$TB/d1_c11.json" "DNN_TUNED_TABLE=$TB/f0d1_c11.json" "DNN_TUNED_TABLE=$TB/f1_c11.json"
