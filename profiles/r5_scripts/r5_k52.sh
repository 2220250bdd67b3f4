R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_cumask 900 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh cumask "DNN_BW_OVERLAP=1" "DNN_SIDE_CU_MASK=ffffffff" "DNN_SIDE_CU_MASK=77777777" "DNN_SIDE_CU_MASK=55555555" "DNN_SIDE_CU_MASK=11111111"
