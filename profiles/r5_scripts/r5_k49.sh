R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_sorder 900 env PREFIX=r5 MODELS=head REPS=4 bash $R/scripts/env_ab.sh sorder "DNN_BW_OVERLAP=1" "DNN_SIDE_ORDER=3,1,2" "DNN_SIDE_ORDER=2,3,1"
