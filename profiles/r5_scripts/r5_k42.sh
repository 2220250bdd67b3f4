R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_split 900 env PREFIX=r5 MODELS=head REPS=4 bash $R/scripts/env_ab.sh split "DNN_BW_OVERLAP=1" "DNN_SPLIT_FINO=0" "DNN_XSTEP=0"
