R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_xwfirst 900 env PREFIX=r5 MODELS=head REPS=4 bash $R/scripts/env_ab.sh xwfirst "DNN_BW_OVERLAP=1" "DNN_DIAG_XWAIT_FIRST=1"
