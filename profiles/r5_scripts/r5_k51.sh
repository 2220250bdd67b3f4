R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_skip2 900 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh skip2 "DNN_BW_OVERLAP=1" "DNN_DIAG_SKIP=W1" "DNN_DIAG_SKIP=W1,W2,W3" "DNN_DIAG_SKIP=W1,W2,W3,FINO1-3" "DNN_DIAG_SKIP=W0"
