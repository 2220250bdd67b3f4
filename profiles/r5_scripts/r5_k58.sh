R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_skip_m8 900 env PREFIX=r5 MODELS=mlp8 REPS=3 bash $R/scripts/env_ab.sh skip_m8 "DNN_BW_OVERLAP=1" "DNN_DIAG_SKIP=W1,W2,W3,W4,W5,W6,W7" "DNN_DIAG_SKIP=W7,W6,W5"
