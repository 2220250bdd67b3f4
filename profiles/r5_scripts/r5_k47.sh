R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_w0w1 900 env PREFIX=r5 MODELS=head REPS=5 bash $R/scripts/env_ab.sh w0w1 "DNN_BW_OVERLAP=1" "DNN_W0_AFTER_W1=1"
