R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_finow0b 600 env PREFIX=r5 MODELS=head REPS=4 bash $R/scripts/env_ab.sh finow0b "DNN_BW_OVERLAP=1" "DNN_FINO_AFTER_W0=1"
