R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_mask0 900 env PREFIX=r5 MODELS=head REPS=4 bash $R/scripts/env_ab.sh mask0 "DNN_BW_OVERLAP=1" "DNN_RELU_MASK=2"
