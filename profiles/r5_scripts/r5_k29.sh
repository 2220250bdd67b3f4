R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_modes 900 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh modes "DNN_BW_OVERLAP=1" "DNN_BW_OVERLAP=2" "DNN_BW_OVERLAP=3" "DNN_BW_OVERLAP=5" "DNN_FORK_ELIDE=1" "DNN_FORK_ELIDE=2" "DNN_BW_OVERLAP=6"
