R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_m8modes 900 env PREFIX=r5 MODELS=mlp8 REPS=3 bash $R/scripts/env_ab.sh m8modes "DNN_BW_OVERLAP=1" "DNN_BW_OVERLAP=2" "DNN_BW_OVERLAP=4" "DNN_BW_OVERLAP=5" "DNN_BW_OVERLAP=1 DNN_FORK_ELIDE=1"
