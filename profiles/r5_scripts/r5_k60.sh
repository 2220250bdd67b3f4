R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_m8elide 900 env PREFIX=r5 MODELS=mlp8,wide REPS=4 bash $R/scripts/env_ab.sh m8elide "DNN_BW_OVERLAP=1" "DNN_FORK_ELIDE=1"
