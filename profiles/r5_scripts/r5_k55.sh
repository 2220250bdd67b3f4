R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step setprio_1 600 bash $R/scripts/setprio_ab.sh 1
step setprio_2 400 bash $R/scripts/setprio_ab.sh 2
