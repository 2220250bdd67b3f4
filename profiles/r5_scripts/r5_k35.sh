R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step graph_ab 600 bash $R/profiles/r5_scripts/graph_ab.sh
