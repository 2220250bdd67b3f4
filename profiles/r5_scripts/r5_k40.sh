R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step first_run 900 bash $R/profiles/r5_scripts/first_run.sh
