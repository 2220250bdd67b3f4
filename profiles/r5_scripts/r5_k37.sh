R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step dgrad_epi 300 python -u bench/probes/dgrad_epi.py
