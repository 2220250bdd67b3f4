R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step w0_halves 300 python -u bench/probes/w0_halves.py
