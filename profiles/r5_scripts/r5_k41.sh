R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step ramp_idle 300 python -u bench/probes/ramp_idle.py
