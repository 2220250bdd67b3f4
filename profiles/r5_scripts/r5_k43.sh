R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step infer_tp 400 python -u bench/infer_throughput.py
