R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step rp4_ab 300 python -u bench/probes/rp4_ab.py --reps 3 --iters 20
