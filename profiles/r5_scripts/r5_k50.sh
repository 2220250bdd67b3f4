R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
for i in 1 2 3; do step sanity_$i 300 python -u $R/bench.py --no-dp-compare; done
