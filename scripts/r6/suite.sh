# Whole GPU suite + smoke + driver-form bench (round 6 checkpoint).
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
step gpu_suite 1000 python -u -m pytest tests -m gpu -v --timeout 420 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_d1 200 python -u bench.py --steps 20 --warmup 5
step bench_d2 200 python -u bench.py --steps 20 --warmup 5
