R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step gpu_suite 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step drv_1 300 python -u $R/bench.py --steps 20 --warmup 5
step bench_default 300 python -u $R/bench.py
