# After removing the fused forward+tail launch: tail / engine / stage GPU tests, smoke, and
# three driver-form benches.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
step tail_engine 500 python -u -m pytest tests/test_mlp_tail_gpu.py tests/test_engine_gpu.py -m gpu -v --timeout 300 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do step bench_p$i 200 python -u bench.py --steps 20 --warmup 5; done
