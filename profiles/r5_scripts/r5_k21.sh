# Round-5 validation with every round-5 default on (XSTEP, H0_DOUBLE, RELU_MASK=auto,
# EVENT_FENCE=device, CHAIN_PERSIST, CHAIN_DOORBELL).
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step gpu_suite 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for i in 1 2 3; do step drv_$i 300 python -u $R/bench.py --steps 20 --warmup 5; done
step bench_default 300 python -u $R/bench.py
step bench_mlp8 300 python -u $R/bench.py --model mlp8
step bench_wide 300 python -u $R/bench.py --model wide --batch 16384
step chain8_a 240 python -u $R/bench/chain_latency.py --iters 400
step chain8_b 240 python -u $R/bench/chain_latency.py --iters 400
