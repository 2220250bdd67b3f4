R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
T="python -u -m pytest -x -v -s --timeout 120 --timeout-method thread"
step persist_unit 240 $T $R/tests/test_chain_fast_gpu.py -k "persistent"
step chain_fast 600 $T $R/tests/test_chain_fast_gpu.py
step chain8_p1_a 240 env DNN_CHAIN_PERSIST=1 python -u $R/bench/chain_latency.py --iters 400 --log $R/gpurun_out/chain8_p1_a.srv
step chain8_p0_a 240 env DNN_CHAIN_PERSIST=0 python -u $R/bench/chain_latency.py --iters 400
step chain8_p1_b 240 env DNN_CHAIN_PERSIST=1 python -u $R/bench/chain_latency.py --iters 400
step chain8_p0_b 240 env DNN_CHAIN_PERSIST=0 python -u $R/bench/chain_latency.py --iters 400
step chain8_p1_c 240 env DNN_CHAIN_PERSIST=1 python -u $R/bench/chain_latency.py --iters 400
step ladder_gpu 600 $T $R/tests/test_bench_ladder_gpu.py
