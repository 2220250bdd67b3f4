R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
T="python -u -m pytest -x -v -s --timeout 120 --timeout-method thread"
step persist_unit 240 $T $R/tests/test_chain_fast_gpu.py -k "persistent"
step chain_fast 600 $T $R/tests/test_chain_fast_gpu.py
step chain8_db1_a 240 env DNN_CHAIN_DOORBELL=1 python -u $R/bench/chain_latency.py --iters 400 --log $R/gpurun_out/chain8_db1_a.srv
step chain8_db0_a 240 env DNN_CHAIN_DOORBELL=0 python -u $R/bench/chain_latency.py --iters 400
step chain8_db1_b 240 env DNN_CHAIN_DOORBELL=1 python -u $R/bench/chain_latency.py --iters 400
step chain8_db0_b 240 env DNN_CHAIN_DOORBELL=0 python -u $R/bench/chain_latency.py --iters 400
step chain8_db1_c 240 env DNN_CHAIN_DOORBELL=1 python -u $R/bench/chain_latency.py --iters 400
