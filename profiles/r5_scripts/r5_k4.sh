R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step persist_unit 240 $T $R/tests/test_chain_fast_gpu.py -k "persistent or one_process"
step chain_fast 600 $T $R/tests/test_chain_fast_gpu.py
for i in 1 2; do
  step chain8_p1_$i 300 env DNN_CHAIN_PERSIST=1 python -u $R/bench/chain_latency.py --iters 400
  step chain8_p0_$i 300 env DNN_CHAIN_PERSIST=0 python -u $R/bench/chain_latency.py --iters 400
done
step env_w0tile 700 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh w0tile "DNN_XSTEP=1" "DNN_XSTEP=1 DNN_TUNED_TABLE=$R/bench/tables/r5/w0_256x128_9.json" "DNN_XSTEP=1 DNN_TUNED_TABLE=$R/bench/tables/r5/w0_256x128_11.json" "DNN_XSTEP=1 DNN_RELU_MASK=2"
