R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
T="python -u -m pytest -x -v -s --timeout 120 --timeout-method thread"
step persist_unit 240 $T $R/tests/test_chain_fast_gpu.py -k "persistent"
step chain_fast 600 $T $R/tests/test_chain_fast_gpu.py
step chain8_p1_q2 300 env DNN_CHAIN_PERSIST=1 python -u $R/bench/chain_latency.py --iters 400 --log $R/gpurun_out/chain8_p1_q2.srv
step chain8_p1_q1 300 env DNN_CHAIN_PERSIST=1 DNN_REHEARSAL_HW_QUEUES=1 python -u $R/bench/chain_latency.py --iters 400 --log $R/gpurun_out/chain8_p1_q1.srv
step chain8_p0_q2 300 env DNN_CHAIN_PERSIST=0 python -u $R/bench/chain_latency.py --iters 400
mkdir -p $R/gpurun_out/r5_trace
cd /tmp && export TMPDIR=/tmp
export DNN_XSTEP=1
step trace_x 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5_trace -o head \
  --output-format csv -- python3 $R/bench.py --steps 30 --warmup 10 --no-dp-compare
unset DNN_XSTEP
cd $R
step env_w0tile 700 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh w0tile "DNN_XSTEP=1" "DNN_XSTEP=1 DNN_TUNED_TABLE=$R/bench/tables/r5/w0_256x128_9.json" "DNN_XSTEP=1 DNN_TUNED_TABLE=$R/bench/tables/r5/w0_256x128_11.json" "DNN_XSTEP=1 DNN_RELU_MASK=2"
