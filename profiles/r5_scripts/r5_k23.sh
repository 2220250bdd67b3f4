R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
T="python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider"
step ladder 600 $T $R/tests/test_bench_ladder_gpu.py
for i in 1 2 3; do
  step chain_nat_$i 240 env DNN_CHAIN_DOORBELL=0 DNN_CHAIN_NATIVE=1 python -u $R/bench/chain_latency.py --iters 400
  step chain_py_$i 240 env DNN_CHAIN_DOORBELL=0 DNN_CHAIN_NATIVE=0 python -u $R/bench/chain_latency.py --iters 400
done
TB=$R/bench/tables/r5
step env_widepp 700 env PREFIX=r5 MODELS=wide REPS=3 bash $R/scripts/env_ab.sh widepp "DNN_XSTEP=1" "DNN_TUNED_TABLE=$TB/wide_fwd_pp.json" "DNN_TUNED_TABLE=$TB/wide_dgrad_pp.json"
