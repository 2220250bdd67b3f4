R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step diag_wg1 60 python -u $R/bench/probes/chain_stage_diag.py --wg 1
step diag_wg4 60 python -u $R/bench/probes/chain_stage_diag.py --wg 4
step diag_wg64 60 python -u $R/bench/probes/chain_stage_diag.py --wg 64
step diag_wg8_k256 60 python -u $R/bench/probes/chain_stage_diag.py --wg 8 --K 256 --N 128
mkdir -p $R/gpurun_out/r5_trace
cd /tmp && export TMPDIR=/tmp
export DNN_XSTEP=1
step trace_x 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5_trace -o head \
  --output-format csv -- python3 $R/bench.py --steps 30 --warmup 10 --no-dp-compare
unset DNN_XSTEP
cd $R
step env_w0tile 700 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh w0tile "DNN_XSTEP=1" "DNN_XSTEP=1 DNN_TUNED_TABLE=$R/bench/tables/r5/w0_256x128_9.json" "DNN_XSTEP=1 DNN_TUNED_TABLE=$R/bench/tables/r5/w0_256x128_11.json" "DNN_XSTEP=1 DNN_RELU_MASK=2"
