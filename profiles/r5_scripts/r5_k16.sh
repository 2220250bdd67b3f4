R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
mkdir -p $R/gpurun_out/r5_trace
cd /tmp && export TMPDIR=/tmp
step trace_wide 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5_trace -o wide \
  --output-format csv -- python3 $R/bench.py --model wide --batch 16384 --steps 10 --warmup 3 --no-dp-compare
step trace_mlp8 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5_trace -o mlp8 \
  --output-format csv -- python3 $R/bench.py --model mlp8 --steps 10 --warmup 3 --no-dp-compare
