# Kernel trace of the mlp8 step -> gpurun_out/r3b_trace_m8/mlp8.summary.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3b_trace_m8; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mlp8 -o run --output-format csv -- python3 $R/bench.py --model mlp8 --steps 10 --warmup 3 > $O/mlp8.log 2>&1 || exit $?
cd $R
python scripts/trace_summary.py $O/mlp8/run_kernel_trace.csv --steps 3 > $O/mlp8.summary.txt
cat $O/mlp8.summary.txt
