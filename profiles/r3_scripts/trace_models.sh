# Kernel traces of the mlp8 and wide steps (bench.py) -> gpurun_out/r3_trace/<model>.summary.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3_trace; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mlp8 -o run --output-format csv -- python3 $R/bench.py --model mlp8 --steps 10 --warmup 3 > $O/mlp8.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/wide -o run --output-format csv -- python3 $R/bench.py --model wide --batch 16384 --steps 6 --warmup 2 > $O/wide.log 2>&1 || exit $?
cd $R
python scripts/trace_summary.py $O/mlp8/run_kernel_trace.csv --steps 3 > $O/mlp8.summary.txt
python scripts/trace_summary.py $O/wide/run_kernel_trace.csv --steps 2 > $O/wide.summary.txt
cat $O/mlp8.summary.txt $O/wide.summary.txt
