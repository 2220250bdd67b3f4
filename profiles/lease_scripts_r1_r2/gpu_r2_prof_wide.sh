# Kernel trace of the wide (784-8192-8192-10, 16384 rows) and mlp8 steps with the current tree.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_prof_wide; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/wide -o run --output-format csv -- python3 $R/bench.py --model wide --batch 16384 --steps 5 --warmup 2 > $O/wide.log 2>&1 || { tail -20 $O/wide.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mlp8 -o run --output-format csv -- python3 $R/bench.py --model mlp8 --steps 10 --warmup 3 > $O/mlp8.log 2>&1 || { tail -20 $O/mlp8.log; exit 1; }
cd $R
for n in wide mlp8; do python scripts/trace_summary.py $O/$n/run_kernel_trace.csv --steps 3 > $O/$n.summary.txt; head -32 $O/$n.summary.txt; done
