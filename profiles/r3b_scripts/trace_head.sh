# Kernel trace of the headline step -> gpurun_out/${OUT:-r3b_trace}/head.summary.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r3b_trace}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/head -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 > $O/head.log 2>&1 || exit $?
cd $R
python scripts/trace_summary.py $O/head/run_kernel_trace.csv --steps 3 > $O/head.summary.txt
cat $O/head.summary.txt
