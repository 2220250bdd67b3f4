# Fresh-container sanity: smoke, default bench, and a kernel trace of the headline step
# -> gpurun_out/r3b_sanity/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3b_sanity; mkdir -p $O
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/head -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 > $O/head.log 2>&1 || exit $?
cd $R
python scripts/trace_summary.py $O/head/run_kernel_trace.csv --steps 3 > $O/head.summary.txt
cat $O/head.summary.txt
cd $R
timeout -k 10 200 python bench/probes/tail_probe.py > $O/tail_probe.jsonl 2> $O/tail_probe.err || { tail -20 $O/tail_probe.err; exit 1; }
cat $O/tail_probe.jsonl
