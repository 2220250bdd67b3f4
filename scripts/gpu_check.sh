# One GPU-box session: tests, smoke, bench variants (A/B), latency, rocprofv3 kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests/ -q -m gpu > $O/tests.log 2>&1; rc=$?; echo "rc=$rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
: > $O/bench_sweep.log
for args in "" "--batch 32768" "--batch 131072" "--graph"; do
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 $args >> $O/bench_sweep.log 2>&1 || exit $?
done
DNN_FUSED_XENT=0 timeout -k 10 180 python bench.py --steps 30 --warmup 5 >> $O/bench_sweep.log 2>&1 || exit $?
DNN_WGRAD_ALGO=streamk timeout -k 10 180 python bench.py --steps 30 --warmup 5 >> $O/bench_sweep.log 2>&1 || exit $?
timeout -k 10 300 python bench/latency.py --iters 300 > $O/latency.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/bench.py --steps 20 --warmup 3 > $O/prof.log 2>&1 || exit $?
echo done >> $O/tests.log
