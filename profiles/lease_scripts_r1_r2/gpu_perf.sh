# One GPU-box session for a perf iteration: GPU tests, bench, rocprofv3 kernel stats of the
# bench step. Every GPU step has its own time limit; the script stops at the first failure.
# Extra bench args: BENCH_ARGS env (e.g. "--model mlp8").
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > $O/tests.log 2>&1; rc=$?; echo "rc=$rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
: > $O/bench.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 $BENCH_ARGS >> $O/bench.log 2>&1 || exit $?
export TMPDIR=/tmp
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
  -- python3 $R/bench.py --steps 20 --warmup 3 $BENCH_ARGS > $O/prof.log 2>&1 || exit $?
echo done >> $O/bench.log
