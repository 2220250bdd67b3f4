# GPU tests, in-situ GEMM tuning (starting from the committed table), bench, step kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > $O/tests.log 2>&1; rc=$?; echo "rc=$rc" >> $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_before.log 2>&1 || exit $?
timeout -k 10 1000 python bench/tune.py ${TUNE_ARGS} > $O/tune.log 2>&1 || exit $?
cp docker_dist_nn_amd/ops/tuned_gfx950.json $O/tuned_gfx950.json
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_tuned.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --batch 131072 >> $O/bench_tuned.log 2>&1 || exit $?
export TMPDIR=/tmp
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
  -- python3 $R/bench.py --steps 20 --warmup 3 > $O/prof.log 2>&1 || exit $?
echo done >> $O/tests.log
