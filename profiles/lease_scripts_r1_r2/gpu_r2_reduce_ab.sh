# reduce_multi source-group A/B: the reduction tests, then old (A) vs new (B) build alternating on
# the headline, then a kernel trace of the new build's step.   -> gpurun_out/r2_reduce/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_reduce; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_opt_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 bash scripts/gpu_ab_so.sh r2_reduce "--steps 50 --warmup 10" 4 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c "head -12 {}"
