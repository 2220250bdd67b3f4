# Kernel tests of the new GEMM ring forms + the interpreter dist tests + ring A/B microbench.
# -> gpurun_out/r3_kab/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3_kab; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "pipeline_depth" \
  > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -2 $O/kern.log
timeout -k 10 400 python bench/stage_ab.py --rounds 5 > $O/stage_ab.jsonl 2> $O/stage_ab.err || { tail -20 $O/stage_ab.err; exit 1; }
cat $O/stage_ab.jsonl
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread -k "interpreted" \
  > $O/dist.log 2>&1; rc=$?
tail -3 $O/dist.log
exit $rc
