# Fork elision: overlap tests, headline A/B, kernel trace.  -> gpurun_out/r2_fork/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_fork; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_overlap_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 bash scripts/gpu_sw_ab.sh r2_fork "--steps 50 --warmup 10" 4 DNN_FORK_ELIDE=0 DNN_FORK_ELIDE=1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R && python scripts/trace_summary.py $O/prof/run_kernel_trace.csv --steps 3 > $O/summary.txt; head -14 $O/summary.txt
