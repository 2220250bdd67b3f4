# Reduction kernels: every source-group class.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_opt_gpu.py -m gpu -x -q -k "reduce" --timeout 120 --timeout-method thread > gpurun_out/reduce_tests.log 2>&1; rc=$?; tail -3 gpurun_out/reduce_tests.log; exit $rc
