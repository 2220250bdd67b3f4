# Multi-process (processes sharing cuda:0) distributed GPU tests: native IPC step, the gloo
# interpreter of the RCCL plans, DP, TP. -> gpurun_out/r3_dist/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3_dist; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1; rc=$?
tail -40 $O/pytest.log
exit $rc
