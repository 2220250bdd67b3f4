# per-layer fused reduce+update (DNN_SPLIT_FINO=2): bitwise test, then step A/B on mlp8 / head
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r3b_fino2
timeout -k 10 300 python -u -m pytest tests/test_overlap_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b_fino2/pytest.log 2>&1 || { tail -30 gpurun_out/r3b_fino2/pytest.log; exit 1; }
tail -1 gpurun_out/r3b_fino2/pytest.log
MODELS=mlp8,head bash scripts/r3b/env_ab.sh fino2 DNN_SPLIT_FINO=0 DNN_SPLIT_FINO=2 DNN_SPLIT_FINO=1 || exit 1
