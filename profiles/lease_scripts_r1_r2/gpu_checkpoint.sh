# Checkpoint run: GPU tests, smoke, every-config bench vs torch-ROCm, a 2-rank (gloo, one GPU)
# rehearsal of the multi-rank bench path. Outputs under gpurun_out/.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/ck_pytest.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/ck_smoke.log 2>&1 || exit $?
DNN_DIST_BACKEND=gloo DNN_FORCE_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 \
  bench.py --gpus 2 --steps 5 --warmup 2 --batch 8192 > $O/ck_rehearsal.log 2>&1 || exit $?
bash scripts/gpu_configs.sh
