# Native-step construction fault -> agreed fallback: the dist GPU tests, then bench.py as the
# driver runs it (2 ranks on one GPU, gloo control plane, IPC hops) with and without the fault.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_fallback; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 180 \
  --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
run() { name=$1; shift
  env DNN_DIST_BACKEND=gloo DNN_FORCE_DEVICE=0 DNN_PIPE=ipc GPU_MAX_HW_QUEUES=8 "$@" timeout -k 10 240 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29600 + RANDOM % 300)) bench.py --gpus 2 --steps 5 --warmup 2 --batch 8192 \
    > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }
  python -c "import json;d=json.loads([l for l in open('$O/$name.json') if l.startswith('{')][-1]);c=d['config'];print('$name', c['parallelism'], c['transport'], c['native_step'], d['native_fallback'], d['last_loss'], d['dp_only'] and d['dp_only']['parallelism'])"
}
run ok
run fault DNN_FAULT_NATIVE_STEP=1
