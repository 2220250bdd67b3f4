# One-GPU rehearsal of the verified IPC transport in bench.py: 4 ranks sharing cuda:0 (gloo
# collectives), DNN_PIPE=ipc with the first-step verification forced on; once clean, once with
# one rank's IPC result corrupted (the fallback branch). -> gpurun_out/r3_ipcr/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r3_ipcr}; mkdir -p $O
cd $R
run() { name=$1; shift
  env DNN_DIST_BACKEND=gloo DNN_FORCE_DEVICE=0 DNN_PIPE=ipc DNN_IPC_VERIFY=1 GPU_MAX_HW_QUEUES=12 "$@" timeout -k 10 300 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $((29600 + RANDOM % 300)) bench.py --gpus 4 --steps 5 --warmup 2 --batch 8192 --no-dp-compare \
    > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }
  python -c "import json;d=json.loads([l for l in open('$O/$name.json') if l.startswith('{')][-1]);c=d['config'];print('$name', c['parallelism'], c['transport'], '|', c['transport_reason'], '|', c['native_step'], d['last_loss'], d['ms_per_step'], d['host_ms_per_step'], d['graph_trial'])"
}
run verified
run fallback DNN_FAULT_IPC_VERIFY=2
run rccl_ref DNN_PIPE=rccl
