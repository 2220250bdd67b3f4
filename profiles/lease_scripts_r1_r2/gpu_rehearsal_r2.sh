# Multi-rank rehearsal of bench.py on ONE GPU (ranks share cuda:0, gloo control plane, IPC
# hops): native step eager vs HIP graph, relayed hops, and the sharded-DP layout over gloo.
# Output: gpurun_out/reh2/*.json
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/reh2; mkdir -p $O
cd $R
run() {  # name nproc env... (bench args in BARGS)
  name=$1; np=$2; shift 2
  env DNN_DIST_BACKEND=gloo DNN_FORCE_DEVICE=0 "$@" timeout -k 10 240 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) \
    bench.py --gpus $np --no-dp-compare $BARGS > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }
  python -c "import json;d=json.loads([l for l in open('$O/$name.json') if l.startswith('{')][-1]);c=d['config'];print('$name', c['parallelism'], c['layer_distribution'], c['transport'], c['native_step'], c['hip_graph'], c.get('dp_reduce'), d['ms_per_step'], round(d['value']/1e6,2), d['last_loss'])"
}
BARGS="--steps 10 --warmup 3 --batch 16384"
run pp2_ipc 2 DNN_PIPE=ipc
BARGS="--steps 10 --warmup 3 --batch 16384 --graph"
run pp2_ipc_graph 2 DNN_PIPE=ipc
BARGS="--steps 10 --warmup 3 --batch 16384"
run pp4_ipc 4 DNN_PIPE=ipc
run pp4_ipc_relay2 4 DNN_PIPE=ipc DNN_IPC_RELAYS=2 GPU_MAX_HW_QUEUES=8
BARGS="--steps 10 --warmup 3 --batch 16384 --graph"
run pp4_ipc_graph 4 DNN_PIPE=ipc
BARGS="--steps 4 --warmup 2 --batch 8192"
run pp4dp2_ipc_shard 8 DNN_PIPE=ipc
echo done
