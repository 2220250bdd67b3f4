# Multi-rank rehearsal of the driver's N-GPU bench on ONE GPU (ranks share cuda:0, gloo
# control plane): the pipeline layouts bench.py picks for N = 2, 4, 8, over the op-by-op
# transport (gloo-staged) and the native step over xGMI-style IPC peer copies.
# Output: gpurun_out/reh/*.json
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/reh; mkdir -p $O
cd $R
run() {  # name nproc env... -- bench args
  name=$1; np=$2; shift 2
  env DNN_DIST_BACKEND=gloo DNN_FORCE_DEVICE=0 "$@" timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) \
    bench.py --gpus $np $BARGS > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }
  python -c "import json;d=json.loads([l for l in open('$O/$name.json') if l.startswith('{')][-1]);c=d['config'];print('$name', c['parallelism'], c['layer_distribution'], c['transport'], c['native_step'], d['ms_per_step'], round(d['value']/1e6,2), d['last_loss'], (d['dp_only'] or {}).get('ms_per_step'))"
}
BARGS="--steps 6 --warmup 2 --batch 16384"
run pp2_staged 2
run pp2_ipc 2 DNN_PIPE=ipc
run pp4_ipc 4 DNN_PIPE=ipc
BARGS="--steps 4 --warmup 2 --batch 8192"
run pp4dp2_ipc 8 DNN_PIPE=ipc
echo done
