#!/bin/bash
# 2 ranks sharing the one GPU (gloo), full per-rank headline batch: the exact per-rank path the
# driver's multi-GPU bench runs (tail, library GEMMs, persistent dgrad, deferred DP update).
set -o pipefail
mkdir -p gpurun_out/reh
DNN_DIST_BACKEND=gloo DNN_FORCE_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29563 \
  bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/reh/dp2.log 2>&1
