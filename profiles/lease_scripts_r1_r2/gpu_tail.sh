#!/bin/bash
# Fused classifier tail: GPU tests, isolated A/B, then the headline step with and without it.
set -o pipefail
mkdir -p gpurun_out/tail
timeout -k 10 400 python -u -m pytest tests/test_mlp_tail_gpu.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/tail/test.log 2>&1 &&
timeout -k 10 120 python -u bench/tail_ab.py > gpurun_out/tail/ab.jsonl 2>&1 &&
DNN_TAIL=1 timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 > gpurun_out/tail/b1a.json 2>gpurun_out/tail/b1a.err &&
DNN_TAIL=0 timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 > gpurun_out/tail/b0a.json 2>gpurun_out/tail/b0a.err &&
DNN_TAIL=1 timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 > gpurun_out/tail/b1b.json 2>gpurun_out/tail/b1b.err &&
DNN_TAIL=0 timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 > gpurun_out/tail/b0b.json 2>gpurun_out/tail/b0b.err
