#!/bin/bash
# Fused linear+CE tile vs library logits GEMM + softmax-CE kernel, per model (in-step), then A/B.
set -o pipefail
O=gpurun_out/tunelg; mkdir -p $O
T=$O/tuned_logits.json
cp docker_dist_nn_amd/ops/tuned_gfx950.json $T
timeout -k 10 600 python -u bench/tune.py --configs 16384:wide,65536:mlp8 --blas 1 \
  --only fwd:16384x64x8192,fwd:65536x64x1024 --out $T > $O/tune.jsonl 2>&1 || exit 1
: > $O/ab.jsonl
for m in "--model wide --batch 16384 --steps 10 --warmup 3" "--model mlp8 --steps 20 --warmup 5"; do
  for t in A B A B; do
    if [ $t = B ]; then export DNN_TUNED_TABLE=$T; else unset DNN_TUNED_TABLE; fi
    timeout -k 10 150 python bench.py $m > $O/one.json 2>>$O/err.log || exit 1
    python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'table':'$t','model':d['config']['model'],'ms':d['ms_per_step']}))" >> $O/ab.jsonl
  done
done
