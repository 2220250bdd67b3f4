#!/bin/bash
# Full in-step re-tune of every mlp8 GEMM (tiles x splits x forms x library), then A/B.
set -o pipefail
O=gpurun_out/tunem8f; mkdir -p $O
T=$O/tuned_mlp8_full.json
cp docker_dist_nn_amd/ops/tuned_gfx950.json $T
timeout -k 10 1050 python -u bench/tune.py --configs 65536:mlp8 --persist 0,1 --blas 1 --steps 4 --reps 2 \
  --only fwd:65536x1024x832,fwd:65536x1024x1024,dgrad:65536x1024x1024 \
  --out $T > $O/tune.jsonl 2>&1 || exit 1
: > $O/ab.jsonl
for t in A B A B; do
  if [ $t = B ]; then export DNN_TUNED_TABLE=$T; else unset DNN_TUNED_TABLE; fi
  timeout -k 10 150 python bench.py --model mlp8 --steps 20 --warmup 5 > $O/one.json 2>>$O/err.log || exit 1
  python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'table':'$t','ms':d['ms_per_step']}))" >> $O/ab.jsonl
done
