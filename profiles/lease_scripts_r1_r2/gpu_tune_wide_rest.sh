#!/bin/bash
# In-step re-tune of the wide model's GEMMs that stay on our kernels, then alternating A/B.
set -o pipefail
O=gpurun_out/tunewr; mkdir -p $O
T=$O/tuned_wide_rest.json
cp docker_dist_nn_amd/ops/tuned_gfx950.json $T
timeout -k 10 1000 python -u bench/tune.py --configs 16384:wide --persist 0,1 --blas 1 --steps 5 --reps 3 \
  --only dgrad:16384x8192x64,wgrad:8192x832x16384,wgrad:64x8192x16384 --out $T > $O/tune.jsonl 2>&1 || exit 1
: > $O/ab.jsonl
for t in A B A B; do
  if [ $t = B ]; then export DNN_TUNED_TABLE=$T; else unset DNN_TUNED_TABLE; fi
  timeout -k 10 150 python bench.py --model wide --batch 16384 --steps 10 --warmup 3 > $O/one.json 2>>$O/err.log || exit 1
  python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'table':'$t','ms':d['ms_per_step']}))" >> $O/ab.jsonl
done
