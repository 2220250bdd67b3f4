#!/bin/bash
# In-step re-tune of the mlp8 GEMMs that stayed on the MFMA kernels, then an alternating A/B.
set -o pipefail
O=gpurun_out/tunem8; mkdir -p $O
T=$O/tuned_mlp8.json
cp docker_dist_nn_amd/ops/tuned_gfx950.json $T
timeout -k 10 1000 python -u bench/tune.py --configs 65536:mlp8 --persist 0,1 --blas 1 --steps 5 --reps 2 \
  --only wgrad:1024x1024x65536,wgrad:1024x832x65536,dgrad:65536x1024x64,wgrad:64x1024x65536 \
  --out $T > $O/tune.jsonl 2>&1 || exit 1
: > $O/ab.jsonl
for t in A B A B; do
  if [ $t = B ]; then export DNN_TUNED_TABLE=$T; else unset DNN_TUNED_TABLE; fi
  timeout -k 10 150 python bench.py --model mlp8 --steps 20 --warmup 5 > $O/one.json 2>>$O/err.log || exit 1
  python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'table':'$t','ms':d['ms_per_step']}))" >> $O/ab.jsonl
done
