#!/bin/bash
# In-step re-tune of the 131072-row headline GEMMs left after the fused tail, then A/B.
set -o pipefail
O=gpurun_out/tune131; mkdir -p $O
T=$O/tuned_131k.json
cp docker_dist_nn_amd/ops/tuned_gfx950.json $T
timeout -k 10 1000 python -u bench/tune.py --configs 131072:mnist-fcnn --persist 0,1 --blas 1 \
  --only fwd:131072x512x832,fwd:131072x256x512,dgrad:131072x512x256,wgrad:512x832x131072,wgrad:256x512x131072,wgrad:128x256x131072,wgrad:64x128x131072 \
  --out $T > $O/tune.jsonl 2>&1 || exit 1
: > $O/ab.jsonl
for t in A B A B; do
  if [ $t = B ]; then export DNN_TUNED_TABLE=$T; else unset DNN_TUNED_TABLE; fi
  timeout -k 10 150 python bench.py --batch 131072 --steps 50 --warmup 10 > $O/one.json 2>>$O/err.log || exit 1
  python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'table':'$t','ms':d['ms_per_step']}))" >> $O/ab.jsonl
done
