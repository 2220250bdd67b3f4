#!/bin/bash
# Full in-step re-tune of the headline GEMMs the fused tail leaves (tiles x splits x forms x
# library), then an alternating A/B of the new table against the in-tree one.
set -o pipefail
O=gpurun_out/tunehl; mkdir -p $O
T=$O/tuned_headline.json
cp docker_dist_nn_amd/ops/tuned_gfx950.json $T
timeout -k 10 1000 python -u bench/tune.py --configs 65536:mnist-fcnn --persist 0,1 --blas 1 \
  --only fwd:65536x512x832,fwd:65536x256x512,dgrad:65536x512x256,wgrad:512x832x65536,wgrad:256x512x65536,wgrad:128x256x65536,wgrad:64x128x65536 \
  --out $T > $O/tune.jsonl 2>&1 || exit 1
: > $O/ab.jsonl
for t in A B A B A B; do
  if [ $t = B ]; then export DNN_TUNED_TABLE=$T; else unset DNN_TUNED_TABLE; fi
  timeout -k 10 150 python bench.py --steps 100 --warmup 20 > $O/one.json 2>>$O/err.log || exit 1
  python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'table':'$t','ms':d['ms_per_step']}))" >> $O/ab.jsonl
done
