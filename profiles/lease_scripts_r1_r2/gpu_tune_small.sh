#!/bin/bash
# In-step re-tune of the 784-128-10 model's GEMMs (kernel forms x library), then A/B.
set -o pipefail
O=gpurun_out/tunesm; mkdir -p $O
T=$O/tuned_small.json
cp docker_dist_nn_amd/ops/tuned_gfx950.json $T
timeout -k 10 900 python -u bench/tune.py --configs 65536:mnist-784-128-10 --persist 0,1 --blas 1 \
  --out $T > $O/tune.jsonl 2>&1 || exit 1
: > $O/ab.jsonl
for t in A B A B; do
  if [ $t = B ]; then export DNN_TUNED_TABLE=$T; else unset DNN_TUNED_TABLE; fi
  timeout -k 10 150 python bench.py --model mnist-784-128-10 --steps 100 --warmup 20 > $O/one.json 2>>$O/err.log || exit 1
  python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'table':'$t','ms':d['ms_per_step']}))" >> $O/ab.jsonl
done
