#!/bin/bash
# Alternating A/B of the dgrad/wgrad two-stream plan (DNN_BW_OVERLAP) on the headline step.
set -o pipefail
mkdir -p gpurun_out/ovab
: > gpurun_out/ovab/ab.jsonl
for f in 0 1 0 1 0 1; do
  DNN_BW_OVERLAP=$f timeout -k 10 150 python bench.py --steps 100 --warmup 20 > gpurun_out/ovab/one.json 2>>gpurun_out/ovab/err.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ovab/one.json'));print(json.dumps({'overlap':'$f','ms':d['ms_per_step']}))" >> gpurun_out/ovab/ab.jsonl
done
