#!/bin/bash
# Alternating bench A/B of two tuned tables: $1 = table B (A = the in-tree table), $2.. = bench args
set -o pipefail
mkdir -p gpurun_out/tableab
B=$1; shift
for t in A B A B A B; do
  if [ $t = B ]; then export DNN_TUNED_TABLE=$B; else unset DNN_TUNED_TABLE; fi
  timeout -k 10 150 python bench.py "$@" > gpurun_out/tableab/one.json 2>>gpurun_out/tableab/err.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/tableab/one.json'));print(json.dumps({'table':'$t','model':d['config']['model'],'ms':d['ms_per_step']}))" >> gpurun_out/tableab/ab.jsonl
done
