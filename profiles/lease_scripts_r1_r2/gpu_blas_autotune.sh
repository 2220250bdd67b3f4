#!/bin/bash
# hipBLASLt candidate autotuning (DNN_BLAS_AUTOTUNE=1) vs the heuristic's first choice.
set -o pipefail
O=gpurun_out/bat; mkdir -p $O; : > $O/ab.jsonl
for m in "--model wide --batch 16384 --steps 10 --warmup 3" "--model mlp8 --steps 20 --warmup 5" "--steps 100 --warmup 20"; do
  for f in 0 1 0 1; do
    DNN_BLAS_AUTOTUNE=$f timeout -k 10 150 python bench.py $m > $O/one.json 2>>$O/err.log || exit 1
    python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'autotune':'$f','model':d['config']['model'],'ms':d['ms_per_step']}))" >> $O/ab.jsonl
  done
done
