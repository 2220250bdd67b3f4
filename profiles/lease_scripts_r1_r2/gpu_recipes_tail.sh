#!/bin/bash
# Reference recipes (batch 64, Adam) and batch 4096: the fused tail on vs off, alternating.
set -o pipefail
O=gpurun_out/recipes; mkdir -p $O; : > $O/ab.jsonl
for m in "--model 784-128-64-10 --batch 64 --optimizer adam --steps 500 --warmup 50" \
         "--model 784-32-16-10 --batch 64 --optimizer adam --steps 500 --warmup 50" \
         "--batch 4096 --steps 300 --warmup 30"; do
  for f in 0 1 0 1; do
    DNN_TAIL=$f timeout -k 10 150 python bench.py $m > $O/one.json 2>>$O/err.log || exit 1
    python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'tail':'$f','model':d['config']['model'],'batch':d['config']['global_batch'],'ms':d['ms_per_step'],'value':d['value']}))" >> $O/ab.jsonl
  done
done
