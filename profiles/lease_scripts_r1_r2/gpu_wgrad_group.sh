#!/bin/bash
# Grouped wgrad launch: GPU tests, then headline / recipe / mlp8 with DNN_WGRAD_GROUP=0/1.
set -o pipefail
O=gpurun_out/wgg; mkdir -p $O; : > $O/ab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_wgrad_group_gpu.py tests/test_fused_opt_gpu.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || exit 1
for m in "--steps 100 --warmup 20" "--model 784-128-64-10 --batch 64 --optimizer adam --steps 500 --warmup 50" "--model mlp8 --steps 20 --warmup 5"; do
  for f in 0 1 0 1; do
    DNN_WGRAD_GROUP=$f timeout -k 10 150 python bench.py $m > $O/one.json 2>>$O/err.log || exit 1
    python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'group':'$f','model':d['config']['model'],'ms':d['ms_per_step']}))" >> $O/ab.jsonl
  done
done
