#!/bin/bash
# In-step hipBLASLt algorithm choice per library GEMM, then alternating table A/B per model.
set -o pipefail
O=gpurun_out/tba; mkdir -p $O
T=$O/tuned_algo.json
cp docker_dist_nn_amd/ops/tuned_gfx950.json $T
timeout -k 10 900 python -u bench/tune_blas_algo.py --configs 65536:mnist-fcnn,65536:mlp8,16384:wide --out $T > $O/tune.jsonl 2>&1 || exit 1
: > $O/ab.jsonl
for m in "--steps 100 --warmup 20" "--model mlp8 --steps 20 --warmup 5" "--model wide --batch 16384 --steps 10 --warmup 3"; do
  for t in A B A B; do
    if [ $t = B ]; then export DNN_TUNED_TABLE=$T; else unset DNN_TUNED_TABLE; fi
    timeout -k 10 150 python bench.py $m > $O/one.json 2>>$O/err.log || exit 1
    python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'table':'$t','model':d['config']['model'],'ms':d['ms_per_step']}))" >> $O/ab.jsonl
  done
done
