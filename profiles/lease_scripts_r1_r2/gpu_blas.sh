#!/bin/bash
# hipBLASLt library-GEMM path: GPU tests, then every BASELINE model with DNN_BLAS=0 / 1.
set -o pipefail
mkdir -p gpurun_out/blasab
timeout -k 10 300 python -u -m pytest tests/test_blas_gpu.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/blasab/test.log 2>&1 || exit 1
: > gpurun_out/blasab/ab.jsonl
for m in "--model wide --batch 16384 --steps 10 --warmup 3" "--model mlp8 --steps 20 --warmup 5" "--steps 50 --warmup 10"; do
  for f in 0 1 0 1; do
    DNN_BLAS=$f timeout -k 10 200 python -u bench.py $m > gpurun_out/blasab/one.json 2>>gpurun_out/blasab/err.log || exit 1
    python -c "import json,sys;d=json.load(open('gpurun_out/blasab/one.json'));print(json.dumps({'blas':'$f','model':d['config']['model'],'ms':d['ms_per_step']}))" >> gpurun_out/blasab/ab.jsonl
  done
done
