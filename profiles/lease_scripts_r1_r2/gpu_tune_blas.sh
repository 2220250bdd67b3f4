#!/bin/bash
# Per-GEMM choice between the hand-written kernels and the hipBLASLt library GEMM: re-tune the
# mlp8 / wide / headline step GEMMs (incumbent vs library) and bench before / after.
set -o pipefail
mkdir -p gpurun_out/tuneblas
O=gpurun_out/tuneblas
T=$O/tuned_blas.json
cp docker_dist_nn_amd/ops/tuned_gfx950.json $T
: > $O/before.jsonl; : > $O/after.jsonl
for m in "mlp8 65536" "wide 16384" "mnist-fcnn 65536"; do
  set -- $m
  timeout -k 10 150 python bench.py --model $1 --batch $2 --steps 30 --warmup 5 >> $O/before.jsonl 2>>$O/err.log || exit 1
done
timeout -k 10 900 python -u bench/tune.py --configs 65536:mnist-fcnn,65536:mlp8,16384:wide --persist 0 --blas only --verbose --out $T > $O/tune.jsonl 2>&1 || exit 1
cp $T docker_dist_nn_amd/ops/tuned_gfx950.json
for m in "mlp8 65536" "wide 16384" "mnist-fcnn 65536"; do
  set -- $m
  timeout -k 10 150 python bench.py --model $1 --batch $2 --steps 30 --warmup 5 >> $O/after.jsonl 2>>$O/err.log || exit 1
done
