#!/bin/bash
# Per-GEMM comparison of the headline / mlp8 / wide steps against hipBLASLt and the HBM floor.
set -o pipefail
mkdir -p gpurun_out/blas
timeout -k 10 240 python -u bench/gemm_vs_blas.py > gpurun_out/blas/headline.jsonl 2>&1 &&
timeout -k 10 240 python -u bench/gemm_vs_blas.py --model 784-1024-1024-1024-1024-1024-1024-1024-10 \
  > gpurun_out/blas/mlp8.jsonl 2>&1 &&
timeout -k 10 300 python -u bench/gemm_vs_blas.py --model 784-8192-8192-10 --rows 16384 \
  > gpurun_out/blas/wide.jsonl 2>&1
