#!/bin/bash
# Kernel trace of the headline step with the fused tail on.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tailprof
DNN_TAIL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/tailprof -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/tailprof/log.txt 2>&1
