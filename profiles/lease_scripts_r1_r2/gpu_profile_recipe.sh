#!/bin/bash
# Kernel trace of the reference recipe step (784-128-64-10, batch 64, Adam).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prof_recipe; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv \
  -- python3 $R/bench.py --model 784-128-64-10 --batch 64 --optimizer adam --steps 50 --warmup 10 > $O/log.txt 2>&1
