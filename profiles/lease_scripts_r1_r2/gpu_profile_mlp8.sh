#!/bin/bash
# Kernel trace of the mlp8 step (kernel-trace + stats only).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prof_mlp8; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv \
  -- python3 $R/bench.py --model mlp8 --steps 5 --warmup 2 > $O/log.txt 2>&1
