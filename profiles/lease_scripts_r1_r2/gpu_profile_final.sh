# Kernel-trace profiles of the current headline step (1 GPU) and of the data-parallel step path
# (deferred update, no-op comm) for profiles/. kernel-trace + stats only.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prof_final; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/step -o run --output-format csv \
  -- python3 $R/bench.py --steps 20 --warmup 5 > $O/step.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/wide -o run --output-format csv \
  -- python3 $R/bench.py --model wide --batch 16384 --steps 5 --warmup 2 > $O/wide.log 2>&1 || exit $?
echo done > $O/status.txt
