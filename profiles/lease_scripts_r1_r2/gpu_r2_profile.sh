# Kernel-trace profiles (kernel-trace + stats only) of the three BASELINE training steps on
# one GPU with the current table: gpurun_out/r2_prof/<name>/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_prof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
p() { name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$name \
  -o run --output-format csv -- python3 $R/bench.py "$@" > $O/$name.log 2>&1 || exit $?; }
p step --steps 20 --warmup 5
p mlp8 --model mlp8 --steps 10 --warmup 3
p wide --model wide --batch 16384 --steps 5 --warmup 2
cd $R
for n in step mlp8 wide; do python scripts/trace_summary.py $O/$n/run_kernel_trace.csv --steps 3 > $O/$n.summary.txt; done
echo done
