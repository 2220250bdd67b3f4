# Round-6 baseline on a fresh box: the driver-form bench three times, then a kernel trace of
# 30 timed steps of the headline.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step bench_a 200 python -u $R/bench.py --steps 20 --warmup 5
step bench_b 200 python -u $R/bench.py --steps 20 --warmup 5
step bench_c 200 python -u $R/bench.py --steps 50 --warmup 10
mkdir -p $R/gpurun_out/r6_base
cd /tmp && export TMPDIR=/tmp
step trace 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6_base -o tr \
  --output-format csv -- python3 $R/bench.py --steps 30 --warmup 5 --no-dp-compare
