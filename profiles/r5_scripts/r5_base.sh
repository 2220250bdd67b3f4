# Round-5 baseline on a fresh box: the driver-form bench twice, then one kernel trace over 120
# timed steps of the headline (the step "ramp" question).
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step bench_a 300 python -u $R/bench.py
step bench_b 300 python -u $R/bench.py
mkdir -p $R/gpurun_out/r5_ramp
cd /tmp && export TMPDIR=/tmp
step ramp_trace 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5_ramp -o ramp \
  --output-format csv -- python3 $R/bench.py --steps 120 --warmup 5 --no-dp-compare
