# Final validation of the round-5 build: the whole GPU suite, smoke(), the driver-form bench
# three times, the default bench, mlp8, wide, per-dispatch PMC and a kernel trace of the step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step gpu_suite 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for i in 1 2 3; do step drv_$i 300 python -u $R/bench.py --steps 20 --warmup 5; done
step bench_default 300 python -u $R/bench.py
step bench_mlp8 300 python -u $R/bench.py --model mlp8
step bench_wide 300 python -u $R/bench.py --model wide --batch 16384
step pmc 600 env OUT=r5_pmc_last bash $R/scripts/pmc_step.sh
mkdir -p $R/gpurun_out/r5_trace_last
cd /tmp && export TMPDIR=/tmp
step trace 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5_trace_last -o head \
  --output-format csv -- python3 $R/bench.py --steps 30 --warmup 10 --no-dp-compare
