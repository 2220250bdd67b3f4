# Round-5 validation on one box: the whole GPU suite, smoke(), the driver-form bench three
# times, the default bench, mlp8 and wide, then per-dispatch PMC of the headline step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step gpu_suite 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for i in 1 2 3; do step drv_$i 300 python -u $R/bench.py --steps 20 --warmup 5; done
step bench_default 300 python -u $R/bench.py
step bench_mlp8 300 python -u $R/bench.py --model mlp8
step bench_wide 300 python -u $R/bench.py --model wide
step pmc 600 env OUT=r5_pmc_final bash $R/scripts/pmc_step.sh
step env_h0 600 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh h0 "DNN_H0_DOUBLE=0" "DNN_H0_DOUBLE=1" "DNN_H0_DOUBLE=1 DNN_XSTEP=0" "DNN_BW_OVERLAP=5" "DNN_BW_OVERLAP=5 DNN_RELU_MASK=2"
