# Overlap mode 7 (W1 first on the side) with / without the layer-0 ReLU mask: bitwise, A/B, traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
step m7_test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_overlap_gpu.py -k "overlap_plan_bitwise or cross_step"
PREFIX=r6 MODELS=head REPS=4 step m7_ab 700 bash scripts/env_ab.sh mode7 "DNN_RELU_MASK=auto" "DNN_RELU_MASK=2" "DNN_BW_OVERLAP=7" "DNN_RELU_MASK=2 DNN_BW_OVERLAP=7"
cd /tmp && export TMPDIR=/tmp
DNN_RELU_MASK=2 DNN_BW_OVERLAP=7 step trace_m7 120 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_m7 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5
