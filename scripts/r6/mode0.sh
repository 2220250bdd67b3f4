# The single-stream plan (no side stream, no events) with / without the layer-0 mask: A/B + traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
step mask_test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_overlap_gpu.py -k "mask"
PREFIX=r6 MODELS=head REPS=3 step m0_ab 600 bash scripts/env_ab.sh mode0 "DNN_RELU_MASK=auto" "DNN_BW_OVERLAP=0" "DNN_BW_OVERLAP=0 DNN_RELU_MASK=2"
cd /tmp && export TMPDIR=/tmp
DNN_BW_OVERLAP=0 step trace_m0 120 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_m0 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5
DNN_BW_OVERLAP=0 DNN_RELU_MASK=2 step trace_m0m 120 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_m0m -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5
