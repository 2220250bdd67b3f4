# One-stream plan with every wgrad in one mixed launch (DNN_BWD_GROUP=2): bitwise test, A/B, trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
step bg2_test 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_overlap_gpu.py -k "mixed"
grep -q "2 passed" gpurun_out/bg2_test.log || exit 1
PREFIX=r6 MODELS=head REPS=4 step bg2_ab 600 bash scripts/env_ab.sh bwdgroup2 "DNN_BWD_GROUP=0" "DNN_BWD_GROUP=2" "DNN_BWD_GROUP=2 DNN_RELU_MASK=2"
cd /tmp && export TMPDIR=/tmp
DNN_BWD_GROUP=2 step trace_bg2 120 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_bg2 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5
DNN_BWD_GROUP=2 DNN_RELU_MASK=2 step trace_bg2m 120 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_bg2m -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5
