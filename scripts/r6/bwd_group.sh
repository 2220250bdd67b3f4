# The mixed grouped backward launch (DNN_BWD_GROUP=1): bitwise test, A/B against the default plan,
# kernel trace of the grouped step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
step bg_test 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_overlap_gpu.py -k "mixed_backward"
grep -q "1 passed" gpurun_out/bg_test.log || exit 1
PREFIX=r6 MODELS=head REPS=4 step bg_ab 600 bash scripts/env_ab.sh bwdgroup "DNN_BWD_GROUP=0" "DNN_BWD_GROUP=1" "DNN_BWD_GROUP=1 DNN_XSTEP=0"
cd /tmp && export TMPDIR=/tmp
DNN_BWD_GROUP=1 step trace_bg 120 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_bg -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5
