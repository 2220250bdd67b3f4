# Layer-0 ReLU mask with the double-buffered layer-0 activation: bitwise test, A/B, traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
step mask_test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_overlap_gpu.py -k "mask or cross_step"
PREFIX=r6 MODELS=head REPS=3 step mask_ab 600 bash scripts/env_ab.sh maskh0 "DNN_RELU_MASK=auto" "DNN_RELU_MASK=2" "DNN_RELU_MASK=2 DNN_H0_DOUBLE=0"
cd /tmp && export TMPDIR=/tmp
for c in auto 2; do
  DNN_RELU_MASK=$c step trace_$c 120 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_mask_$c -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5
done
