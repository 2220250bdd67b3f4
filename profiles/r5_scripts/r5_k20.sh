R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step mask_tests 600 $T $R/tests/test_relu_mask_gpu.py $R/tests/test_engine_gpu.py $R/tests/test_overlap_gpu.py
step env_m6 700 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh m6 "DNN_BW_OVERLAP=1" "DNN_BW_OVERLAP=6" "DNN_BW_OVERLAP=6 DNN_RELU_MASK=2" "DNN_BW_OVERLAP=1 DNN_RELU_MASK=2"
