R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step mask_tests 600 $T $R/tests/test_relu_mask_gpu.py $R/tests/test_engine_gpu.py $R/tests/test_overlap_gpu.py
step env_auto 900 env PREFIX=r5 MODELS=head,mlp8,wide REPS=3 bash $R/scripts/env_ab.sh auto "DNN_RELU_MASK=0" "DNN_RELU_MASK=auto"
