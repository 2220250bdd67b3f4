R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step gpu_suite 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step env_mask8 700 env PREFIX=r5 MODELS=mlp8,wide REPS=3 bash $R/scripts/env_ab.sh mask8 "DNN_RELU_MASK=0" "DNN_RELU_MASK=2" "DNN_RELU_MASK=1"
