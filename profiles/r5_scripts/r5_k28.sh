R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step reduce_tests 300 $T $R/tests/test_kernels_gpu.py -k reduce_multi
step env_fino 900 env PREFIX=r5 MODELS=head,mlp8 REPS=3 bash $R/scripts/env_ab.sh fino "DNN_FINO_SIDE_BLOCKS=0" "DNN_FINO_SIDE_BLOCKS=64" "DNN_FINO_SIDE_BLOCKS=128" "DNN_FINO_SIDE_BLOCKS=256"
