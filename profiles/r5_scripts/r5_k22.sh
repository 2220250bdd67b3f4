R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step ov_tests 600 $T $R/tests/test_overlap_gpu.py
step env_delay 900 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh delay "DNN_FORK_ELIDE=0" "DNN_FORK_ELIDE=1 DNN_SIDE_DELAY_US=8" "DNN_FORK_ELIDE=1 DNN_SIDE_DELAY_US=15" "DNN_FORK_ELIDE=1 DNN_SIDE_DELAY_US=25" "DNN_FORK_ELIDE=1 DNN_SIDE_DELAY_US=40" "DNN_FORK_ELIDE=0 DNN_SIDE_DELAY_US=10"
