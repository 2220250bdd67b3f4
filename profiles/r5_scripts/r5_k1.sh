R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step kern_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $R/tests/test_kernels_gpu.py
source $R/scripts/r5_ab.sh
OUT=r5_pmc_a bash $R/scripts/pmc_step.sh > $R/gpurun_out/r5_pmc_a.log 2>&1
step fan_gpu 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread $R/tests/test_fan_gpu.py
