# Round-6 changes on the GPU: fan (co-location, bench rehearsal with uniform + DP measured),
# overlap plans after the pruning, the persistent chain kernel (stop polling, acq_rel counter).
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
step t_overlap 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_overlap_gpu.py
step t_chain 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_chain_fast_gpu.py
step t_fan 1000 python -u -m pytest -x -v --timeout 420 --timeout-method thread tests/test_fan_gpu.py
