# IPC fan plan (interpreted, processes sharing cuda:0) + the capture-after-eager test.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
step t_ipcfan 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_fan_gpu.py -k "ipc"
step t_capture 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_overlap_gpu.py -k "capture or interleaved"
