# Side-stream priority for the overlap plan, with and without fork elision (headline A/B).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_prio; mkdir -p $O
cd $R
timeout -k 10 900 bash scripts/gpu_sw_ab.sh r2_prio "--steps 50 --warmup 10" 3 DNN_SIDE_PRIORITY=0 "DNN_SIDE_PRIORITY=1" "DNN_SIDE_PRIORITY=1 DNN_FORK_ELIDE=1" || exit 1
