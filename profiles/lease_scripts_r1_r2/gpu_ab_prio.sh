# A/B: GEMM main loop without / with s_setprio around MFMA bursts (rebuild on the box).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
(cd bench && timeout -k 10 400 python raster_sweep.py > $O/rasterA.jsonl 2> $O/rasterA.err) || exit $?
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/benchA.log 2>&1 || exit $?
DNN_HIP_DEFINES="-DDNN_GEMM_SETPRIO=1" timeout -k 10 600 python -m docker_dist_nn_amd._build > $O/buildB.log 2>&1 || exit $?
(cd bench && timeout -k 10 400 python raster_sweep.py > $O/rasterB.jsonl 2> $O/rasterB.err) || exit $?
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/benchB.log 2>&1 || exit $?
echo done > $O/ab.done
