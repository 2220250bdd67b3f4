# In-step tuning of the headline's micro-batch GEMM shapes (the fan stages' fwd / dgrad at
# 8192-32768 rows; DNN_TAIL=0 so layers 2-3 run as plain GEMMs, as in a fan's heavy stage).
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
cp docker_dist_nn_amd/ops/tuned_gfx950.json gpurun_out/tuned_micro.json
ONLY=""
for r in 8192 16384 32768; do
  ONLY="$ONLY,fwd:${r}x512x832,fwd:${r}x256x512,fwd:${r}x128x256,dgrad:${r}x512x256,dgrad:${r}x256x128"
done
DNN_TAIL=0 step tune_micro 1000 python -u bench/tune.py --configs 8192:mnist-fcnn,16384:mnist-fcnn,32768:mnist-fcnn --only ${ONLY#,} --stages 2,9 --persist 0 --tiles 256x256,256x128,256x64,128x128,128x64 --out gpurun_out/tuned_micro.json --steps 10 --reps 3
