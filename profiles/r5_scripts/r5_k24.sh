R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cp $R/docker_dist_nn_amd/ops/tuned_gfx950.json $R/gpurun_out/tune_head.json
step tune_head 1000 python -u $R/bench/tune.py --configs 65536:mnist-fcnn --out $R/gpurun_out/tune_head.json --stages 9,11 --persist 0 --steps 20 --reps 3 --margin 0.005
