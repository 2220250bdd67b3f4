R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cp $R/docker_dist_nn_amd/ops/tuned_gfx950.json $R/gpurun_out/tune_mlp8.json
step tune_mlp8 1000 python -u $R/bench/tune.py --configs 65536:mlp8 --out $R/gpurun_out/tune_mlp8.json --stages 9,11 --persist 0 --steps 8 --reps 3 --margin 0.005
