R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cp $R/docker_dist_nn_amd/ops/tuned_gfx950.json $R/gpurun_out/tune_wide.json
step tune_wide 1100 python -u $R/bench/tune.py --configs 16384:wide --out $R/gpurun_out/tune_wide.json --stages 9,11 --persist 0 --steps 4 --reps 3 --margin 0.005 --verbose
