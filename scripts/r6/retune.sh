# Re-tune the wide and mlp8 models in-step on the round-6 kernels (a copy of the table), then an
# alternating A/B of the new table against the shipped one.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
cp docker_dist_nn_amd/ops/tuned_gfx950.json gpurun_out/retuned.json
step retune 900 python -u bench/tune.py --configs 16384:wide,65536:mlp8 --stages 2,9,11 --persist 0 --out gpurun_out/retuned.json --steps 6 --reps 3
PREFIX=r6 MODELS=wide,mlp8 REPS=3 step retune_ab 600 bash scripts/env_ab.sh retune "DNN_TUNED=1" "DNN_TUNED_TABLE=$R/gpurun_out/retuned.json"
