# In-step tuning of the 256x256 fwd/dgrad GEMMs with the asymmetric A3/B2 ring (stages 5)
# against the incumbents. -> gpurun_out/r3_tune/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3_tune; mkdir -p $O
cd $R
cp docker_dist_nn_amd/ops/tuned_gfx950.json $O/tuned.json
ONLY=fwd:65536x512x832,fwd:65536x256x512,dgrad:65536x512x256,dgrad:65536x256x128,fwd:65536x1024x1024,fwd:65536x1024x832,dgrad:65536x1024x1024,fwd:16384x8192x8192,fwd:16384x8192x832,dgrad:16384x8192x8192
timeout -k 10 1000 python bench/tune.py --configs 65536:mnist-fcnn,65536:mlp8,16384:wide \
  --only $ONLY --tiles 256x256 --stages 2,5 --persist 0,1 --verbose --steps 10 --reps 3 \
  --out $O/tuned.json > $O/tune.jsonl 2> $O/tune.err || { tail -20 $O/tune.err; exit 1; }
grep -v '"cand"' $O/tune.jsonl
