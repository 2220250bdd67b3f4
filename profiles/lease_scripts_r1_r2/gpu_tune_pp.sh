# Re-tune the mlp8 / wide / headline step GEMMs with the ping-pong form as a candidate, and
# bench each model before and after (same box).
set -e
mkdir -p gpurun_out
T=gpurun_out/tuned_pp.json
cp docker_dist_nn_amd/ops/tuned_gfx950.json $T
for m in "mlp8 65536" "wide 16384" "mnist-fcnn 65536"; do
  set -- $m
  timeout -k 10 120 python bench.py --model $1 --batch $2 --steps 30 --warmup 5 | grep metric >> gpurun_out/tune_pp_before.jsonl
done
timeout -k 10 1000 python bench/tune.py --configs 65536:mlp8,16384:wide,65536:mnist-fcnn --persist 0 --out $T > gpurun_out/tune_pp.jsonl 2>&1
cp $T docker_dist_nn_amd/ops/tuned_gfx950.json
for m in "mlp8 65536" "wide 16384" "mnist-fcnn 65536"; do
  set -- $m
  timeout -k 10 120 python bench.py --model $1 --batch $2 --steps 30 --warmup 5 | grep metric >> gpurun_out/tune_pp_after.jsonl
done
