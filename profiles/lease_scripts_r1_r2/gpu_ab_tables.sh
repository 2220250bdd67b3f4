set -e
mkdir -p gpurun_out
for i in 1 2 3; do
  cp docker_dist_nn_amd/ops/tuned_gfx950.json /tmp/old.json 2>/dev/null || true
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 | grep metric | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('old', d['ms_per_step'])" >> gpurun_out/ab_tables.txt
  cp profiles/r1_persist/tuned_persist.json docker_dist_nn_amd/ops/tuned_gfx950.json
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 | grep metric | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('new', d['ms_per_step'])" >> gpurun_out/ab_tables.txt
  cp /tmp/old.json docker_dist_nn_amd/ops/tuned_gfx950.json
done
