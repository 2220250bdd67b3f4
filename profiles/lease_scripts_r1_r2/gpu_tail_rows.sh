set -o pipefail
mkdir -p gpurun_out/tailrows
for r in 16384 32768 65536 131072 262144; do
  timeout -k 10 100 python -u bench/tail_ab.py --rows $r --iters 30 >> gpurun_out/tailrows/ab.jsonl 2>&1 || exit 1
done
