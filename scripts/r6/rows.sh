# Per-sample rate of the headline step at 16384 / 32768 / 65536 / 131072 rows (one micro-batch,
# the overlap plan) and 65536 rows as 2 x 32768 micro-batches.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
for b in 16384 32768 65536 131072; do
  step rows_$b 200 python -u $R/bench.py --batch $b --steps 50 --warmup 10
done
step micro_32768 200 python -u $R/bench.py --micro 32768 --steps 50 --warmup 10
step micro_16384 200 python -u $R/bench.py --micro 16384 --steps 50 --warmup 10
for f in $R/gpurun_out/rows_*.log $R/gpurun_out/micro_*.log; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f)"; done > $R/gpurun_out/rows_summary.txt
