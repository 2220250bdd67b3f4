R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
for i in 1 2 3; do
  step mlp8_$i 200 python -u bench.py --model mlp8 --steps 20 --warmup 5
  step wide_$i 200 python -u bench.py --model wide --batch 16384 --steps 10 --warmup 3
done
grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/mlp8_*.log gpurun_out/wide_*.log > gpurun_out/models_summary.txt
