# Round-6 final checkpoint: whole GPU suite, smoke, a 10-run driver-form bench series.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
step gpu_suite 700 python -u -m pytest tests -m gpu -v --timeout 420 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
for i in $(seq 10); do
  step bench_d$i 200 python -u bench.py --steps 20 --warmup 5
done
grep -h '^{' gpurun_out/bench_d*.log | python -c "
import json, sys
v = [json.loads(l)['ms_per_step'] for l in sys.stdin]
print('driver-form ms_per_step', sorted(v), 'spread %.1f %%' % (100 * (max(v) / min(v) - 1)))
" | tee gpurun_out/bench_series.txt
