# Round-6 second-session final checkpoint: whole GPU suite, smoke, five driver-form benches,
# and a kernel-trace + stats profile of a driver-form run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
step gpu_suite 720 python -u -m pytest tests -m gpu -v --timeout 420 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3 4 5; do
  step bench_f$i 200 python -u bench.py --steps 20 --warmup 5
done
grep -h '^{' gpurun_out/bench_f*.log | python -c "
import json, sys
v = [json.loads(l)['ms_per_step'] for l in sys.stdin]
print('driver-form ms_per_step', sorted(v), 'spread %.1f %%' % (100 * (max(v) / min(v) - 1)))
" | tee gpurun_out/bench_series_final.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_final -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof_final.log 2>&1
echo "prof rc=$?" | tee -a $R/gpurun_out/steps.txt
