# Session-2 re-check: the co-located fan GPU tests fixed after the last commit, then an A/B of
# the fused fwd(512->256)+tail launch (DNN_FWD_TAIL) on the round-6 build, driver form.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
step fan_gpu 400 python -u -m pytest tests/test_fan_gpu.py -m gpu -v --timeout 300 --timeout-method thread
for i in 1 2 3; do
  for v in 0 1; do
    step fwdtail_${v}_$i 200 env DNN_FWD_TAIL=$v python -u bench.py --steps 20 --warmup 5
  done
done
grep -h '^{' gpurun_out/fwdtail_*.log > /dev/null
for v in 0 1; do
  echo "DNN_FWD_TAIL=$v: $(cat gpurun_out/fwdtail_${v}_*.log | grep '^{' | python -c 'import json,sys; print(sorted(json.loads(l)["ms_per_step"] for l in sys.stdin))')" | tee -a gpurun_out/fwdtail_ab.txt
done
