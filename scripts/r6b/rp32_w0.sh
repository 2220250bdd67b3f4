# W0 (512x832 wgrad) on stage code 20 in the step (alternate tuned table), driver form.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
for i in 1 2 3 4; do
  step w9_$i 200 python -u bench.py --steps 20 --warmup 5
  step w20_$i 200 env DNN_TUNED_TABLE=bench/probes/tuned_w0_code20.json python -u bench.py --steps 20 --warmup 5
done
for v in 9 20; do
  echo "W0 code $v: $(cat gpurun_out/w${v}_*.log | grep '^{' | python -c 'import json,sys; print(sorted(json.loads(l)["ms_per_step"] for l in sys.stdin))')" | tee -a gpurun_out/rp32_w0_ab.txt
done
