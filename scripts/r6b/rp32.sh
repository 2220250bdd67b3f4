# 32-deep register-prefetched ring (codes 20 / 21): bitwise test, cold isolated A/B, then
# in-step driver-form A/Bs of the forward / dgrad kinds on it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
step rp_bitwise 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -v -k register_prefetch --timeout 240 --timeout-method thread
grep -q "failed" gpurun_out/rp_bitwise.log && exit 1
step rp32_ab 300 python -u bench/probes/rp32_ab.py --reps 15
for i in 1 2 3; do
  step st9_$i 200 python -u bench.py --steps 20 --warmup 5
  step st20_$i 200 env DNN_GEMM_STAGES=fwd=20,dgrad=20 python -u bench.py --steps 20 --warmup 5
  step st21_$i 200 env DNN_GEMM_STAGES=fwd=21,dgrad=21 python -u bench.py --steps 20 --warmup 5
done
for v in 9 20 21; do
  echo "code $v: $(cat gpurun_out/st${v}_*.log | grep '^{' | python -c 'import json,sys; print(sorted(json.loads(l)["ms_per_step"] for l in sys.stdin))')" | tee -a gpurun_out/rp32_step_ab.txt
done
