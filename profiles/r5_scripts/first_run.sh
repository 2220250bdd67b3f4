# Is the first bench process on a box slower, and is it the previous process's freed memory?
# A: smoke, then the driver-form bench 3x (per-step events). B: a process that fills and frees
# 120 GiB of HBM, then the bench 2x right after it, then again after a 60 s pause.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r5_first; mkdir -p $O; cd $R
export DNN_BENCH_STEP_EVENTS=1
run() { timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-dp-compare | sed "s/^/$1 $(date +%s) /" >> $O/runs.txt || exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
run A1; run A2; run A3
timeout -k 10 200 python -u -c "
import torch, time
t = torch.empty(120 << 30, dtype=torch.uint8, device='cuda'); t.fill_(1); torch.cuda.synchronize()
print('filled', time.time(), flush=True)" > $O/fill.log 2>&1 || exit 1
run B1; run B2
sleep 60
run C1
