# where the overlap plan starts to pay: headline model, SGD, rows 1024..32768, overlap (min 0)
# vs single-stream (min 1e9)
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r3b_small; mkdir -p $O
for i in 1 2; do for r in 1024 4096 8192 16384 32768; do for t in 0 1000000000; do
  DNN_BW_OVERLAP_MIN_ROWS=$t timeout -k 10 120 python bench.py --batch $r --steps 100 --warmup 20 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.readlines()[-1]);print('rows $r', 'min_rows=$t', d['ms_per_step'], d['host_ms_per_step'])" | tee -a $O/threshold.txt || exit 1
done; done; done
