# host-bound small steps: overlap plan (threshold 0) vs the single-stream plan (default for
# < 4096 rows), the reference's small recipes; plus overlap tests
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r3b_small; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_overlap_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do for m in 784-128-64-10 784-32-16-10 784-512-256-128-10; do for t in 0 4096; do
  DNN_BW_OVERLAP_MIN_ROWS=$t timeout -k 10 120 python bench.py --model $m --batch 64 --optimizer adam --steps 300 --warmup 50 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.readlines()[-1]);print('$m', 'min_rows=$t', d['ms_per_step'], d['host_ms_per_step'])" | tee -a $O/small.txt || exit 1
done; done; done
