# BK=32 tile variants: bitwise tests + microbench A/B; split-FINO overlap plan: bitwise test +
# alternating step A/B. -> gpurun_out/r3_bk32/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3_bk32; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_overlap_gpu.py -x -q --timeout 300 --timeout-method thread -k "bk32 or pipeline_depth or overlap" \
  > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -2 $O/kern.log
for i in 1 2 3; do
  for f in 0 1; do
    DNN_SPLIT_FINO=$f timeout -k 10 200 python bench.py --steps 50 --warmup 10 | sed "s/^/fino$f head /" >> $O/fino_ab.txt || exit 1
    DNN_SPLIT_FINO=$f timeout -k 10 200 python bench.py --model mlp8 --steps 20 --warmup 5 | sed "s/^/fino$f mlp8 /" >> $O/fino_ab.txt || exit 1
  done
done
python - $O/fino_ab.txt <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    t, m, js = l.split(" ", 2)
    d[(m, t)].append(json.loads(js)["ms_per_step"])
for k in sorted(d):
    v = sorted(d[k]); print(k, "median", v[len(v)//2], "all", v)
PY
timeout -k 10 600 python bench/stage_ab.py --rounds 5 > $O/stage_ab.jsonl 2> $O/stage_ab.err || { tail -20 $O/stage_ab.err; exit 1; }
cat $O/stage_ab.jsonl
