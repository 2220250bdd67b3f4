# Alternating whole-step A/B of two tuned tables (current vs $1), bench.py default form,
# 4 rounds x {headline, mlp8, wide}. -> gpurun_out/r3_abt/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3_abt_${2:-x}; mkdir -p $O
cd $R
B=${1:-bench/tables/table_asym.json}
test -f $B || { echo "missing table $B"; exit 1; }
for i in 1 2 3 4; do
  for t in cur new; do
    if [ $t = new ]; then export DNN_TUNED_TABLE=$B; else unset DNN_TUNED_TABLE; fi
    timeout -k 10 200 python bench.py --steps 50 --warmup 10 | sed "s/^/$t head /" >> $O/ab.txt || exit 1
    timeout -k 10 200 python bench.py --model mlp8 --steps 20 --warmup 5 | sed "s/^/$t mlp8 /" >> $O/ab.txt || exit 1
    timeout -k 10 200 python bench.py --model wide --batch 16384 --steps 10 --warmup 3 | sed "s/^/$t wide /" >> $O/ab.txt || exit 1
  done
done
python - $O/ab.txt <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    t, m, js = l.split(" ", 2)
    d[(m, t)].append(json.loads(js)["ms_per_step"])
for k in sorted(d):
    v = sorted(d[k]); print(k, "median", v[len(v)//2], "all", v)
PY
