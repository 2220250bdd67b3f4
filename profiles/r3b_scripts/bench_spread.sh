# Process-to-process spread of the default bench on one box: 8 fresh runs -> gpurun_out/r3b_spread/
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r3b_spread; mkdir -p $O
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 python bench.py > $O/one.json 2>> $O/err.txt || exit 1
  tail -1 $O/one.json >> $O/runs.jsonl
done
python - $O/runs.jsonl <<'PY'
import json, sys, statistics as st
v = [json.loads(l)["ms_per_step"] for l in open(sys.argv[1])]
print("ms per step:", v, "median", st.median(v), "min", min(v), "max", max(v))
PY
