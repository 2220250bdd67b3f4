# Alternating A/B of tuned-table variants (DNN_TUNED_TABLE) on one model.
# Usage: bash scripts/gpu_r2_table_ab.sh <tag> "<bench args>" table1.json [table2.json ...]
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
ARGS=$2; shift 2
cd $R
b() { t=$1; env DNN_TUNED_TABLE=$t timeout -k 10 200 python bench.py --no-dp-compare $ARGS > $O/one.json 2>> $O/bench.err || exit $?
  python - "$t" $O/one.json >> $O/ab.jsonl <<'PY'
import json, sys, os
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(json.dumps({"table": os.path.basename(sys.argv[1]) or "default", "model": d["config"]["model"], "ms": d["ms_per_step"]}))
PY
}
for i in 1 2 3; do
  b ""
  for t in "$@"; do b $t; done
done
cat $O/ab.jsonl
