# Alternating A/B of env switch settings on one bench config. Usage:
#   bash scripts/gpu_sw_ab.sh <tag> "<bench args>" <rounds> ENV=a ENV=b ...  -> gpurun_out/<tag>/ab.jsonl
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
ARGS=$2; N=$3; shift 3
cd $R
b() { tag=$1; env $tag timeout -k 10 200 python bench.py --no-dp-compare $ARGS > $O/one.json 2>> $O/bench.err || exit $?
  python - "$tag" $O/one.json >> $O/ab.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(json.dumps({"env": sys.argv[1], "model": d["config"]["model"], "ms": d["ms_per_step"]}))
PY
}
for i in $(seq $N); do for e in "$@"; do b "$e"; done; done
python - $O/ab.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); d[r["env"]].append(r["ms"])
for k, v in d.items():
    print(k, "mean %.4f min %.4f" % (sum(v) / len(v), min(v)), v)
PY
