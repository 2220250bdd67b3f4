# A/B of two builds of the native extension on one box: the tree as is (B) against a copy of it
# running build_ab/_native_old.so (A), alternating. Usage:
#   bash scripts/r3b/ab_so.sh <tag> "<bench args>" [rounds]  -> gpurun_out/<tag>/ab.jsonl
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab_so}; mkdir -p $O
ARGS=$2; N=${3:-3}
OLD=/tmp/ab_old_tree; rm -rf $OLD; mkdir -p $OLD
cd $R && tar --exclude=./gpurun_out --exclude=./build_ab --exclude=./build -cf - . | (cd $OLD && tar xf -)
cp $R/build_ab/_native_old.so $OLD/docker_dist_nn_amd/_native.cpython-310-x86_64-linux-gnu.so
b() { tag=$1; dir=$2; (cd $dir && timeout -k 10 200 python bench.py --no-dp-compare $ARGS) > $O/one.json 2>> $O/bench.err || exit $?
  python - "$tag" $O/one.json >> $O/ab.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(json.dumps({"build": sys.argv[1], "model": d["config"]["model"], "ms": d["ms_per_step"]}))
PY
}
for i in $(seq $N); do b A $OLD; b B $R; done
python - $O/ab.jsonl <<'PY'
import json, sys, statistics as st
rows = [json.loads(l) for l in open(sys.argv[1])]
for m in sorted({r["model"] for r in rows}):
    for b in "AB":
        v = [r["ms"] for r in rows if r["model"] == m and r["build"] == b]
        if v:
            print(m, b, "median", st.median(v), "all", v)
PY
