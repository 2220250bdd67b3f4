# Eager vs HIP-graph replay of the headline step (alternating), then a trace of the graph run.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_graph; mkdir -p $O
cd $R
b() { tag=$1; shift; timeout -k 10 200 python bench.py --no-dp-compare --steps 50 --warmup 10 "$@" > $O/one.json 2>> $O/bench.err || exit $?
  python - "$tag" $O/one.json >> $O/ab.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(json.dumps({"mode": sys.argv[1], "model": d["config"]["model"], "ms": d["ms_per_step"]}))
PY
}
for i in 1 2 3; do b eager; b graph --graph; b graph1 --graph --graph-copies 1; done
cat $O/ab.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --graph > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R && python scripts/trace_summary.py $O/prof/run_kernel_trace.csv --steps 3 > $O/summary.txt; head -14 $O/summary.txt
