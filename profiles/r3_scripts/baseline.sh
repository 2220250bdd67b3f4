# Round-3 baseline on today's box: default bench (driver form), the three BASELINE steps, and a
# kernel trace of the headline step. -> gpurun_out/r3_base/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r3_base}; mkdir -p $O
cd $R
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-200
b() { timeout -k 10 300 python bench.py --no-dp-compare "$@" >> $O/bench.jsonl 2>> $O/bench.err || exit $?; }
b --model mlp8 --steps 20 --warmup 5
b --model wide --batch 16384 --steps 10 --warmup 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/step -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $O/step.log 2>&1 || exit $?
cd $R
python scripts/trace_summary.py $O/step/run_kernel_trace.csv --steps 3 > $O/step.summary.txt
cat $O/step.summary.txt
python - $O/bench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"]["model"], d["ms_per_step"], round(d["value"] / 1e6, 2), "M samples/s")
PY
