# Round-end dress rehearsal: the whole GPU suite, smoke(), and bench.py exactly as the driver
# runs it at N=1 (default flags), plus the three BASELINE steps. -> gpurun_out/r2_final/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_final; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-300
b() { timeout -k 10 300 python bench.py --no-dp-compare "$@" >> $O/bench.jsonl 2>> $O/bench.err || exit $?; }
b --steps 50 --warmup 10
b --model mlp8 --steps 20 --warmup 5
b --model wide --batch 16384 --steps 10 --warmup 3
python - $O/bench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"]["model"], d["ms_per_step"], round(d["value"] / 1e6, 2), "M samples/s")
PY
