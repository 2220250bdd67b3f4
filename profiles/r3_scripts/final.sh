# Round-end rehearsal: the driver's GPU tier (pytest -m gpu, smoke) and the default bench plus
# the three BASELINE models. -> gpurun_out/${OUT:-r3_final}/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r3_final}; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-220
for m in "--model mlp8 --steps 20 --warmup 5" "--model wide --batch 16384 --steps 10 --warmup 3" "--steps 50 --warmup 10"; do
  timeout -k 10 300 python bench.py --no-dp-compare $m >> $O/bench_models.jsonl 2>> $O/bench_models.err || exit 1
done
python - $O/bench_models.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"]["model"], d["ms_per_step"], round(d["value"] / 1e6, 2), "M samples/s")
PY
