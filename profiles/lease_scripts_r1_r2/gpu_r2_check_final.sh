# Reduction + fused-optimizer tests and the three BASELINE steps with the current tree.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_check_final; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_opt_gpu.py tests/test_overlap_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
b() { timeout -k 10 300 python bench.py --no-dp-compare "$@" >> $O/bench.jsonl 2>> $O/bench.err || exit $?; }
b --steps 50 --warmup 10
b --model mlp8 --steps 20 --warmup 5
b --model wide --batch 16384 --steps 10 --warmup 3
python - $O/bench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["config"]["model"], d["ms_per_step"], round(d["value"] / 1e6, 2))
PY
