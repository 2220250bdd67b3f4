# GEMM numerics (ct / K-major / epilogue tests) + the three BASELINE steps, 3 runs each.
# -> gpurun_out/r2_epi/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_epi; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
b() { timeout -k 10 300 python bench.py --no-dp-compare "$@" > $O/one.json 2>> $O/bench.err || exit $?
  python - $O/one.json >> $O/ab.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(json.dumps({"model": d["config"]["model"], "ms": d["ms_per_step"]}))
PY
}
for i in 1 2 3; do
  b --steps 50 --warmup 10
  b --model mlp8 --steps 20 --warmup 5
  b --model wide --batch 16384 --steps 10 --warmup 3
done
cat $O/ab.jsonl
