# GEMM kernel tests, isolated epilogue cases, the three BASELINE steps (3 rounds).
# Usage: bash scripts/gpu_r2_epi2.sh <tag>  -> gpurun_out/<tag>/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-epi2}; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python bench/ct_ab.py > $O/ct.jsonl 2>/dev/null || exit 1
cat $O/ct.jsonl
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
