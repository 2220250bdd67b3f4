# GPU tests + the three BASELINE training configs on one GPU (own kernels only: DNN_BLAS=0).
# Usage: bash scripts/gpu_r2_check.sh <tag> [pytest-args]   -> gpurun_out/<tag>/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-check}; mkdir -p $O
shift
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  "$@" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
export DNN_BLAS=0
b() { timeout -k 10 300 python bench.py "$@" >> $O/bench.jsonl 2>> $O/bench.err || exit $?; }
b --steps 50 --warmup 10
b --steps 20 --warmup 5 --model mlp8
b --steps 10 --warmup 3 --model wide --batch 16384
python - $O/bench.jsonl <<'EOF'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["config"]["model"], d["ms_per_step"], round(d["value"] / 1e6, 2), "M samples/s")
EOF
