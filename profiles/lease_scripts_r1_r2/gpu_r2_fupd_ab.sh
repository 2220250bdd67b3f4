# Fused-update wgrad epilogue (master prefetch): bitwise tests, then wide with the fused
# update on / off, alternating. -> gpurun_out/r2_fupd/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_fupd; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_overlap_gpu.py tests/test_kernels_gpu.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
b() { tag=$1; shift; env $tag timeout -k 10 200 python bench.py --no-dp-compare "$@" \
  > $O/one.json 2>> $O/bench.err || exit $?
  python - "$tag" $O/one.json >> $O/ab.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(json.dumps({"env": sys.argv[1], "model": d["config"]["model"], "ms": d["ms_per_step"]}))
PY
}
for i in 1 2 3; do
  b DNN_WGRAD_FUSED_UPDATE=0 --model wide --batch 16384 --steps 10 --warmup 3
  b DNN_WGRAD_FUSED_UPDATE=1 --model wide --batch 16384 --steps 10 --warmup 3
done
cat $O/ab.jsonl
