# Persistent dgrad with the post-swap ReLU mask: kernel tests, isolated cases, and an
# alternating mlp8 / wide / headline A/B of DNN_GEMM_PERSIST=dgrad=1. -> gpurun_out/r2_pdgrad/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_pdgrad; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gemm_persist_gpu.py tests/test_kernels_gpu.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python bench/ct_ab.py > $O/ct.jsonl 2>/dev/null || exit 1
grep 1024 $O/ct.jsonl
b() { tag=$1; shift; env $tag timeout -k 10 300 python bench.py --no-dp-compare "$@" \
  > $O/one.json 2>> $O/bench.err || exit $?
  python - "$tag" $O/one.json >> $O/ab.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(json.dumps({"env": sys.argv[1], "model": d["config"]["model"], "ms": d["ms_per_step"]}))
PY
}
for i in 1 2 3; do
  b DNN_X=0 --model mlp8 --steps 20 --warmup 5
  b DNN_GEMM_PERSIST=dgrad=1 --model mlp8 --steps 20 --warmup 5
  b DNN_X=0 --model wide --batch 16384 --steps 10 --warmup 3
  b DNN_GEMM_PERSIST=dgrad=1 --model wide --batch 16384 --steps 10 --warmup 3
  b DNN_X=0 --steps 50 --warmup 10
  b DNN_GEMM_PERSIST=dgrad=1 --steps 50 --warmup 10
done
cat $O/ab.jsonl
