# dgrad/wgrad overlap plan (DNN_BW_OVERLAP) on all three BASELINE steps, alternating, plus its
# bitwise test. -> gpurun_out/r2_ov/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_ov; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_overlap_gpu.py tests/test_engine_gpu.py -x -q \
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
  for e in DNN_BW_OVERLAP=0 DNN_BW_OVERLAP=1; do
    b $e --steps 50 --warmup 10
    b $e --model mlp8 --steps 20 --warmup 5
    b $e --model wide --batch 16384 --steps 10 --warmup 3
  done
done
cat $O/ab.jsonl
