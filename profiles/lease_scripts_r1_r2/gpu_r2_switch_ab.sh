# Alternating A/B of engine switches on the headline step (3 rounds). -> gpurun_out/r2_sw/ab.jsonl
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_sw; mkdir -p $O
cd $R
b() { tag=$1; shift; env $tag timeout -k 10 200 python bench.py --no-dp-compare "$@" \
  > $O/one.json 2>> $O/bench.err || exit $?
  python - "$tag" $O/one.json >> $O/ab.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(json.dumps({"env": sys.argv[1], "model": d["config"]["model"], "ms": d["ms_per_step"]}))
PY
}
for i in 1 2 3; do
  for e in DNN_X=0 DNN_WGRAD_STREAMS=2 DNN_BW_OVERLAP=1 DNN_GEMM_PERSIST=fwd=1 DNN_TAIL=0; do
    b $e --steps 50 --warmup 10
  done
done
cat $O/ab.jsonl
