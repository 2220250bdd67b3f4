# Ping-pong 256x256 form (DNN_GEMM_STAGES=fwd=8) against the one-tile form on the wide and
# mlp8 steps, alternating. -> gpurun_out/r2_pp/ab.jsonl
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_pp; mkdir -p $O
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
  b DNN_X=0 --model wide --batch 16384 --steps 10 --warmup 3
  b DNN_GEMM_STAGES=fwd=8 --model wide --batch 16384 --steps 10 --warmup 3
done
cat $O/ab.jsonl
