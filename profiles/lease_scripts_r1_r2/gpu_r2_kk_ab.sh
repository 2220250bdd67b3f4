# Alternating A/B of K-major weight gradients for every eligible layer (DNN_WGRAD_KK=1) vs the
# default (auto: layers >= 16M weights) on the headline and mlp8 steps. -> gpurun_out/r2_kk/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_kk; mkdir -p $O
cd $R
b() { tag=$1; shift; env $tag timeout -k 10 300 python bench.py --no-dp-compare "$@" \
  > $O/one.json 2>> $O/bench.err || exit $?
  python - "$tag" $O/one.json >> $O/ab.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(json.dumps({"env": sys.argv[1], "model": d["config"]["model"], "ms": d["ms_per_step"]}))
PY
}
for i in 1 2 3; do
  b DNN_WGRAD_KK=auto --steps 50 --warmup 10
  b DNN_WGRAD_KK=1 --steps 50 --warmup 10
  b DNN_WGRAD_KK=auto --model mlp8 --steps 20 --warmup 5
  b DNN_WGRAD_KK=1 --model mlp8 --steps 20 --warmup 5
done
cat $O/ab.jsonl
