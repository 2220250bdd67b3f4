# Alternating whole-step A/B of environment settings (bench.py default form).
# usage: env_ab.sh NAME "VAR=a VAR2=b" "VAR=c" ... ; models from $MODELS (default head,mlp8)
# -> gpurun_out/r3b_env_NAME/ab.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; NAME=$1; shift; O=$R/gpurun_out/r3b_env_$NAME; mkdir -p $O
cd $R
MODELS=${MODELS:-head,mlp8}
for i in 1 2 3; do
  k=0
  for cfg in "$@"; do
    for m in ${MODELS//,/ }; do
      case $m in
        head) args="--steps 50 --warmup 10";;
        mlp8) args="--model mlp8 --steps 20 --warmup 5";;
        wide) args="--model wide --batch 16384 --steps 10 --warmup 3";;
      esac
      env $cfg timeout -k 10 200 python bench.py --no-dp-compare $args | sed "s/^/c$k $m /" >> $O/ab.txt || exit 1
    done
    k=$((k+1))
  done
done
printf '%s\n' "$@" | nl -v0 > $O/configs.txt
cat $O/configs.txt
python - $O/ab.txt <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    t, m, js = l.split(" ", 2)
    d[(m, t)].append(json.loads(js)["ms_per_step"])
for k in sorted(d):
    v = sorted(d[k]); print(k, "median", v[len(v)//2], "all", v)
PY
