# Same-box A/B of the round-5 final tree (built in ./_r5) against this tree: alternating runs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_vs_r6; mkdir -p $O; rm -f $O/ab.txt
for i in 1 2 3 4 5; do
  for t in r6 r5; do
    d=$R; [ $t = r5 ] && d=$R/_r5
    for m in head mlp8 wide; do
      case $m in
        head) args="--steps 20 --warmup 5";;
        mlp8) args="--model mlp8 --steps 20 --warmup 5";;
        wide) args="--model wide --batch 16384 --steps 10 --warmup 3";;
      esac
      (cd $d && timeout -k 10 200 python bench.py $args) | grep '^{' | sed "s/^/$t $m /" >> $O/ab.txt || exit 1
    done
  done
done
python - $O/ab.txt <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    t, m, js = l.split(" ", 2)
    d[(m, t)].append(json.loads(js)["ms_per_step"])
for k in sorted(d):
    v = sorted(d[k]); print(k, "median", v[len(v)//2], "all", v)
PY
