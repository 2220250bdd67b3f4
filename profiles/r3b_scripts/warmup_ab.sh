# Is the first timed window of a fresh bench process slower (clock ramp)? fresh processes,
# alternating --warmup 10 / 300 / 3000 -> gpurun_out/r3b_warm/ab.txt
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r3b_warm; mkdir -p $O
for i in 1 2 3; do for w in 10 300 3000; do
  timeout -k 10 200 python bench.py --steps 50 --warmup $w > $O/one.json 2>> $O/err.txt || exit 1
  python -c "import json;d=json.loads(open('$O/one.json').readlines()[-1]);print('w$w', d['ms_per_step'])" >> $O/ab.txt
done; done
cat $O/ab.txt
