set -o pipefail
O=gpurun_out/wgg2; mkdir -p $O; : > $O/ab.jsonl
for f in 256 2048 256 2048 256 2048; do
  DNN_WGRAD_GROUP_MAX_WG=$f timeout -k 10 150 python bench.py --steps 100 --warmup 20 > $O/one.json 2>>$O/err.log || exit 1
  python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'maxwg':'$f','ms':d['ms_per_step']}))" >> $O/ab.jsonl
done
