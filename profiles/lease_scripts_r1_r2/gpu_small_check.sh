set -o pipefail
O=gpurun_out/smab; mkdir -p $O; : > $O/ab.jsonl
for m in "--model mnist-784-128-10 --steps 100 --warmup 20" "--steps 100 --warmup 20"; do
  for i in 1 2; do
    timeout -k 10 150 python bench.py $m > $O/one.json 2>>$O/err.log || exit 1
    python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'model':d['config']['model'],'ms':d['ms_per_step']}))" >> $O/ab.jsonl
  done
done
