# Same-box comparison: ours (bench.py) vs PyTorch-ROCm (bench/torch_baseline.py) on the three
# BASELINE one-GPU models -> gpurun_out/r3b_vs_torch/vs_torch.jsonl
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r3b_vs_torch; mkdir -p $O
for m in "mnist-fcnn:65536:50:10" "mlp8:65536:20:5" "wide:16384:10:3"; do
  IFS=: read model batch steps warm <<< "$m"
  timeout -k 10 300 python bench.py --model $model --batch $batch --steps $steps --warmup $warm > $O/ours.json 2>> $O/err.txt || exit 1
  python -c "import json;d=json.loads(open('$O/ours.json').readlines()[-1]);print(json.dumps({'impl':'ours','model':'$model','batch':$batch,'ms':d['ms_per_step'],'samples_per_s':d['value']}))" >> $O/vs_torch.jsonl
  timeout -k 10 600 python bench/torch_baseline.py --model $model --batch $batch --steps $steps --warmup $warm > $O/torch.jsonl 2>> $O/err.txt || exit 1
  python - $O/torch.jsonl $model $batch >> $O/vs_torch.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); d["impl"] = "torch"; d["model"] = sys.argv[2]; print(json.dumps(d))
PY
done
cat $O/vs_torch.jsonl
