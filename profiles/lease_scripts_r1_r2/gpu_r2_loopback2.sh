# Loopback pipelines: graph replay x per-stage streams x micro-batch size.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_lb2; mkdir -p $O
cd $R
: > $O/ab.jsonl
run() {
  DNN_LOOPBACK_STREAMS=$1 timeout -k 10 200 python bench.py --model $2 --parallelism $3 --steps $4 --warmup 3 $5 > $O/one.json 2>> $O/err.log || exit 1
  python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'model':'$2','par':'$3','streams':$1,'args':'$5','ms':d['ms_per_step'],'nm':d['config']['num_micro']}))" | tee -a $O/ab.jsonl
}
for rep in 1 2; do
  for v in 0 1; do
    run $v mnist-fcnn pp4 30 ""
    run $v mnist-fcnn pp4 30 "--micro 4096"
    run $v mnist-fcnn pp4 30 "--micro 8192"
    run $v mlp8 pp8 8 ""
    run $v mnist-fcnn pp2 30 ""
  done
done
