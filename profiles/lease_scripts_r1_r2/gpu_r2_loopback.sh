# Single-process pipelines on one GPU (loopback): the schedule on one stream vs one stream per
# stage (DNN_LOOPBACK_STREAMS), alternating; engine parity tests first.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_lb; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.jsonl
for cfg in "mnist-fcnn pp4 20" "mlp8 pp8 6" "mnist-fcnn pp2 20"; do
  set -- $cfg
  for v in 0 1 0 1; do
    DNN_LOOPBACK_STREAMS=$v timeout -k 10 200 python bench.py --model $1 --parallelism $2 --steps $3 --warmup 3 > $O/one.json 2>> $O/err.log || exit 1
    python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'model':'$1','par':'$2','streams':$v,'ms':d['ms_per_step'],'nm':d['config']['num_micro']}))" | tee -a $O/ab.jsonl
  done
done
