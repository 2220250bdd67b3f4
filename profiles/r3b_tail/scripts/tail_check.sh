# Tail kernel change: GPU tests of the tail, the probe sweep, and the headline bench
# -> gpurun_out/${OUT:-r3b_tail}/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r3b_tail}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_mlp_tail_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench/probes/tail_probe.py > $O/tail_probe.jsonl 2> $O/tail_probe.err || { tail -20 $O/tail_probe.err; exit 1; }
cat $O/tail_probe.jsonl
for i in 1 2 3; do
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').readlines()[-1]);print(d['ms_per_step'], round(d['value']/1e6,1))"
done
