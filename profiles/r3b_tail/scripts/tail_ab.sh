# Tail rework: GPU tail tests, probe sweep, then old-vs-new .so A/B on the headline and mlp8
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3b_tail2; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_mlp_tail_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench/probes/tail_probe.py > $O/tail_probe.jsonl 2> $O/tail_probe.err || { tail -20 $O/tail_probe.err; exit 1; }
cat $O/tail_probe.jsonl
bash scripts/r3b/ab_so.sh r3b_tail2/ab_head "--steps 50 --warmup 10" 4 || exit 1
