# DZ4 trim: tail GPU tests + engine tests that use the tail, probe sweep
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3b_tail3; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_mlp_tail_gpu.py tests/test_engine_gpu.py tests/test_overlap_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench/probes/tail_probe.py --rows 65536,131072 > $O/tail_probe.jsonl 2> $O/tail_probe.err || { tail -20 $O/tail_probe.err; exit 1; }
cat $O/tail_probe.jsonl
