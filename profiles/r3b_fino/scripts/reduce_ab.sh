# occupancy-aware reduce split: reduction tests, then old/new .so step A/B (head, mlp8)
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r3b_reduce; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_opt_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/r3b/ab_so.sh r3b_reduce/ab_head "--steps 50 --warmup 10" 4 || exit 1
bash scripts/r3b/ab_so.sh r3b_reduce/ab_m8 "--model mlp8 --steps 20 --warmup 5" 3 || exit 1
