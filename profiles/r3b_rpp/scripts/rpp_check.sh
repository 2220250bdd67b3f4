# persistent RP forward (stage code 15): bitwise tests, then whole-step A/B via table overrides
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r3b_rpp; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_persist_gpu.py -x -q -k rp_persist --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
MODELS=mlp8 bash scripts/r3b/env_ab.sh rpp_m8 DNN_TUNED=1 DNN_TUNED_TABLE=bench/tables/m8_fwd15.json DNN_TUNED_TABLE=bench/tables/m8_fwd15_all.json || exit 1
MODELS=head bash scripts/r3b/env_ab.sh rpp_head DNN_TUNED=1 DNN_TUNED_TABLE=bench/tables/h_fwd15.json || exit 1
MODELS=wide bash scripts/r3b/env_ab.sh rpp_wide DNN_TUNED=1 DNN_TUNED_TABLE=bench/tables/w_fwd15.json || exit 1
