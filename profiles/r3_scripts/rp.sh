# Register-prefetched main loop (stage codes 6/7): bitwise tests, then ring-form microbench A/B.
# -> gpurun_out/r3_rp/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r3_rp3}; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "register_prefetch or pipeline_depth" \
  > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -2 $O/kern.log
timeout -k 10 200 python bench/probes/gemm_timeline.py --variants 256x256:9,256x256:17,256x256:18 --wvariants 128x128:9,128x128:11 > $O/tl.jsonl && cat $O/tl.jsonl && timeout -k 10 600 python bench/stage_ab.py --rounds 5 > $O/stage_ab.jsonl 2> $O/stage_ab.err || { tail -20 $O/stage_ab.err; exit 1; }
python - $O/stage_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); print(d["case"], d["tile"], d["stages"], d["us_median"], d["tflops"], d["bitwise_equal_first"])
PY
