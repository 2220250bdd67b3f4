# reduce_multi loads per thread: A = build_ab/_native_old.so (8 loads), B = tree (4 loads).
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 900 bash $R/scripts/gpu_ab_so.sh r2_reduce_loads "--steps 50 --warmup 10" 4 || exit 1
bash $R/scripts/gpu_r2_prof_ab.sh r2_reduce_loads_prof "--steps 20 --warmup 5" > /dev/null 2>&1 || exit 1
grep reduce_multi $R/gpurun_out/r2_reduce_loads_prof/A.summary.txt $R/gpurun_out/r2_reduce_loads_prof/B.summary.txt | grep calls
