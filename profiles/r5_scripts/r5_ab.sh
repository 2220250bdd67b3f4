# Same-box A/B of two native builds: NEW = in-tree .so, OLD = $OLD_SO (default ab/r4_native.so),
# interleaved bench runs (driver form 20 / 5 and a longer 50 / 10), then optional extra steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
OLD=${OLD_SO:-$R/ab/r4_native.so}
for i in 1 2 3; do
  step ab_new_$i 200 python -u $R/bench.py --steps 50 --warmup 10
  step ab_old_$i 200 env DNN_NATIVE_PATH=$OLD python -u $R/bench.py --steps 50 --warmup 10
done
for f in $R/gpurun_out/ab_*_?.log; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done | tee $R/gpurun_out/ab_summary.txt
