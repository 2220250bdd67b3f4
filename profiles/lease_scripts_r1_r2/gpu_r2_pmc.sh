# PMC counters of every kernel of the headline and wide training steps (own kernels), one
# pass per counter group (kernel-trace + pmc only). -> gpurun_out/r2_pmc/<model>/<pass>/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {
  local d=$1 name=$2; shift 2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $O/$d/$name -o run --output-format csv \
    -- python3 $R/bench.py $BARGS > $O/$d/$name.log 2>&1
  local rc=$?
  echo "$d $name rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || exit $rc
}
for m in step wide; do
  mkdir -p $O/$m
  if [ $m = step ]; then BARGS="--steps 3 --warmup 2"; else BARGS="--model wide --batch 16384 --steps 2 --warmup 1"; fi
  run $m sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE
  run $m fetch FETCH_SIZE
  run $m write WRITE_SIZE
done
cd $R
python scripts/pmc_step_summary.py $O/step > $O/step_summary.txt && python scripts/pmc_step_summary.py $O/wide > $O/wide_summary.txt
cat $O/step_summary.txt $O/wide_summary.txt
