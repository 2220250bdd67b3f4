# PMC counters of every kernel of the headline training step (bench.py, 1 GPU), one pass per
# counter group (kernel-trace + pmc only). Output: gpurun_out/pmc_step/<pass>/...
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r3_pmc_step}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $O/$name -o run --output-format csv \
    -- python3 $R/bench.py --steps 3 --warmup 2 > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || exit $rc
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
echo done >> $O/status.txt
python $R/scripts/pmc_step_summary.py $O > $O/summary.txt
cat $O/summary.txt
