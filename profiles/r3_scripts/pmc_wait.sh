# Where the headline step's kernels wait: wave-cycle breakdown (parked in s_waitcnt/barrier vs
# issue-stalled vs issuing) and L2/TA load-path counters, one pass per group (kernel-trace +
# pmc only). -> gpurun_out/r3_pmc/<pass>/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3_pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" -d $O/$name -o run --output-format csv \
    -- python3 $R/bench.py --steps 3 --warmup 2 > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || exit $rc
}
run wait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
run l2 TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE
run inst SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE
echo done
