# PMC stall breakdown of the big-GEMM tiles (kernel-trace + pmc only).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc_big; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
run() {
  local name=$1 pass=$2; shift 2
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $pass -d $O/$name -o run --output-format csv \
    -- python3 $R/bench/one_gemm.py "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/status.txt
  [ $rc -le 1 ] || exit $rc
}
for cfg in "f256:--op fwd --M 16384 --K 8192 --N 8192 --tile 256x256 --iters 5" \
           "f128:--op fwd --M 16384 --K 8192 --N 8192 --tile 128x128 --iters 5" \
           "d256:--op dgrad --M 16384 --K 8192 --N 8192 --tile 256x256 --iters 5"; do
  name=${cfg%%:*}; args=${cfg#*:}
  run ${name}_p1 "$P1" $args
  run ${name}_p2 "$P2" $args
  run ${name}_p3 "$P3" $args
done
echo done >> $O/status.txt
