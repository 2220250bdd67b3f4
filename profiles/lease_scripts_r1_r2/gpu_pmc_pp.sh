# PMC A/B: one-tile 256x256 (stages 2) vs ping-pong (stages 8) on the wide fwd GEMM.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc_pp; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
run() {
  local name=$1 pass=$2; shift 2
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pass -d $O/$name -o run --output-format csv \
    -- python3 $R/bench/one_gemm.py "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/status.txt
  [ $rc -le 1 ] || exit $rc
}
for cfg in "s2:--op fwd --M 16384 --K 8192 --N 8192 --tile 256x256 --stages 2 --iters 5" \
           "s8:--op fwd --M 16384 --K 8192 --N 8192 --tile 256x256 --stages 8 --iters 5"; do
  name=${cfg%%:*}; args=${cfg#*:}
  run ${name}_p1 "$P1" $args
  run ${name}_p2 "$P2" $args
done
echo done >> $O/status.txt
