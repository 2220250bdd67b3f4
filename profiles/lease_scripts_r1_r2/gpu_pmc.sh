# PMC counters of single GEMM configurations (kernel-trace + pmc only; no sys/runtime traces).
# Each rocprofv3 step is time-limited; a step that fails for a reason other than a clean
# counter-selection error (rc 1) ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE GRBM_COUNT"
run() {  # name, pass counters, gemm args...
  local name=$1 pass=$2; shift 2
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $pass -d $O/$name -o run --output-format csv \
    -- python3 $R/bench/one_gemm.py "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/status.txt
  [ $rc -le 1 ] || exit $rc
}
for cfg in "fwd128:--op fwd --tile 128x128" "fwd64x128:--op fwd --tile 64x128" \
           "wgrad:--op wgrad --tile 128x64 --splits 10" "dgrad:--op dgrad --K 512 --N 256 --tile 64x64"; do
  name=${cfg%%:*}; args=${cfg#*:}
  run ${name}_p1 "$P1" $args
  run ${name}_p2 "$P2" $args
done
echo done >> $O/status.txt
