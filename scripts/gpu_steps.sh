# Helper for a batch of GPU steps in one gpurun call: source it, then
#   step NAME SECONDS cmd args...   (output -> gpurun_out/NAME.log)
# A step that times out, aborts or crashes (rc 124/134/137/139 or any signal) ends the batch:
# nothing else touches the GPU after a fault. A plain failure (e.g. a failing test, rc 1) is
# recorded and the batch goes on. Status lines -> gpurun_out/steps.txt.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > $R/gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a $R/gpurun_out/steps.txt
  if [ $rc -ge 124 ]; then
    echo "stopping the batch after $name (rc $rc)" | tee -a $R/gpurun_out/steps.txt
    exit $rc
  fi
  return 0
}
