# Planner calibration (bench/planner_calibrate.py): stage-replica step times per model.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
mkdir -p $R/gpurun_out/r6_planner
for m in mnist-fcnn wide mlp8; do
  step cal_$m 420 python -u $R/bench/planner_calibrate.py --models $m
  cp $R/gpurun_out/cal_$m.log $R/gpurun_out/r6_planner/stage_times_$m.jsonl
done
