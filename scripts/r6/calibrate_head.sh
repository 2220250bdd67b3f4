# Re-calibrate the headline model's stage times after the micro-batch tuning.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
step cal_mnist-fcnn 600 python -u bench/planner_calibrate.py --models mnist-fcnn
