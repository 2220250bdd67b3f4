# HIP runtime environment A/B on the headline step (kernel arguments in device memory, more
# hardware queues).
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
PREFIX=r6 MODELS=head REPS=4 step hipenv_ab 700 bash scripts/env_ab.sh hipenv "DNN_XSTEP=1" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "GPU_MAX_HW_QUEUES=8"
