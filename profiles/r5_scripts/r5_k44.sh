R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_mdelay 900 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh mdelay "DNN_BW_OVERLAP=1" "DNN_MAIN_DELAY_US=1" "DNN_MAIN_DELAY_US=5" "DNN_MAIN_DELAY_US=10" "DNN_MAIN_DELAY_US=20"
