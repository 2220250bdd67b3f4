R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_elide_md 900 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh elide_md "DNN_BW_OVERLAP=1" "DNN_FORK_ELIDE=1" "DNN_FORK_ELIDE=1 DNN_DIAG_MAIN_DELAY_US=5" "DNN_FORK_ELIDE=1 DNN_DIAG_MAIN_DELAY_US=9" "DNN_FORK_ELIDE=1 DNN_DIAG_MAIN_DELAY_US=15"
