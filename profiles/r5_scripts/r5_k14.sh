R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_sched 700 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh sched "DNN_H0_DOUBLE=1" "DNN_FORK_ELIDE=1" "DNN_FORK_ELIDE=2" "DNN_MAIN_PRIORITY=1" "DNN_SIDE_PRIORITY=1" "DNN_SPLIT_FINO=0" "DNN_EVENT_FENCE=system"
