R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step diag_host64 60 python -u $R/bench/probes/chain_stage_diag.py --wg 64 --ctl host
step diag_dev64 60 python -u $R/bench/probes/chain_stage_diag.py --wg 64 --ctl device
TB=$R/bench/tables/r5
step env_wtiles 900 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh wtiles "DNN_XSTEP=1" "DNN_TUNED_TABLE=$TB/w0_256x256_s32.json" "DNN_TUNED_TABLE=$TB/w0_256x256_s24.json" "DNN_TUNED_TABLE=$TB/w1_256x256_s32.json" "DNN_TUNED_TABLE=$TB/w1_256x256_s64.json" "DNN_FORK_ELIDE=1"
