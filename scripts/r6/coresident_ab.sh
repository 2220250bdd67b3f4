# Side-stream wgrads with 32-KiB LDS tiles (co-resident with the 128-KiB dgrad workgroups)
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
T=$R/bench/tables/r6
step cores_ab 900 env PREFIX=r6 MODELS=head REPS=3 bash $R/scripts/env_ab.sh cores "DNN_TUNED=1" "DNN_TUNED_TABLE=$T/w1_64_s16.json" "DNN_TUNED_TABLE=$T/w1_64_s8.json" "DNN_TUNED_TABLE=$T/w1_64_s16_w2_64_s32.json"
