R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step ldsdma 300 python -u $R/bench/probes/ldsdma_rate.py
step env_w0tile 700 env PREFIX=r5 MODELS=head REPS=3 bash $R/scripts/env_ab.sh w0tile "DNN_XSTEP=1" "DNN_XSTEP=1 DNN_TUNED_TABLE=$R/profiles/r5_tables/w0_256x128_9.json" "DNN_XSTEP=1 DNN_TUNED_TABLE=$R/profiles/r5_tables/w0_256x128_11.json" "DNN_XSTEP=1 DNN_RELU_MASK=2"
