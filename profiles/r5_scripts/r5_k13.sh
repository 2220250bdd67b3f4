R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step env_h0b 700 env PREFIX=r5 MODELS=head,mlp8,wide REPS=5 bash $R/scripts/env_ab.sh h0b "DNN_H0_DOUBLE=0" "DNN_H0_DOUBLE=1"
step wide_a 300 python -u $R/bench.py --model wide --batch 16384
step wide_b 300 env DNN_H0_DOUBLE=1 python -u $R/bench.py --model wide --batch 16384
