# Headline: fragment-order ReLU mask on the 512-wide layer (DNN_RELU_MASK=2) with the default
# overlap plan and with mode 5 (W1 then W0 on the main stream: fixed order).
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step mask_ab 600 env PREFIX=r6 MODELS=head REPS=3 bash $R/scripts/env_ab.sh mask "DNN_RELU_MASK=auto" "DNN_RELU_MASK=2" "DNN_RELU_MASK=2 DNN_BW_OVERLAP=5" "DNN_BW_OVERLAP=5"
