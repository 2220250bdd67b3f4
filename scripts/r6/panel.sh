# 128x512 row-panel tiles for the headline's fwd 784->512 / dgrad 256->512: isolated probe, then
# whole-step A/B through table overrides.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
step panel_probe 200 python -u bench/probes/fwd_panel.py
grep -q cold_us gpurun_out/panel_probe.log || exit 1
T=$R/bench/tables/r6
PREFIX=r6 MODELS=head REPS=4 step panel_ab 700 bash scripts/env_ab.sh panel "DNN_TUNED=1" "DNN_TUNED_TABLE=$T/fwd0_128x512.json" "DNN_TUNED_TABLE=$T/dgrad1_128x512.json" "DNN_TUNED_TABLE=$T/both_128x512.json"
