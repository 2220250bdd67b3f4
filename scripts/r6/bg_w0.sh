# The grouped backward (DNN_BWD_GROUP=1) with the A3/B2-ring W0 (code 11): A/B + trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd $R
rm -f gpurun_out/steps.txt
PREFIX=r6 MODELS=head REPS=4 step bgw0_ab 700 bash scripts/env_ab.sh bgw0 "DNN_BWD_GROUP=0" "DNN_BWD_GROUP=1" "DNN_BWD_GROUP=1 DNN_TUNED_TABLE=$R/bench/tables/r6/w0_code11.json" "DNN_TUNED_TABLE=$R/bench/tables/r6/w0_code11.json"
cd /tmp && export TMPDIR=/tmp
DNN_BWD_GROUP=1 DNN_TUNED_TABLE=$R/bench/tables/r6/w0_code11.json step trace_bgw0 120 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_bgw0 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5
