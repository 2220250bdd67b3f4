R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd $R
step graph_trace 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5_graph_trace -o run -- python3 bench.py --no-dp-compare --steps 20 --warmup 5 --graph on
