R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd $R
export DNN_FORK_ELIDE=1
step elide_trace 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5_elide_trace -o run -- python3 bench.py --no-dp-compare --steps 30 --warmup 10
unset DNN_FORK_ELIDE
step default_trace 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5_default_trace -o run -- python3 bench.py --no-dp-compare --steps 30 --warmup 10
