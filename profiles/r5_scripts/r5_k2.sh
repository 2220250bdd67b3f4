R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step fan_gpu 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread $R/tests/test_fan_gpu.py
step overlap_gpu 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread $R/tests/test_overlap_gpu.py
step env_xstep 600 env PREFIX=r5 MODELS=head,mlp8 REPS=3 bash $R/scripts/env_ab.sh xfence "DNN_XSTEP=0 DNN_EVENT_FENCE=system" "DNN_XSTEP=0 DNN_EVENT_FENCE=device" "DNN_XSTEP=1 DNN_EVENT_FENCE=device"
step tl_cold 200 python -u $R/bench/probes/gemm_timeline.py --cold --cases f0,f1,d1,w0 --variants 256x256:9,256x256:11 --wvariants 128x128:9,128x128:11
mkdir -p $R/gpurun_out/r5_ramp_clk
cd /tmp && export TMPDIR=/tmp
step ramp_clk 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $R/gpurun_out/r5_ramp_clk -o clk --output-format csv -- python3 $R/bench.py --steps 120 --warmup 5
