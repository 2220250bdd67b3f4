R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step w0_codes 300 python -u bench/probes/w0_codes.py
step wide_raster 300 python -u bench/probes/wide_raster.py
