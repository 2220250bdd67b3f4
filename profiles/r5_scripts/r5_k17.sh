R=${GRAFT_REPO_ROOT:-$(pwd)}
source $R/scripts/gpu_steps.sh
step blas_wide 400 python -u $R/bench/gemm_vs_blas.py --model 784-8192-8192-10 --rows 16384
step blas_mlp8 400 python -u $R/bench/gemm_vs_blas.py --model 784-1024-1024-1024-1024-1024-1024-1024-10 --rows 65536
step blas_head 300 python -u $R/bench/gemm_vs_blas.py
