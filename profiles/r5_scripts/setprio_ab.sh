# A/B of the s_setprio builds of the GEMM main loop (DNN_GEMM_SETPRIO=1 per-cluster, =2 static
# younger-half) against the product build: per-GEMM times (bench/gemm_vs_blas.py) and the three
# model steps, variants alternated. Usage: setprio_ab.sh REP (one pass over the variants)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r5_setprio; mkdir -p $O; cd $R
SO=docker_dist_nn_amd/_native.cpython-310-x86_64-linux-gnu.so
[ -f bench/ab/_native_product.so ] || cp $SO bench/ab/_native_product.so
M8=784-1024-1024-1024-1024-1024-1024-1024-10
for v in product setprio1 setprio2; do
  cp bench/ab/_native_$v.so $SO || exit 1
  if [ "$1" = 1 ]; then
    timeout -k 10 200 python bench/gemm_vs_blas.py --model 784-8192-8192-10 --rows 16384 --iters 10 | sed "s/^/$v wide /" >> $O/gemm.txt || exit 1
    timeout -k 10 200 python bench/gemm_vs_blas.py --model $M8 | sed "s/^/$v mlp8 /" >> $O/gemm.txt || exit 1
    timeout -k 10 200 python bench/gemm_vs_blas.py | sed "s/^/$v head /" >> $O/gemm.txt || exit 1
  fi
  timeout -k 10 200 python bench.py --no-dp-compare | sed "s/^/$v head /" >> $O/bench.txt || exit 1
  timeout -k 10 200 python bench.py --no-dp-compare --model mlp8 | sed "s/^/$v mlp8 /" >> $O/bench.txt || exit 1
  timeout -k 10 200 python bench.py --no-dp-compare --model wide --batch 16384 | sed "s/^/$v wide /" >> $O/bench.txt || exit 1
done
cp bench/ab/_native_product.so $SO
