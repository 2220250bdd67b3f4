# The reference's own training recipes at their batch sizes: ours (eager native / HIP graph)
# vs PyTorch-ROCm on the same GPU. Output: gpurun_out/recipes.jsonl
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
: > $O/recipes.jsonl
b() { timeout -k 10 300 python bench.py "$@" >> $O/recipes.jsonl 2>> $O/recipes.err || exit $?; }
t() { timeout -k 10 300 python bench/torch_baseline.py "$@" >> $O/recipes.jsonl 2>> $O/recipes.err || exit $?; }
b --model pytorch-recipe --batch 64 --optimizer adam --lr 0.001 --steps 500 --warmup 50
b --model pytorch-recipe --batch 64 --optimizer adam --lr 0.001 --steps 500 --warmup 50 --graph
t --model pytorch-recipe --batch 64 --optimizer adam --steps 300 --warmup 30
b --model notebook --batch 64 --optimizer adam --lr 0.001 --steps 500 --warmup 50 --graph
t --model notebook --batch 64 --optimizer adam --steps 300 --warmup 30
b --model mnist-fcnn --batch 4096 --steps 200 --warmup 20
b --model mnist-fcnn --batch 4096 --steps 200 --warmup 20 --graph
t --model mnist-fcnn --batch 4096 --steps 200 --warmup 20
echo done >> $O/recipes.err
