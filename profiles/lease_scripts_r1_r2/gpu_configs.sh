# Every BASELINE config that fits one GPU: our bench (dp1 and loopback pipelines) and the
# torch-ROCm baseline of the same step; 8-stage batch-1 latency. Output: gpurun_out/configs.jsonl
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
: > $O/configs.jsonl
b() { timeout -k 10 300 python bench.py "$@" >> $O/configs.jsonl 2>> $O/configs.err || exit $?; }
t() { timeout -k 10 300 python bench/torch_baseline.py "$@" >> $O/configs.jsonl 2>> $O/configs.err || exit $?; }
b --steps 50 --warmup 10
b --steps 30 --warmup 5 --batch 131072
t --model mnist-fcnn --batch 65536
b --steps 20 --warmup 5 --parallelism pp4 --schedule 1f1b
b --steps 20 --warmup 5 --model mlp8
t --model mlp8 --batch 65536 --steps 20
b --steps 10 --warmup 3 --model mlp8 --parallelism pp8 --schedule 1f1b
b --steps 10 --warmup 3 --model wide --batch 16384
t --model wide --batch 16384 --steps 10
t --model mnist-784-128-10 --batch 65536
b --steps 50 --warmup 10 --model mnist-784-128-10
timeout -k 10 300 python bench/latency.py --iters 300 >> $O/configs.jsonl 2>> $O/configs.err || exit $?
echo done >> $O/configs.err
