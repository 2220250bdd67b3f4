# One GPU-box session: tests, smoke, bench variants (A/B), multi-rank rehearsal (gloo ranks
# sharing cuda:0), latency, rocprofv3 kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests/ -q -m gpu > $O/tests.log 2>&1; rc=$?; echo "rc=$rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
: > $O/bench_sweep.log
for args in "" "--batch 131072"; do
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 $args >> $O/bench_sweep.log 2>&1 || exit $?
done
: > $O/rehearsal.log
for par in dp2 pp2; do
  DNN_DIST_BACKEND=gloo DNN_FORCE_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 5 --warmup 2 --batch 8192 --parallelism $par >> $O/rehearsal.log 2>&1 || exit $?
done
timeout -k 10 300 python bench/latency.py --iters 300 > $O/latency.log 2>&1 || exit $?
echo done >> $O/tests.log
