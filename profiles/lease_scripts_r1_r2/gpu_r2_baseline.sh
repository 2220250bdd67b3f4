# Round-2 starting point on a fresh box: GPU tests, the headline bench, and the three
# BASELINE configs with the library path forbidden (DNN_BLAS=0) plus kernel-trace profiles of
# the own-kernel steps. Output under gpurun_out/r2_base/.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_base; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1 || exit $?
b() { timeout -k 10 300 python bench.py "$@" >> $O/bench.jsonl 2>> $O/bench.err || exit $?; }
b --steps 50 --warmup 10
DNN_BLAS=0 b --steps 50 --warmup 10
DNN_BLAS=0 b --steps 20 --warmup 5 --model mlp8
b --steps 20 --warmup 5 --model mlp8
DNN_BLAS=0 b --steps 10 --warmup 3 --model wide --batch 16384
b --steps 10 --warmup 3 --model wide --batch 16384
cd /tmp && export TMPDIR=/tmp
p() { name=$1; shift; DNN_BLAS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$name \
  -o run --output-format csv -- python3 $R/bench.py "$@" > $O/$name.log 2>&1 || exit $?; }
p step --steps 20 --warmup 5
p mlp8 --model mlp8 --steps 10 --warmup 3
p wide --model wide --batch 16384 --steps 5 --warmup 2
echo done > $O/status.txt
