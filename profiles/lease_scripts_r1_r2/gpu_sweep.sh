# GPU tests, then the tile sweep of the step GEMMs (and the 1024-wide / 8192-wide models).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > $O/tests.log 2>&1; rc=$?; echo "rc=$rc" >> $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench/stage_sweep.py > $O/sweep_fcnn.jsonl 2> $O/sweep.err || exit $?
timeout -k 10 600 python bench/stage_sweep.py --model 784-1024-1024-10 --iters 20 > $O/sweep_1024.jsonl 2>> $O/sweep.err || exit $?
timeout -k 10 600 python bench/stage_sweep.py --rows 16384 --model 784-8192-8192-10 --iters 10 > $O/sweep_8192.jsonl 2>> $O/sweep.err || exit $?
echo done >> $O/tests.log
