# Alternating A/B of the persistent GEMM form for dgrad (and wide's wgrad) on mlp8 / wide,
# then kernel-trace profiles of the three BASELINE steps with the current build.
# -> gpurun_out/r2_persist_ab/{ab.jsonl, prof_*}
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_persist_ab; mkdir -p $O
cd $R
b() { tag=$1; shift; env $tag timeout -k 10 300 python bench.py --no-dp-compare "$@" \
  > $O/one.json 2>> $O/bench.err || exit $?
  python - "$tag" $O/one.json >> $O/ab.jsonl <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(json.dumps({"env": sys.argv[1], "model": d["config"]["model"], "ms": d["ms_per_step"]}))
EOF
}
for i in 1 2 3; do
  b DNN_X=0 --model mlp8 --steps 20 --warmup 5
  b DNN_GEMM_PERSIST=dgrad=1 --model mlp8 --steps 20 --warmup 5
  b DNN_X=0 --model wide --batch 16384 --steps 10 --warmup 3
  b DNN_GEMM_PERSIST=dgrad=1 --model wide --batch 16384 --steps 10 --warmup 3
  b DNN_GEMM_PERSIST=dgrad=1,wgrad=1 --model wide --batch 16384 --steps 10 --warmup 3
done
cat $O/ab.jsonl
cd /tmp && export TMPDIR=/tmp
p() { name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$name \
  -o run --output-format csv -- python3 $R/bench.py --no-dp-compare "$@" > $O/prof_$name.log 2>&1 || exit $?; }
p step --steps 20 --warmup 5
p mlp8 --model mlp8 --steps 10 --warmup 3
p wide --model wide --batch 16384 --steps 5 --warmup 2
cd $R
for n in step mlp8 wide; do python scripts/trace_summary.py $O/prof_$n/run_kernel_trace.csv --steps 3 > $O/prof_$n.summary.txt; done
echo done
