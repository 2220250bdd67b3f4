# Single-process pipelines (all stages on one GPU): micro-batch size x schedule for pp4 and
# pp8 (mlp8) at a 65536-row step. -> gpurun_out/r2_lb3/ab.jsonl
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_lb3; mkdir -p $O
cd $R
b() { tag=$1; shift; timeout -k 10 200 python bench.py "$@" > $O/one.json 2>> $O/bench.err || exit $?
  python - "$tag" $O/one.json >> $O/ab.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
c = d["config"]
print(json.dumps({"tag": sys.argv[1], "model": c["model"], "par": c["parallelism"],
                  "micro": c["micro_batch"], "nm": c["num_micro"], "schedule": c["schedule"],
                  "ms": d["ms_per_step"]}))
PY
}
for i in 1 2; do
  for m in 8192 16384; do
    for s in 1f1b gpipe; do
      b pp4 --parallelism pp4 --micro $m --schedule $s --steps 30 --warmup 5
    done
  done
  for m in 8192 16384; do
    b pp8 --model mlp8 --parallelism pp8 --micro $m --schedule 1f1b --steps 10 --warmup 3
  done
done
cat $O/ab.jsonl
