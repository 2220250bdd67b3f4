# In-step re-tune of every GEMM of the three BASELINE training configs on OWN kernels only
# (no hipBLASLt candidates; transposed-weight dgrad; persistent forms with overlapped
# epilogues), then an alternating A/B of the new table against the old table with the library
# path stripped. Output: gpurun_out/retune/{tuned.json,tune.jsonl,ab.jsonl}
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/retune; mkdir -p $O
cd $R
OLD=$O/old_stripped.json; NEW=$O/tuned.json
python - docker_dist_nn_amd/ops/tuned_gfx950.json $OLD <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for e in d["entries"].values():
    e.pop("blas", None); e.pop("blas_algo", None)
json.dump(d, open(sys.argv[2], "w"), indent=1, sort_keys=True)
PY
cp $OLD $NEW
export DNN_TUNED_TABLE=$NEW
timeout -k 10 900 python -u bench/tune.py --configs ${CONFIGS:-65536:mnist-fcnn,65536:mlp8,16384:wide} \
  --blas 0 --persist 0,1 --verbose --out $NEW > $O/tune.jsonl 2>&1 || exit 1
: > $O/ab.jsonl
for m in "mnist-fcnn 65536 40" "mlp8 65536 10" "wide 16384 6"; do
  set -- $m
  for t in A B A B; do
    if [ $t = B ]; then export DNN_TUNED_TABLE=$NEW; else export DNN_TUNED_TABLE=$OLD; fi
    timeout -k 10 150 python bench.py --model $1 --batch $2 --steps $3 --warmup 5 > $O/one.json 2>>$O/err.log || exit 1
    python -c "import json;d=json.load(open('$O/one.json'));print(json.dumps({'model':'$1','table':'$t','ms':d['ms_per_step']}))" >> $O/ab.jsonl
  done
done
cat $O/ab.jsonl
