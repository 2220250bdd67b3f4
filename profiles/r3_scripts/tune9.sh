# In-step re-tune with the register-prefetched forms (codes 9 / 6 / 2, one-tile) starting from
# the current table -> bench/tables/table_tune9.json (+ log), then whole-step A/B vs current.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3_tune9; mkdir -p $O
cd $R
timeout -k 10 900 python bench/tune.py --configs ${CONFIGS:-65536:mnist-fcnn,65536:mlp8,16384:wide} --stages 9,6,2 --persist 0 \
  --tiles 256x256,256x128,128x128,128x64,64x64 --out bench/tables/table_tune9.json > $O/tune.jsonl 2> $O/tune.err || { tail -20 $O/tune.err; exit 1; }
cp bench/tables/table_tune9.json $O/
grep -E '"(sig|rows)"' $O/tune.jsonl | tail -40
bash scripts/r3/ab_table.sh bench/tables/table_tune9.json tune9
