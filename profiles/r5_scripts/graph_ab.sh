# Alternating headline A/B: eager native plan vs the step replayed as a HIP graph (--graph on).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r5_graph; mkdir -p $O; cd $R
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-dp-compare --steps 50 --warmup 10 | sed "s/^/eager /" >> $O/ab.txt || exit 1
  timeout -k 10 200 python bench.py --no-dp-compare --steps 50 --warmup 10 --graph on | sed "s/^/graph /" >> $O/ab.txt || exit 1
done
