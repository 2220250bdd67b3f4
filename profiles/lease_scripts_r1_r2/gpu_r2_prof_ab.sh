# Kernel traces of the headline step with the old build (A, build_ab/_native_old.so) and the
# current tree (B).  Usage: bash scripts/gpu_r2_prof_ab.sh <tag> "<bench args>" -> gpurun_out/<tag>/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-prof_ab}; mkdir -p $O
ARGS=${2:-"--steps 20 --warmup 5"}
OLD=/tmp/ab_old_tree; rm -rf $OLD; mkdir -p $OLD
cd $R && tar --exclude=./gpurun_out --exclude=./build_ab -cf - . | (cd $OLD && tar xf -)
cp $R/build_ab/_native_old.so $OLD/docker_dist_nn_amd/_native.cpython-310-x86_64-linux-gnu.so
cd /tmp && export TMPDIR=/tmp
p() { name=$1; dir=$2; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$name \
  -o run --output-format csv -- python3 $dir/bench.py --no-dp-compare $ARGS > $O/$name.log 2>&1 || exit $?; }
p A $OLD
p B $R
cd $R
for n in A B; do python scripts/trace_summary.py $O/$n/run_kernel_trace.csv --steps 3 > $O/$n.summary.txt; tail -14 $O/$n.summary.txt; done
