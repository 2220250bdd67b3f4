set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench/tune.py --configs 65536:mnist-fcnn --only wgrad:512x832x65536 --verbose --out gpurun_out/t.json > gpurun_out/tune_v.log 2>&1
