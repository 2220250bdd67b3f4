# Kernel trace of the headline step with DNN_FORK_ELIDE=1 vs default -> gpurun_out/r3_elide/
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3_elide; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  DNN_FORK_ELIDE=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $O/e$v -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $O/e$v.log 2>&1 || exit $?
done
cd $R
for v in 0 1; do
python3 - $O/e$v/run_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'reduce_multi' in r['Kernel_Name']]
a, b = idx[-2], idx[-1]
t0 = int(rows[a]['End_Timestamp'])
for r in rows[a:b + 1]:
    s = (int(r['Start_Timestamp']) - t0) / 1e3; e = (int(r['End_Timestamp']) - t0) / 1e3
    print(f"{s:8.2f} {e:8.2f} q={r['Queue_Id']:>3} {r['Kernel_Name'][:60]}")
PY
echo ---
done
