"""Summarise a rocprofv3 --kernel-trace CSV of a training run: the last complete step as a
timeline (duration, gap to the previous kernel, grid, VGPR/AGPR, LDS) and per-kernel totals per
step over the last N steps. A step ends with the kernel whose name contains --end (default:
reduce_multi, the fused gradient reduction + SGD of the native plan).

Usage: python scripts/trace_summary.py run_kernel_trace.csv [--steps 10] [--end reduce_multi]"""
import argparse
import csv
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("void ", "").replace("dnn::", "")
    return n[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--end", default="reduce_multi")
    ap.add_argument("--end-grid", type=int, default=None)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])),
                         r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"]))
    rows.sort()
    # --end-grid: with the split reduction (DNN_SPLIT_FINO) a step has two reduce_multi
    # launches; the main stream's last one (layer 0's) is picked by its grid
    ends = [i for i, r in enumerate(rows)
            if a.end in r[2] and (a.end_grid is None or r[3] == a.end_grid)]
    if len(ends) < 2:
        raise SystemExit("fewer than two step ends found")
    n = min(a.steps, len(ends) - 1)
    per = defaultdict(float)
    calls = defaultdict(int)
    for k in range(len(ends) - n, len(ends)):
        for r in rows[ends[k - 1] + 1:ends[k] + 1]:
            per[short(r[2])] += (r[1] - r[0]) / 1e3 / n
            calls[short(r[2])] += 1
    lo, hi = ends[-2] + 1, ends[-1] + 1
    print("last step timeline (us):")
    prev_end = rows[lo - 1][1]
    for r in rows[lo:hi]:
        print(f"  {(r[1] - r[0]) / 1e3:8.2f}  gap {(r[0] - prev_end) / 1e3:6.2f}  grid {r[3]:6d}  "
              f"vgpr {r[4]:>3} agpr {r[5]:>3} lds {r[6]:>6}  {short(r[2])}")
        prev_end = r[1]
    print(f"step span {(rows[hi - 1][1] - rows[lo - 1][1]) / 1e3:.1f} us "
          f"(end of previous step to end of this one)")
    print(f"\nper-step kernel time over the last {n} steps:")
    tot = sum(per.values())
    for name, us in sorted(per.items(), key=lambda kv: -kv[1]):
        print(f"  {us:8.2f} us  {calls[name] / n:4.1f} calls  {100 * us / tot:5.1f} %  {name}")
    print(f"  {tot:8.2f} us  total")


if __name__ == "__main__":
    main()
