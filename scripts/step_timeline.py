"""Absolute timeline of the last complete steps of a rocprofv3 --kernel-trace CSV: every kernel
of a step with its start / end offset from the step's first kernel (us), so main-stream gaps
(event packets, dependencies) and side-stream overlap can be read directly. A step begins with
the first kernel whose grid matches --first-grid after a kernel whose grid matches --end-grid.

Usage: python scripts/step_timeline.py trace.csv [--steps 3] [--end-grid 424] [--first-grid 512]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--end-grid", type=int, default=424)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            g = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), g,
                         r["Kernel_Name"].replace("void ", "").replace("dnn::", "")[:70]))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if r[2] == a.end_grid and "reduce" in r[3]]
    for k in range(max(1, len(ends) - a.steps), len(ends)):
        lo, hi = ends[k - 1] + 1, ends[k] + 1
        t0 = rows[lo][0]
        print(f"--- step ending at kernel {hi - 1}: span {(rows[hi - 1][1] - rows[ends[k - 1]][1]) / 1e3:.1f} us")
        for s, e, g, n in rows[lo:hi]:
            print(f"  {(s - t0) / 1e3:7.1f} -> {(e - t0) / 1e3:7.1f}  ({(e - s) / 1e3:6.1f})  grid {g:4d}  {n}")


if __name__ == "__main__":
    main()
