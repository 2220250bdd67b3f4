"""Per-kernel duration versus step index from a rocprofv3 kernel trace of bench.py (the step
"ramp" question).

Usage: python scripts/ramp_summary.py TRACE.csv [--period P] [--steps N]

The last N*P dispatches are cut into N steps of P dispatches (the step's kernel sequence must
repeat exactly; checked). Prints, per dispatch position, the mean duration over steps in blocks
of 10 (first block = the first timed steps), plus the step span (start of the step's first
kernel to the end of its last) and the sum of kernel durations per block. If every position
slows or speeds up by the same factor, the ramp is the clock; if one position or the gaps
drift, it is that kernel or the engine.
"""
from __future__ import annotations

import argparse
import csv
import statistics as st


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r["Grid_Size_X"])))
    rows.sort()
    return rows


def short(name: str) -> str:
    n = name.replace("void ", "").replace("dnn::", "")
    return n.split("(")[0][:60]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--period", type=int, default=10)
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--block", type=int, default=10)
    a = ap.parse_args(argv)
    rows = load(a.trace)
    P, N = a.period, a.steps
    rows = rows[-(N + 1) * P:]
    # a step starts at the dispatch whose (name, grid) is the first kernel of the step's
    # sequence: the most common (name, grid) among the dispatches that follow the largest
    # idle gap before it (the host's step boundary)
    starts = [i for i in range(1, len(rows)) if rows[i][0] - rows[i - 1][1] > 0]
    first = max(set((rows[i][2], rows[i][3]) for i in starts),
                key=lambda k: sum(1 for i in starts if (rows[i][2], rows[i][3]) == k))
    idx = [i for i, r in enumerate(rows) if (r[2], r[3]) == first]
    steps = [rows[idx[i]:idx[i + 1]] for i in range(len(idx) - 1)][-N:]
    # concurrent kernels may dispatch in either order: key each by (name, grid, occurrence)
    def keyed(s):
        seen, out = {}, {}
        for r in s:
            k = (r[2], r[3]); n = seen.get(k, 0); seen[k] = n + 1
            out[(k[0], k[1], n)] = r
        return out
    ks = [keyed(s) for s in steps]
    sig = sorted(ks[0], key=lambda k: ks[0][k][0])
    bad = sum(1 for k in ks if set(k) != set(sig))
    N = len(steps)
    print(f"{N} steps; {bad} steps deviate from the first step's kernel set")
    steps = [[k[s] for s in sig] for k in ks]
    P = len(sig)
    nb = N // a.block
    hdr = "pos  kernel" + "".join(f"  b{b:02d}" for b in range(nb)) + "   last/first"
    print(hdr)
    for p in range(P):
        means = []
        for b in range(nb):
            ds = [(s[p][1] - s[p][0]) / 1000 for s in steps[b * a.block:(b + 1) * a.block]]
            means.append(st.mean(ds))
        print(f"{p:3d}  {short(sig[p][0]):60s} g{sig[p][1] // 256:5d}" +
              "".join(f" {m:5.1f}" for m in means) + f"   {means[-1] / means[0]:.3f}")
    spans, sums = [], []
    for b in range(nb):
        blk = steps[b * a.block:(b + 1) * a.block]
        spans.append(st.mean((max(r[1] for r in s) - s[0][0]) / 1000 for s in blk))
        sums.append(st.mean(sum(r[1] - r[0] for r in s) / 1000 for s in blk))
    print("span " + " ".join(f"{x:6.1f}" for x in spans) + f"   {spans[-1] / spans[0]:.3f}")
    print("sum  " + " ".join(f"{x:6.1f}" for x in sums) + f"   {sums[-1] / sums[0]:.3f}")
    # step-to-step period (start to start) per block
    per = []
    for b in range(nb):
        blk = steps[b * a.block:(b + 1) * a.block + 1]
        ds = [(blk[i + 1][0][0] - blk[i][0][0]) / 1000 for i in range(len(blk) - 1)]
        per.append(st.mean(ds))
    print("per  " + " ".join(f"{x:6.1f}" for x in per) + f"   {per[-1] / per[0]:.3f}")


if __name__ == "__main__":
    main()
