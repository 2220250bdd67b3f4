"""Per-DISPATCH derived metrics of one training step from a PMC run (scripts/pmc_step.sh):
HBM read/write MB (FETCH_SIZE / WRITE_SIZE, KiB units), MFMA busy share of the kernel's GPU
cycles, LDS bank-conflict share of LDS cycles, duration.

Rows are keyed by the kernel's POSITION in the step (dispatch order), not by name + grid: the
headline step's fwd 784->512 and dgrad 256->512 are the same kernel with the same grid and
used to be merged into one row. The step period is found as the shortest
repeating suffix of the dispatch-name sequence; each position is averaged over the last
``--steps`` periods of every pass. Usage:
    python scripts/pmc_step_summary.py gpurun_out/pmc_step [--steps 2]

Calibration (MI355X, measured): SQ_VALU_MFMA_BUSY_CYCLES = MFMA instructions x 16 summed over
all SIMDs; GRBM_GUI_ACTIVE counts GPU cycles summed over the 8 XCDs. MFMA% = busy / (cycles/8 x
1024 SIMDs) = the kernel's share of the dense bf16 MFMA peak at the clock it ran."""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name)
    name = name.replace("gemm_bf16_kernel<", "gemm<").replace("dnn::", "")
    return name[:60]


def load_pass(d):
    """{dispatch id: (name, grid, {counter: value}, us)} of one pass directory."""
    cnt = defaultdict(dict)
    meta = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                i = int(r["Dispatch_Id"])
                cnt[i][r["Counter_Name"]] = cnt[i].get(r["Counter_Name"], 0.0) + \
                    float(r["Counter_Value"])
                meta[i] = (r["Kernel_Name"], r.get("Grid_Size", r.get("Grid_Size_X", "")))
    dur = {}
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                i = int(r["Dispatch_Id"])
                dur[i] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                if i not in meta:
                    meta[i] = (r["Kernel_Name"], r.get("Grid_Size_X", r.get("Grid_Size", "")))
    return {i: (meta[i][0], meta[i][1], cnt.get(i, {}), dur.get(i, 0.0)) for i in sorted(meta)}


def period(names, max_p=200, max_tail=8):
    """(p, t): the shortest p such that, after dropping the last t dispatches (end-of-run work
    such as the final loss read-back), the last 2p names are two copies of one period."""
    for p in range(2, min(max_p, len(names) // 2) + 1):
        for t in range(0, max_tail + 1):
            body = names[:len(names) - t]
            if len(body) >= 2 * p and body[-p:] == body[-2 * p:-p]:
                return p, t
    return len(names), 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(list))
    names_of = {}
    p_seen = None
    for pas in sorted(os.listdir(a.root)):
        d = os.path.join(a.root, pas)
        if not os.path.isdir(d):
            continue
        disp = load_pass(d)
        if not disp:
            continue
        ids = list(disp)
        names = [disp[i][0] for i in ids]
        p, t = period(names)
        p_seen = p
        ids = ids[:len(ids) - t]
        last = ids[-p * a.steps:]
        for k, i in enumerate(last):
            pos = k % p
            name, grid, c, us = disp[i]
            names_of[pos] = (name, grid)
            acc[pos]["us"].append(us)
            for cn, v in c.items():
                acc[pos][cn].append(v)
    print(f"step period: {p_seen} dispatches; averaged over the last {a.steps} steps")
    print(f"{'#':>3s} {'kernel':60s} {'grid':>8s} {'us':>7s} {'rd MB':>7s} {'wr MB':>7s} "
          f"{'TB/s':>6s} {'MFMA%':>6s} {'LDSc%':>6s}")
    tot = 0.0
    for pos in sorted(acc):
        m = {k: sum(v) / len(v) for k, v in acc[pos].items() if v}
        name, grid = names_of[pos]
        us = sorted(acc[pos]["us"])[len(acc[pos]["us"]) // 2] if acc[pos]["us"] else 0.0
        tot += us
        rd = m.get("FETCH_SIZE", 0) / 1024
        wr = m.get("WRITE_SIZE", 0) / 1024
        bw = (rd + wr) / us if us else 0  # MB/us = TB/s
        cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
        mf = 100 * m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1.0, cyc * 1024)
        lc = 100 * m.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, m.get("SQ_LDS_IDX_ACTIVE", 1))
        print(f"{pos:3d} {short(name):60s} {grid:>8s} {us:7.1f} {rd:7.1f} {wr:7.1f} {bw:6.2f} "
              f"{mf:6.1f} {lc:6.2f}")
    print(f"sum of kernel durations (profiled, serialised): {tot:.1f} us")


if __name__ == "__main__":
    main()
