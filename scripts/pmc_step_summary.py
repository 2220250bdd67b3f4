"""Per-kernel derived metrics of the headline step from scripts/gpu_pmc_step.sh output:
HBM read/write MB (FETCH_SIZE / WRITE_SIZE, KiB units), MFMA busy share of the kernel's GPU
cycles, LDS bank-conflict share of LDS cycles. Kernels are keyed by name + grid, averaged over
dispatches. Usage: python scripts/pmc_step_summary.py gpurun_out/pmc_step

Calibration (MI355X, measured): SQ_VALU_MFMA_BUSY_CYCLES = MFMA instructions x 16 summed over
all SIMDs; GRBM_GUI_ACTIVE counts GPU cycles summed over the 8 XCDs. MFMA% = busy / (cycles/8 x
1024 SIMDs) = the kernel's share of the dense bf16 MFMA peak at the clock it ran.
FETCH_SIZE / WRITE_SIZE are KiB."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for pas in ("sq", "fetch", "write"):
    for f in glob.glob(f"{root}/{pas}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                key = (r["Kernel_Name"][:70], r.get("Grid_Size", r.get("Grid_Size_X", "")))
                vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(f"{root}/{pas}/**/*kernel_trace.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                key = (r["Kernel_Name"][:70], r.get("Grid_Size_X", ""))
                dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

print(f"{'kernel':72s} {'grid':>8s} {'us':>7s} {'rd MB':>7s} {'wr MB':>7s} {'TB/s':>6s} "
      f"{'MFMA%':>6s} {'LDSc%':>6s}")
for key, c in sorted(vals.items(), key=lambda kv: kv[0][0]):
    if not any(t in key[0] for t in ("gemm", "reduce", "sgd", "mlp_tail", "Cijk", "colsum")):
        continue
    m = {k: sum(v) / len(v) for k, v in c.items()}
    us = dur.get(key) or dur.get((key[0], ""), [0.0])
    us = sorted(us)[len(us) // 2] if us else 0.0
    rd = m.get("FETCH_SIZE", 0) / 1024
    wr = m.get("WRITE_SIZE", 0) / 1024
    bw = (rd + wr) / us if us else 0  # MB/us = TB/s
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    mf = 100 * m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1.0, cyc * 1024)
    lc = 100 * m.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, m.get("SQ_LDS_IDX_ACTIVE", 1))
    print(f"{key[0]:72s} {key[1]:>8s} {us:7.1f} {rd:7.1f} {wr:7.1f} {bw:6.2f} {mf:6.1f} {lc:6.2f}")
