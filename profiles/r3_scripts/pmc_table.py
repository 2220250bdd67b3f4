"""Per-kernel table of arbitrary rocprofv3 --pmc passes: median duration and the mean of every
counter per (kernel, grid), plus derived wave-cycle shares when the SQ wait counters are there.
Usage: python scripts/r3/pmc_table.py gpurun_out/r3_pmc [pass ...]"""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
passes = sys.argv[2:] or sorted(p.split("/")[-1] for p in glob.glob(f"{root}/*") if "." not in p.split("/")[-1])
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for pas in passes:
    for f in glob.glob(f"{root}/{pas}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"].replace("void ", "").replace("dnn::", "")[:58], r.get("Grid_Size", ""))
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(f"{root}/{pas}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"].replace("void ", "").replace("dnn::", "")[:58], r.get("Grid_Size_X", ""))
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
names = sorted({c for v in vals.values() for c in v})
for key, c in sorted(vals.items()):
    if not any(t in key[0] for t in ("gemm", "reduce", "mlp_tail")):
        continue
    m = {k: sum(v) / len(v) for k, v in c.items()}
    us = dur.get(key, [0.0])
    us = sorted(us)[len(us) // 2]
    print(f"{key[0]} grid={key[1]} us={us:.1f}")
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        print("   wave-cycle shares: wait(waitcnt/barrier) {:.0%}  issue-stall {:.0%}  active {:.0%}  "
              "lds-issue-stall {:.0%}".format(m.get("SQ_WAIT_ANY", 0) / wc, m.get("SQ_WAIT_INST_ANY", 0) / wc,
                                              m.get("SQ_ACTIVE_INST_ANY", 0) / wc, m.get("SQ_WAIT_INST_LDS", 0) / wc))
    if m.get("TCC_HIT_sum") is not None:
        h, mi = m["TCC_HIT_sum"], m.get("TCC_MISS_sum", 0)
        print(f"   L2 hit {h / max(1, h + mi):.0%}")
    print("   " + "  ".join(f"{k}={m[k]:.3g}" for k in names if k in m))
