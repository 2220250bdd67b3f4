"""Summarise rocprofv3 --pmc CSV output: mean per dispatch of every counter, for kernels whose
name contains a substring. Usage: python scripts/pmc_summary.py DIR [substring]"""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "gemm"
out = {}
for d in sorted(glob.glob(f"{root}/*/")):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not files:
        continue
    acc = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if sub in row.get("Kernel_Name", ""):
                    acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    name = d.rstrip("/").split("/")[-1]
    out[name] = {k: round(sum(v) / len(v), 1) for k, v in sorted(acc.items())}
print(json.dumps(out, indent=1))
