"""Summarise rocprofv3 --pmc CSVs per kernel (average per dispatch)."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
filt = sys.argv[2:] or None
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:48]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[k]["VGPR"].append(float(r["VGPR_Count"]))
for k, d in agg.items():
    if filt and not any(s in k for s in filt):
        continue
    avg = {c: sum(v) / len(v) for c, v in d.items()}
    line = " ".join(f"{c}={avg[c]:.4g}" for c in sorted(avg))
    print(k, "\n   ", line)
