"""Summarise rocprofv3 --pmc CSVs (run_counter_collection.csv) per kernel name."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "zfp" not in name:
            continue
        short = name.split("(")[0].replace("void cuzfp::", "")
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        # median over dispatches
        v = sorted(v)
        print(f"   {c:24s} {v[len(v) // 2]:16.4g}   (n={len(v)})")
