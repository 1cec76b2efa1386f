"""Aggregate rocprofv3 --pmc CSVs (gpurun_out/pmc/p*/run_counter_collection.csv) per kernel."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0][:48]
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    if "rocclr" in k or "elementwise" in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"    {c:32s} mean/launch {sum(v) / len(v):14.1f}  (n={len(v)})")
