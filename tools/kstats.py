"""Summarise a rocprofv3 kernel trace: per (kernel, grid) class time share and average."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
agg = collections.defaultdict(lambda: [0, 0])
for r in rows:
    key = (r["Kernel_Name"].split("(")[0][:60], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])),
           int(r["Grid_Size_Y"]))
    agg[key][0] += 1
    agg[key][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
tot = sum(v[1] for v in agg.values())
print(f"total {tot / 1e6:.2f} ms")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:n]:
    print(f"{100 * v[1] / tot:5.1f}% {v[1] / 1e6:7.2f}ms {v[0]:4d} x {v[1] / v[0] / 1e3:8.1f}us  {k}")
