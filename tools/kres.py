"""Per-kernel register / spill / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage
output on stdin (developer tool): python tools/kres.py [REGEX] < remarks.txt"""
import re
import subprocess
import sys

pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Name: (\S+)", line)
    if m:
        name = m.group(1)
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        cur = {"name": name}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "VGPRs Spill", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        m = re.search(r"\s" + key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split(" ")[0] + ("_spill" if "Spill" in key else "")] = int(m.group(1))
for r in rows:
    if pat and not pat.search(r["name"]):
        continue
    print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>4} a spill {r.get('VGPRs_spill', '?'):>4} "
          f"occ {r.get('Occupancy', '?')}  {r['name'][:110]}")
