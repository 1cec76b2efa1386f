"""One-line summary of bench.py JSON outputs: value, ms/step and every roofline entry."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    parts = [f"{d['value']:.1f} {d['unit']}", f"{d['ms_per_step']:.3f} ms/step"]
    rl = dict(d.get("rooflines", {}))
    if "roofline" in d:
        rl.setdefault(d["roofline"].get("kernel", "dominant"), d["roofline"])
    for k, r in rl.items():
        parts.append(f"{k}: {r.get('avg_launch_us')} us frac {r.get('frac')}")
    print(f + ": " + " | ".join(parts))
