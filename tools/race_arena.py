"""Two encoder forwards at once on two streams: one shared module (one weight arena, refreshed
by both forwards) vs two modules with identical weights (separate arenas).  Counts runs whose
outputs differ from the sequential reference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
m1 = bench.build_encoder(128, dev)
m2 = bench.build_encoder(128, dev)
m2.load_state_dict(m1.state_dict())
torch.manual_seed(0)
xa = torch.randn(4, 4, 128, 128, 128, device=dev)
xb = torch.randn(4, 4, 128, 128, 128, device=dev)
with torch.no_grad():
    ra = [o.clone() for o in m1(xa)[0]]
    rb = [o.clone() for o in m1(xb)[0]]
    rb2 = [o.clone() for o in m2(xb)[0]]
print("m2 vs m1 sequential:", max((a - b).abs().max().item() for a, b in zip(rb, rb2)), flush=True)
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
REPS = int(os.environ.get("REPS", "6"))
for name, mb in ((("shared", m1), ("separate", m2)) if not os.environ.get("ONLY_SEP") else (("separate", m2),)):
    bad = 0
    for _ in range(REPS):
        with torch.no_grad():
            main = torch.cuda.current_stream()
            s0.wait_stream(main)
            s1.wait_stream(main)
            with torch.cuda.stream(s0):
                ga = m1(xa)[0]
            with torch.cuda.stream(s1):
                gb = mb(xb)[0]
            main.wait_stream(s0)
            main.wait_stream(s1)
            torch.cuda.synchronize()
        da = max((a - b).abs().max().item() for a, b in zip(ga, ra))
        db = max((a - b).abs().max().item() for a, b in zip(gb, rb))
        bad += (da > 0) or (db > 0)
        print(f"{name:9s} diff a {da:.2e} b {db:.2e}", flush=True)
    print(f"{name}: {bad}/{REPS} runs differ", flush=True)
