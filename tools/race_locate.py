"""Where do concurrent two-stream encoder forwards go wrong?  Runs separate-module pairs (as
race_arena.py) and, for every differing stage output, prints the differing region: samples,
channel / z / y / x extents and the element count -- a 4x8 (y, x) tile points at ffn_dwfc, an
x row at msfuse, an 8^3 window at attention, whole planes at the DWT / merges."""
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
    rb = [o.clone() for o in m2(xb)[0]]
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()


def region(d, tag):
    nz = (d > 1e-6).nonzero()
    if nz.numel() == 0:
        return
    lo, hi = nz.min(0).values.tolist(), nz.max(0).values.tolist()
    print(f"  {tag}: {nz.shape[0]} elements, samples {sorted(set(nz[:, 0].tolist()))}, "
          f"c {lo[1]}-{hi[1]}, z {lo[2]}-{hi[2]}, y {lo[3]}-{hi[3]}, x {lo[4]}-{hi[4]}, "
          f"max {d.max().item():.2e}", flush=True)


for rep in range(int(os.environ.get("REPS", "8"))):
    with torch.no_grad():
        main = torch.cuda.current_stream()
        s0.wait_stream(main)
        s1.wait_stream(main)
        with torch.cuda.stream(s0):
            ga = m1(xa)[0]
        with torch.cuda.stream(s1):
            gb = m2(xb)[0]
        main.wait_stream(s0)
        main.wait_stream(s1)
        torch.cuda.synchronize()
    print(f"rep {rep}", flush=True)
    for st, (a, b) in enumerate(zip(ga, ra)):
        region((a - b).abs(), f"A stage {st}")
        if (a - b).abs().max().item() > 0:
            break
    for st, (a, b) in enumerate(zip(gb, rb)):
        region((a - b).abs(), f"B stage {st}")
        if (a - b).abs().max().item() > 0:
            break
