"""Focused driver for kernel-trace A/Bs: the 128^3x4 encoder forward at B (default 8), eager,
3 warm-up + ITERS timed forwards (env switches pass through to the library)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

B = int(os.environ.get("B", "8"))
ITERS = int(os.environ.get("ITERS", "5"))
dev = torch.device("cuda", 0)
m = bench.build_encoder(128, dev)
torch.manual_seed(0)
x = torch.randn(B, 4, 128, 128, 128, device=dev)
with torch.no_grad():
    for _ in range(3):
        m(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(ITERS):
        m(x)
    torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / ITERS
print(f"encoder B={B}: {dt * 1e3:.3f} ms/forward eager ({B / dt:.1f} volumes/s)")
