"""conv3d_k3 timing for shapes given as SHAPES="prec,B,Cin,Cout,S;..." (channel-last fp32
input, fused InstanceNorm statistics), HIP events around ITERS calls per shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from waveformer_amd import _lib, ops  # noqa: E402

_lib.load()
ITERS = int(os.environ.get("ITERS", "6"))
for spec in os.environ.get("SHAPES", "bf16x3,4,48,48,128;bf16x3,4,96,96,64").split(";"):
    prec, B, cin, cout, s = spec.split(",")
    B, cin, cout, s = int(B), int(cin), int(cout), int(s)
    x = torch.randn(B, cin, s, s, s, device="cuda").contiguous(memory_format=torch.channels_last_3d)
    w = torch.randn(cout, cin, 3, 3, 3, device="cuda") * (cin * 27) ** -0.5
    b = torch.randn(cout, device="cuda")
    with ops.precision(prec):
        ops.conv3d_k3(x, w, b, norm_eps=1e-5)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(ITERS):
            ops.conv3d_k3(x, w, b, norm_eps=1e-5)
        e1.record()
        torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / ITERS * 1e3
    fl = 2 * B * cin * cout * 27 * s ** 3
    print(f"{prec:6s} B={B} {cin:3d}->{cout:3d} {s:3d}^3: {us:9.1f} us {fl / us / 1e6:7.1f} TFLOP/s "
          f"({fl / us / 1e6 / 2500 * 100:5.1f}% of 2.5 PF)", flush=True)
    del x
