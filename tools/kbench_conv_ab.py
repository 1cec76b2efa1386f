"""conv3d_k3 timing at the config-3 / config-5 decoder shapes under the environment's switches
(WF_CONV_PERSIST, WF_CONV_RW, ...), HIP events around ITERS calls per shape:
    python tools/kbench_conv_ab.py            (one line per shape)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from waveformer_amd import _lib, ops  # noqa: E402

_lib.load()
SHAPES = [  # (precision, B, Cin, Cout, S, fp16 input)
    ("fp16", 2, 96, 48, 192, False), ("fp16", 2, 48, 48, 192, True), ("fp16", 2, 48, 48, 192, False),
    ("bf16x3", 2, 96, 48, 128, False), ("bf16x3", 2, 48, 48, 128, False),
    ("bf16", 2, 96, 48, 128, False),
]
ITERS = int(os.environ.get("ITERS", "6"))
ONLY = os.environ.get("ONLY")  # comma-separated shape indices
EPS = None if os.environ.get("STATS", "1") == "0" else 1e-5  # fused InstanceNorm statistics
for i, (prec, B, cin, cout, s, xh) in enumerate(SHAPES):
    if ONLY and str(i) not in ONLY.split(","):
        continue
    x = torch.randn(B, cin, s, s, s, device="cuda").contiguous(memory_format=torch.channels_last_3d)
    if xh:
        x = x.half().contiguous(memory_format=torch.channels_last_3d)
    w = torch.randn(cout, cin, 3, 3, 3, device="cuda") * (cin * 27) ** -0.5
    b = torch.randn(cout, device="cuda")
    with ops.precision(prec):
        ops.conv3d_k3(x, w, b, norm_eps=EPS)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(ITERS):
            ops.conv3d_k3(x, w, b, norm_eps=EPS)
        e1.record()
        torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / ITERS * 1e3
    fl = 2 * B * cin * cout * 27 * s ** 3
    print(f"{prec:6s} B={B} {cin:3d}->{cout:3d} {s:3d}^3 xh={int(xh)}: {us:9.1f} us "
          f"{fl / us / 1e6:7.1f} TFLOP/s ({fl / us / 1e6 / 2500 * 100:5.1f}% of 2.5 PF)", flush=True)
    del x
