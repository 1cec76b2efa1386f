"""HIP implicit-GEMM conv3d (ops.conv3d_k3) timing at the decoder's shapes, with the MFMA
roofline fraction (logical fp32 flops; bf16x3 issues 3 MFMAs per product).
    python tools/kbench_conv_hip.py [ONLY_INDEX]      (XH=1: fp16 input, with WAVEFORMER_PRECISION=fp16)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from waveformer_amd import _lib, ops  # noqa: E402

_lib.load()
SHAPES = [  # (B, Cin, Cout, S) -- sliding-window batches of 2
    (2, 4, 48, 128), (2, 48, 48, 128), (2, 96, 48, 128), (2, 96, 48, 64), (2, 48, 48, 64),
    (2, 384, 192, 8), (2, 384, 96, 8), (2, 192, 96, 16), (2, 96, 96, 32),
    (2, 96, 48, 192), (2, 48, 48, 192),  # config 5's full-resolution decoder convs
]
ITERS = int(os.environ.get("ITERS", "10"))
only = int(sys.argv[1]) if len(sys.argv) > 1 else None
ops.set_precision(os.environ.get("WAVEFORMER_PRECISION", "bf16x3"))
for i, (B, cin, cout, s) in enumerate(SHAPES):
    if only is not None and i != only:
        continue
    x = torch.randn(B, cin, s, s, s, device="cuda").contiguous(memory_format=torch.channels_last_3d)
    if os.environ.get("XH"):  # fp16 input in HBM (wf_conv3d_k3_fwd_xh; fp16 precision only)
        x = x.half().contiguous(memory_format=torch.channels_last_3d)
    w = torch.randn(cout, cin, 3, 3, 3, device="cuda") * (cin * 27) ** -0.5
    ops.conv3d_k3(x, w)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(ITERS):
        ops.conv3d_k3(x, w)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / ITERS
    fl = 2 * B * cin * cout * 27 * s ** 3
    mult = 3 if ops.get_precision() == "bf16x3" else 1
    print(f"B={B} {cin:4d}->{cout:3d} {s:3d}^3: {t * 1e3:8.3f} ms {fl / t / 1e12:7.1f} TFLOP/s "
          f"(MFMA issue {mult * fl / t / 2.5e15 * 100:5.1f}% of 2.5 PF)", flush=True)
