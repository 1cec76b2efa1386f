"""Focused driver: the stage-1 CCF_FFN (+norm2, Q4 residual) at B x 64^3 x 48 (for rocprofv3)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import waveformer_amd.network_models as NM  # noqa: E402
from waveformer_amd import ops  # noqa: E402

B = int(os.environ.get("B", "4"))
C = int(os.environ.get("C", "48"))
S = int(os.environ.get("S", "64"))
ITERS = int(os.environ.get("ITERS", "20"))
ops.set_precision(os.environ.get("WAVEFORMER_PRECISION", "bf16x3"))
torch.manual_seed(0)
mlp = NM.CCF_FFN(C, 4 * C, img_size=(S, S, S)).cuda().eval()
norm2 = torch.nn.LayerNorm(C, eps=1e-6).cuda()
x = torch.randn(B, S, S, S, C, device="cuda")
xh, stats = ops.msfuse([], x, 1e-6)
for _ in range(3):
    ops.ccf_ffn(xh, stats, norm2, mlp)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(ITERS):
    ops.ccf_ffn(xh, stats, norm2, mlp)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / ITERS
M = B * S ** 3
e = 4 if ops.get_precision() == "bf16x3" else 2
alg = M * C * 4 * 3 + 2 * 2 * M * 4 * C * e + M * 8  # x (pw+fc reads, out write), h1/h2 w+r, stats
print(f"ccf_ffn B={B} S={S} C={C}: {dt * 1e3:.3f} ms  ({alg / dt / 1e9:.0f} GB/s algorithmic)")
