"""Stage-1 window attention (qkv GEMM + core + proj, table bias, ws 8 / head_dim 16) on a
B x 32^3 x 48 raster (the 32^3 scale of a stage-1 Block), timed with HIP events."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import waveformer_amd.network_models as NM  # noqa: E402

B = int(os.environ.get("B", "8"))
S = int(os.environ.get("S", "32"))
ITERS = int(os.environ.get("ITERS", "20"))
torch.manual_seed(0)
m = NM.Attention(48, num_heads=3, qkv_bias=True, window_size=8).cuda().eval()
x = torch.randn(B, S, S, S, 48, device="cuda")
with torch.no_grad():
    for _ in range(3):
        m.forward_raster(x)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(ITERS):
        m.forward_raster(x)
    e.record()
torch.cuda.synchronize()
print(f"window_attention B={B} {S}^3 x 48: {s.elapsed_time(e) / ITERS * 1e3:.1f} us", flush=True)
