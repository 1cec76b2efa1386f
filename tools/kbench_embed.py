"""PatchEmbed (Conv3d 4 -> 48, k2 s2) at B x 4 x 128^3, HIP-event timed."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from waveformer_amd import ops  # noqa: E402

B = int(os.environ.get("B", "8"))
x = torch.randn(B, 4, 128, 128, 128, device="cuda")
w = torch.randn(48, 4, 2, 2, 2, device="cuda")
b = torch.randn(48, device="cuda")
for _ in range(3):
    ops.patch_embed(x, w, b)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20):
    ops.patch_embed(x, w, b)
e.record()
torch.cuda.synchronize()
t = s.elapsed_time(e) / 20
gb = (x.numel() + B * 64 ** 3 * 48) * 4 / 1e9
print(f"patch_embed B={B}: {t * 1e3:.1f} us  {gb / t:.0f} GB/s", flush=True)
