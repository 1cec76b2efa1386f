"""Phase attribution of the whole-FFN kernel (ffn_fused.hip): the stage-1 CCF_FFN op at
B x 64^3 x 48 timed with HIP events for each WF_FFN_DBG phase mask (results of a masked build
are invalid -- only the time counts).  Usage: python tools/kbench_ffn_fused.py [masks...]"""
import os
import sys

import torch

os.environ["WF_FFN_FUSED"] = "1"  # before the library is loaded

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import waveformer_amd.network_models as NM  # noqa: E402
from waveformer_amd import ops  # noqa: E402

B = int(os.environ.get("B", "8"))
S = int(os.environ.get("S", "64"))
ITERS = int(os.environ.get("ITERS", "20"))
NAMES = {1: "scatter", 2: "pw", 4: "ln1", 8: "ln2", 16: "fc", 32: "fetch", 64: "h2t"}
masks = [int(m) for m in sys.argv[1:]] or [0, 1, 2, 4, 8, 16, 32, 64, 127]
torch.manual_seed(0)
mlp = NM.CCF_FFN(48, 192, img_size=(S, S, S)).cuda().eval()
norm2 = torch.nn.LayerNorm(48, eps=1e-6).cuda()
x = torch.randn(B, S, S, S, 48, device="cuda")
xh, stats = ops.msfuse([], x, 1e-6)
for m in masks:
    os.environ["WF_FFN_DBG"] = str(m)
    for _ in range(2):
        ops.ccf_ffn(xh, stats, norm2, mlp)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(ITERS):
        ops.ccf_ffn(xh, stats, norm2, mlp)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / ITERS * 1e3
    skipped = "+".join(n for b, n in NAMES.items() if m & b) or "none"
    print(f"mask {m:3d} (skip {skipped:40s}): {us:8.1f} us", flush=True)
os.environ.pop("WF_FFN_DBG")
