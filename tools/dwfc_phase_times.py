"""Per-phase cycle counts of one ffn_dwfc_ws workgroup (a build with the timing probes,
WF_FFN_DBG=16): D wave 0 and E wave 0, per phase: work, barrier-1 wait, work, barrier-2 wait."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import waveformer_amd.network_models as NM  # noqa: E402
from waveformer_amd import _lib, ops  # noqa: E402

B, C, S = 8, 48, 64
torch.manual_seed(0)
mlp = NM.CCF_FFN(C, 4 * C, img_size=(S, S, S)).cuda().eval()
norm2 = torch.nn.LayerNorm(C, eps=1e-6).cuda()
x = torch.randn(B, S, S, S, C, device="cuda")
xh, stats = ops.msfuse([], x, 1e-6)
for _ in range(3):
    ops.ccf_ffn(xh, stats, norm2, mlp)
torch.cuda.synchronize()
buf = (ctypes.c_longlong * 64)()
_lib.load().wf_debug_tbuf(buf)
names = ["phase-1 work", "barrier-1 wait", "phase-2 work", "barrier-2 wait"]
for role, off in (("D wave 0", 0), ("D wave 5", 16), ("E wave 0", 8), ("E wave 5", 24)):
    v = [buf[off + i] for i in range(4)]
    tot = sum(v)
    print(role, "  ".join(f"{n} {c / 66:8.0f} cyc/plane ({100 * c / max(tot, 1):4.1f}%)"
                          for n, c in zip(names, v)), flush=True)
