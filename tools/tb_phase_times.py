"""Per-phase cycles of one ffn_dwfc_tb workgroup (stage-1 CCF_FFN back half, three VALU waves
per SIMD, one barrier per plane) from a library built with -DWF_TB_PROBE (loaded via
WAVEFORMER_HIP_LIB): per hardware wave its role (0..11 D, 12..15 E), SIMD / arrival slot, and
cycles per iteration: D = staging, scatter part 1, LN2, scatter part 2 + h2 store, barrier
wait; E = fc + epilogue, residual loads, -, -, barrier wait."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import waveformer_amd.network_models as NM  # noqa: E402
from waveformer_amd import _lib, ops  # noqa: E402

B, C, S = int(os.environ.get("B", "8")), 48, 64
torch.manual_seed(0)
mlp = NM.CCF_FFN(C, 4 * C, img_size=(S, S, S)).cuda().eval()
norm2 = torch.nn.LayerNorm(C, eps=1e-6).cuda()
x = torch.randn(B, S, S, S, C, device="cuda")
xh, stats = ops.msfuse([], x, 1e-6)
for _ in range(3):
    ops.ccf_ffn(xh, stats, norm2, mlp)
torch.cuda.synchronize()
buf = (ctypes.c_longlong * 128)()
assert _lib.load().wf_debug_tb_probe(buf) == 0
iters = int(os.environ.get("ITERS_WG", "36"))
names = ["stage/fc", "scat1/res", "ln2", "scat2", "barrier"]
print(f"(cycles per iteration, {iters} iterations of workgroup 0)")
print("wave role simd slot even " + "  ".join(f"{n:>9}" for n in names) + "   total")
for w in range(16):
    v = [buf[w * 8 + i] / iters for i in range(5)]
    tag = buf[w * 8 + 7]
    print(f"{w:4d} {buf[w * 8 + 6]:4d} {(tag & 255) // 16:4d} {tag & 15:4d} {tag >> 8:4d} " +
          "  ".join(f"{c:9.0f}" for c in v) + f"  {sum(v):7.0f}", flush=True)
