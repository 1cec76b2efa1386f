"""Does ffn_dwfc_tb4's time depend on where its buffers sit?  The encoder's two stage-1 blocks
run it at ~700 and ~800 us with the same code and shapes.  Stage-1 CCF_FFN at B = 8 with the
workspace (h1) and the output placed at varied offsets inside larger allocations; HIP events
around REPS tb4 launches (wf_ccf_ffn_stage 2) after the pwconv (stage 1) filled h1."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import waveformer_amd.network_models as NM  # noqa: E402
from waveformer_amd import _lib, ops  # noqa: E402

B, S, C = 8, 64, 48
REPS = int(os.environ.get("REPS", "5"))
dev = torch.device("cuda", 0)
torch.manual_seed(0)
mlp = NM.CCF_FFN(C, 4 * C, img_size=(S, S, S)).to(dev).eval()
norm2 = torch.nn.LayerNorm(C, eps=1e-6).to(dev)
x = torch.randn(B, S, S, S, C, device=dev)
xh, stats = ops.msfuse([], x, 1e-6)
prec = ops.prec_id()
hid = 4 * C
pw = ops.split_weight(mlp.pwconv.weight, (hid, C), prec)
fc = ops.split_weight(mlp.fc.weight, prec=prec)
wsb = _lib.query("wf_ccf_ffn_workspace_bytes", B, C, hid, S, S, S, prec)
MB = 1 << 20
big_w = torch.empty(wsb + 96 * MB, dtype=torch.uint8, device=dev)
big_o = torch.empty(xh.numel() * 4 + 96 * MB, dtype=torch.uint8, device=dev)
p = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731


def run(wo, oo):
    args = (xh.data_ptr(), stats.data_ptr(), norm2.weight.data_ptr(), norm2.bias.data_ptr(),
            pw.data_ptr(), p(mlp.pwconv.bias), mlp.norm1.weight.data_ptr(),
            mlp.norm1.bias.data_ptr(), float(mlp.norm1.eps), mlp.dwconv.weight.data_ptr(),
            mlp.dwconv.bias.data_ptr(), mlp.norm2.weight.data_ptr(), mlp.norm2.bias.data_ptr(),
            float(mlp.norm2.eps), fc.data_ptr(), p(mlp.fc.bias), 0,
            big_o.data_ptr() + oo, big_w.data_ptr() + wo, B, C, hid, S, S, S, prec,
            torch.cuda.current_stream().cuda_stream)
    _lib.call("wf_ccf_ffn_stage", 1, *args)
    _lib.call("wf_ccf_ffn_stage", 2, *args)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        _lib.call("wf_ccf_ffn_stage", 2, *args)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / REPS


for wo in (0, 1 * MB, 2 * MB, 4 * MB, 8 * MB, 16 * MB, 32 * MB, 64 * MB, 256):
    print(f"workspace +{wo / MB:6.3f} MB, out +0: {run(wo, 0):7.1f} us", flush=True)
for oo in (1 * MB, 2 * MB, 8 * MB, 32 * MB, 256):
    print(f"workspace +0, out +{oo / MB:6.3f} MB: {run(0, oo):7.1f} us", flush=True)
print(f"workspace +0, out +0 again: {run(0, 0):7.1f} us")
