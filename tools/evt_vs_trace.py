"""Event timing vs kernel-trace duration of the stage-1 CCF_FFN depthwise conv (B x 64^3 x 192):
HIP events around 1, 4 and 20 back-to-back launches, and the host time per launch call.
Run plain and under `rocprofv3 --kernel-trace --stats` to compare."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import waveformer_amd.network_models as NM  # noqa: E402
from waveformer_amd import ops  # noqa: E402

B, C, S = 4, 48, 64
torch.manual_seed(0)
mlp = NM.CCF_FFN(C, 4 * C, img_size=(S, S, S)).cuda().eval()
norm2 = torch.nn.LayerNorm(C, eps=1e-6).cuda()
x = torch.randn(B, S, S, S, C, device="cuda")
xh, stats = ops.msfuse([], x, 1e-6)
captured = {}
orig = ops.ccf_ffn_dwconv


def grab(args, P, Hd):
    captured["a"] = (args, P, Hd)
    return orig(args, P, Hd)


ops.ccf_ffn_dwconv = grab
with torch.no_grad():
    ops.ccf_ffn(xh, stats, norm2, mlp)
ops.ccf_ffn_dwconv = orig
a = captured["a"]
for _ in range(3):
    orig(*a)
torch.cuda.synchronize()
for reps in (1, 4, 20):
    res = []
    for _ in range(5):
        orig(*a)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            orig(*a)
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / reps * 1e3)
    print(f"events, {reps:2d} back-to-back: {min(res):8.1f} us min  {sum(res) / len(res):8.1f} us mean")
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    orig(*a)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host enqueue {1e6 * (t1 - t0) / 50:.1f} us/launch, wall {1e6 * (t2 - t0) / 50:.1f} us/launch")
