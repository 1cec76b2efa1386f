"""Encoder forward of chunk A on stream 0 while stream 1 runs ONE kind of op (repeated) on
its own data: which concurrent op corrupts chunk A?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from waveformer_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
m = bench.build_encoder(128, dev)
torch.manual_seed(0)
xa = torch.randn(4, 4, 128, 128, 128, device=dev)
with torch.no_grad():
    ref = [o.clone() for o in m(xa)[0]]
    ref2 = [o.clone() for o in m(xa)[0]]
print("ref2 vs ref", [f"{(a - b).abs().max().item():.1e}" for a, b in zip(ref2, ref)], flush=True)
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
x1 = torch.randn(4, 64, 64, 64, 48, device=dev)
x2 = torch.randn(4, 32, 32, 32, 96, device=dev)
xh2, st2 = ops.msfuse([], x2, 1e-6)
blk2 = m.block2[0]
blk1 = m.block1[0]
xh1, st1 = ops.msfuse([], x1, 1e-6)
cases = {
    "none": lambda: None,
    "bare": lambda: None,
    "block1": lambda: m.block1[0](x1),
    "merge1": lambda: m.downsample_1(x1),
    "ffn1": lambda: ops.ccf_ffn(xh1, st1, blk1.norm2, blk1.mlp),
    "attn1": lambda: blk1.attn.forward_raster(x1[:, :32, :32, :32].contiguous()),
    "msfuse1": lambda: ops.msfuse([], x1, 1e-6),
    "block2": lambda: blk2(x2),
    "ffn2": lambda: ops.ccf_ffn(xh2, st2, blk2.norm2, blk2.mlp),
    "attn2": lambda: blk2.attn.forward_raster(x2[:, :16, :16, :16].contiguous()),
    "dwt2": lambda: blk2.dwt(x2.permute(0, 4, 1, 2, 3), 1) if hasattr(blk2, "dwt") else None,
}
for name in os.environ.get("CASES", ",".join(cases)).split(","):
    fn = cases[name]
    with torch.no_grad():
        main = torch.cuda.current_stream()
        s0.wait_stream(main)
        s1.wait_stream(main)
        if name != "bare":
            with torch.cuda.stream(s1):
                with ops.weight_scope(m):
                    for _ in range(6):
                        fn()
        with torch.cuda.stream(s0):
            got = m(xa)[0]
        main.wait_stream(s0)
        main.wait_stream(s1)
        torch.cuda.synchronize()
    print(f"{name:8s}", [f"{(a - b).abs().max().item():.1e}" for a, b in zip(got, ref)], flush=True)
    with torch.no_grad():
        r3 = m(xa)[0]
    print("  main after", [f"{(a - b).abs().max().item():.1e}" for a, b in zip(r3, ref)], flush=True)
