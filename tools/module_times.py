"""Per-module GPU time of one full Waveformer forward (CUDA events around every module whose
name matches a depth filter).  usage: python tools/module_times.py [img] [precision] [batch] [hf]"""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from waveformer_amd import _lib, ops  # noqa: E402

img = int(sys.argv[1]) if len(sys.argv) > 1 else 192
prec = sys.argv[2] if len(sys.argv) > 2 else "fp16"
B = int(sys.argv[3]) if len(sys.argv) > 3 else 2
hf = (sys.argv[4] != "0") if len(sys.argv) > 4 else True
_lib.load()
ops.set_precision(prec)
dev = torch.device("cuda", 0)
m = bench.build_full(img, dev, hf)
x = torch.randn(B, 4, img, img, img, device=dev)
rec = {}


def hook(name):
    def pre(mod, inp):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        rec.setdefault(name, []).append([e, None])

    def post(mod, inp, out):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        rec[name][-1][1] = e
    return pre, post


for n, mod in m.named_modules():
    depth = n.count(".")
    if n and (depth == 0 or (depth <= 2 and ("decoder" in n or "learnable" in n))
              or n.startswith("waveformer_encoder.block") and depth == 1
              or n.startswith("waveformer_encoder.downsample")):
        pre, post = hook(n)
        mod.register_forward_pre_hook(pre)
        mod.register_forward_hook(post)
with torch.no_grad():
    for _ in range(3):
        rec.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m(x)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
tot = {n: sum(s.elapsed_time(e) for s, e in v) for n, v in rec.items()}
print(f"img {img} prec {prec} B {B} hf {hf}: forward wall {wall * 1e3:.2f} ms")
for n, t in tot.items():
    print(f"{t:9.3f} ms  x{len(rec[n])}  {n}")
