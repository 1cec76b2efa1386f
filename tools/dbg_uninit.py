"""Uninitialised-read probe: fill the caching allocator's free memory with NaN before each
encoder forward, then look for NaN / run-to-run differences per module output (forward hooks),
so a kernel that reads memory it never wrote shows up by name."""
import sys

import torch

sys.path.insert(0, ".")
from tests import cases as C  # noqa: E402
from waveformer_amd import _lib  # noqa: E402

_lib.load()
name = sys.argv[1] if len(sys.argv) > 1 else "enc128"
case = C.cases()[name]
m, _ = C.build(case, "cuda")
x = C.case_input(case).cuda()
rec = {}


def hook(n):
    def f(mod, inp, out):
        outs = out if isinstance(out, (tuple, list)) else (out,)
        flat = []
        for o in outs:
            if isinstance(o, torch.Tensor):
                flat.append(o)
            elif isinstance(o, (tuple, list)):
                for d in o:
                    if isinstance(d, dict):
                        flat += [d[k] for k in sorted(d)]
        rec.setdefault(n, []).append([t.detach().clone() for t in flat])
    return f


for n, mod in m.named_modules():
    if n.count(".") <= 2 and n:
        mod.register_forward_hook(hook(n))
for it in range(4):
    junk = torch.full((6 * 1024 ** 3 // 4,), float("nan"), device="cuda")
    del junk
    with torch.no_grad():
        m(x)
    torch.cuda.synchronize()
for n, runs in rec.items():
    worst, nan = 0.0, False
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            nan |= bool(torch.isnan(b).any()) or bool(torch.isnan(a).any())
            d = (a - b).abs().max().item() if a.numel() else 0.0
            worst = max(worst, d)
    if worst > 0 or nan:
        print(f"{n:40s} max run-to-run diff {worst:.3e} nan {nan}", flush=True)
print("done", flush=True)
