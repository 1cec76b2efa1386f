"""Encoder B=8 step as ONE forward vs N concurrent sub-batch forwards on N streams (one HIP
graph each), replay-timed -- does overlapping the VALU-bound and HBM-bound kernels of
different sub-batches pay?"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from waveformer_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", "8"))
m = bench.build_encoder(128, dev)
x = torch.randn(B, 4, 128, 128, 128, device=dev)


SERIAL = os.environ.get("SERIAL") == "1"   # sub-batches chained (no overlap): race check
EAGER_CHECK = os.environ.get("EAGER_CHECK") == "1"


def make_step(n):
    streams = [torch.cuda.Stream() for _ in range(n)]

    def step():
        with torch.no_grad():
            if n == 1:
                return m(x)
            main = torch.cuda.current_stream()
            outs = []
            with ops.weight_scope(m):
                prev = main
                for s, xi in zip(streams, x.chunk(n)):
                    s.wait_stream(prev if SERIAL else main)
                    with torch.cuda.stream(s):
                        outs.append(m(xi))
                    prev = s
                for s in streams:
                    main.wait_stream(s)
            return outs
    return step


ref = [o.clone() for o in m(x)[0]]
with torch.no_grad():
    refc = {n: [[o.clone() for o in m(xi)[0]] for xi in x.chunk(n)] for n in (2, 4)}
for n in [int(v) for v in os.environ.get("SPLITS", "1,2,4,1,2").split(",")]:
    step = make_step(n)
    for _ in range(3):
        out = step()
    torch.cuda.synchronize()
    if EAGER_CHECK and n > 1:
        for c, o in enumerate(out):
            for i, r in enumerate(refc[n][c]):
                err = (o[0][i] - r).abs().max().item()
                print(f"eager split {n}: chunk {c} stage {i} |diff| {err:.2e}", flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = step()
    g.replay()
    torch.cuda.synchronize()
    if n > 1 and os.environ.get("CHECK", "1") == "1":  # bit-equal to the sub-batches run one after the other
        for c, o in enumerate(out):
            for i, r in enumerate(refc[n][c]):
                err = (o[0][i] - r).abs().max().item()
                assert err == 0.0, f"split {n}: chunk {c} stage {i} differs by {err}"
        e8 = max((torch.cat([o[0][i] for o in out], 0) - r).abs().max().item()
                 for i, r in enumerate(ref))
        print(f"splits={n}: max |diff| vs the B={B} forward {e8:.2e}", flush=True)
    K = 100
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    print(f"splits={n}: {dt * 1e3:.3f} ms/step  {B / dt:.1f} vol/s", flush=True)
    del g
