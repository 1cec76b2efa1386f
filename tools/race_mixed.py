"""Encoder forward (this library) on one stream while a plain-PyTorch GEMM / LayerNorm / GELU
chain runs on another: does the encoder still differ from its sequential reference?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
m = bench.build_encoder(128, dev)
torch.manual_seed(0)
xa = torch.randn(4, 4, 128, 128, 128, device=dev)
xb = torch.randn(4, 64 ** 3, 48, device=dev)
w1 = torch.randn(48, 192, device=dev) / 7
w2 = torch.randn(192, 48, device=dev) / 14


def chain(x):
    for _ in range(6):
        h = torch.nn.functional.gelu(torch.nn.functional.layer_norm(x @ w1, (192,)))
        x = x + torch.nn.functional.layer_norm(h @ w2, (48,))
    return x


with torch.no_grad():
    ra = [o.clone() for o in m(xa)[0]]
    rb = chain(xb).clone()
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
bad_a = bad_b = 0
REPS = int(os.environ.get("REPS", "6"))
for _ in range(REPS):
    with torch.no_grad():
        main = torch.cuda.current_stream()
        s0.wait_stream(main)
        s1.wait_stream(main)
        with torch.cuda.stream(s1):
            gb = chain(xb)
        with torch.cuda.stream(s0):
            ga = m(xa)[0]
        main.wait_stream(s0)
        main.wait_stream(s1)
        torch.cuda.synchronize()
    bad_a += max((a - b).abs().max().item() for a, b in zip(ga, ra)) > 0
    bad_b += (gb - rb).abs().max().item() > 0
print(f"encoder beside a PyTorch chain: encoder differs in {bad_a}/{REPS}, chain in {bad_b}/{REPS}",
      flush=True)
