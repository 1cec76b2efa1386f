"""Control for the multi-stream issue: two chains of plain PyTorch (rocBLAS / MIOpen-free
elementwise + GEMM) ops at once on two streams vs the same chains run one after the other."""
import os

import torch

dev = torch.device("cuda", 0)
torch.manual_seed(0)
B = 4
xa = torch.randn(B, 64 * 64 * 64, 48, device=dev)
xb = torch.randn(B, 64 * 64 * 64, 48, device=dev)
w1 = torch.randn(48, 192, device=dev) / 7
w2 = torch.randn(192, 48, device=dev) / 14


def chain(x):
    for _ in range(4):
        h = torch.nn.functional.gelu(torch.nn.functional.layer_norm(x @ w1, (192,)))
        x = x + torch.nn.functional.layer_norm(h @ w2, (48,))
        x = x.view(B, 64, 64, 64, 48)[:, ::1].reshape(B, -1, 48)
    return x


with torch.no_grad():
    ra, rb = chain(xa).clone(), chain(xb).clone()
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    bad = 0
    for i in range(int(os.environ.get("REPS", "6"))):
        main = torch.cuda.current_stream()
        s0.wait_stream(main)
        s1.wait_stream(main)
        with torch.cuda.stream(s0):
            ga = chain(xa)
        with torch.cuda.stream(s1):
            gb = chain(xb)
        main.wait_stream(s0)
        main.wait_stream(s1)
        torch.cuda.synchronize()
        da, db = (ga - ra).abs().max().item(), (gb - rb).abs().max().item()
        bad += (da > 0) or (db > 0)
        print(f"torch chains concurrent: diff a {da:.2e} b {db:.2e}", flush=True)
    print(f"torch: {bad} runs differ", flush=True)
