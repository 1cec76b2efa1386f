"""MIOpen conv3d timing for the decoder's shapes, fp32 / bf16, NCDHW and
channels_last_3d.  Prints one line per configuration."""
import time

import torch
import torch.nn.functional as F

SHAPES = [  # (Cin, Cout, S, k)
    (4, 48, 128, 3), (48, 48, 128, 3), (96, 48, 128, 3), (48, 48, 64, 3), (144, 48, 64, 3),
    (384, 48, 8, 3),
]


def bench(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


for dt in (torch.float32, torch.bfloat16):
    for cl in (False, True):
        for cin, cout, s, k in SHAPES:
            x = torch.randn(1, cin, s, s, s, device="cuda", dtype=dt)
            w = torch.randn(cout, cin, k, k, k, device="cuda", dtype=dt)
            if cl:
                x = x.to(memory_format=torch.channels_last_3d)
                w = w.to(memory_format=torch.channels_last_3d)
            t0 = time.perf_counter()
            F.conv3d(x, w, padding=k // 2)
            torch.cuda.synchronize()
            first = time.perf_counter() - t0
            t = bench(lambda: F.conv3d(x, w, padding=k // 2))
            fl = 2 * cin * cout * k ** 3 * s ** 3
            print(f"{str(dt):15s} cl={int(cl)} {cin:4d}->{cout:3d} {s:3d}^3 k{k}: first {first:7.2f}s "
                  f"{t * 1e3:9.3f} ms {fl / t / 1e12:7.2f} TFLOP/s", flush=True)
