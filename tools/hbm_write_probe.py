"""HBM write / read / copy rates on this GPU with torch's own kernels (the ceiling a store-heavy
kernel such as the stage-1 pwconv -- 0.4 GB read, 1.6 GB written per B = 8 launch -- is up against).
    python tools/hbm_write_probe.py"""
import torch

n = 1_610_612_736 // 4  # 1.5 GiB of fp32
a = torch.empty(n, device="cuda")
b = torch.empty(n // 4, device="cuda").normal_()
c = torch.empty(n, device="cuda")


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


t = timed(lambda: a.fill_(1.0))
print(f"fill  {4 * n / 1e9:.2f} GB written: {t * 1e6:8.1f} us  {4 * n / t / 1e12:.2f} TB/s")
t = timed(lambda: a.sum())
print(f"sum   {4 * n / 1e9:.2f} GB read:    {t * 1e6:8.1f} us  {4 * n / t / 1e12:.2f} TB/s")
t = timed(lambda: c.copy_(a))
print(f"copy  {8 * n / 1e9:.2f} GB r+w:     {t * 1e6:8.1f} us  {8 * n / t / 1e12:.2f} TB/s")
# 1 : 4 read : write, the pwconv's mix: a (n/4) broadcast-expanded into c (n)
t = timed(lambda: c.view(4, -1).copy_(b.view(1, -1).expand(4, -1)))
print(f"1:4   {5 * n / 1e9:.2f} GB r+w:     {t * 1e6:8.1f} us  {5 * n / t / 1e12:.2f} TB/s (reads counted once)")
