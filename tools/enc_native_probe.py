"""ATen ops with device time of their own in one eager encoder forward (B = 8, 128^3): where
the replay trace's __amd_rocclr_copyBuffer launches and other non-framework kernels come from."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
m = bench.build_encoder(128, dev)
x = torch.randn(8, 4, 128, 128, 128, device=dev)
with torch.no_grad():
    for _ in range(2):
        m(x)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=True) as prof:
        m(x)
        torch.cuda.synchronize()
agg = collections.defaultdict(lambda: [0.0, 0])
for ev in prof.events():
    t = getattr(ev, "self_device_time_total", None)
    if t is None:
        t = ev.self_cuda_time_total
    if t <= 0 or not ev.name.startswith(("aten::", "cuda", "Memcpy", "Memset")):
        continue
    frames = [s.split("/")[-1] for s in (ev.stack or []) if "waveformer_amd" in s or "bench.py" in s][:3]
    agg[(ev.name, str(ev.input_shapes)[:80], " < ".join(frames))][0] += t
    agg[(ev.name, str(ev.input_shapes)[:80], " < ".join(frames))][1] += 1
for (n, sh, fr), (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:30]:
    print(f"{t:9.1f} us x{c:3d}  {n:22s} {sh:80s} {fr}")
print(prof.key_averages().table(sort_by="self_device_time_total", row_limit=12, max_name_column_width=60))
