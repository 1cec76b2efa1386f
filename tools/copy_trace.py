"""Which aten copies run in one config-5 forward (192^3 x 4, fp16, HF refinement, B = 2):
torch.profiler over one forward, the copy-like aten ops with their input shapes / strides and
the Python module they were called from, sorted by GPU time."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from waveformer_amd import ops  # noqa: E402

ops.set_precision("fp16")
dev = torch.device("cuda:0")
m = bench.build_full(192, dev, True)
x = torch.randn(2, 4, 192, 192, 192, device=dev)
with torch.no_grad():
    m(x)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=True, with_modules=True) as prof:
        m(x)
        torch.cuda.synchronize()
names = ("aten::copy_", "aten::contiguous", "aten::cat", "aten::clone", "aten::add", "aten::add_")
rows = []
for e in prof.events():
    if e.name in names and e.device_type.name == "CPU":
        t = getattr(e, "device_time_total", 0) or getattr(e, "cuda_time_total", 0)
        st = [s for s in (e.stack or []) if "waveformer_amd" in s][:3]
        rows.append((t, e.name, str(e.input_shapes)[:90], " <- ".join(st)[:260]))
rows.sort(key=lambda r: -r[0])
for r in rows[:25]:
    print(f"{r[0]:9.1f} us  {r[1]:18s} {r[2]}\n        {r[3]}")
