"""Where a config-4 train step's non-framework (ATen) device time comes from: one step at B
(default 2) under torch.profiler; every aten op with device time of its own, grouped by (op,
shapes, origin) -- origin = the Python frames in waveformer_amd for forward ops, the autograd
node for backward ops -- sorted by device time."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import waveformer_amd.network_models as NM  # noqa: E402
from waveformer_amd.losses import DiceCELoss  # noqa: E402

B = int(os.environ.get("B", "2"))
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = NM.Waveformer(img_size=(128,) * 3, in_chans=4, out_chans=4, depths=[2, 2, 2, 2],
                      feat_size=[48, 96, 192, 384], num_heads=[3, 6, 12, 24]).train().to(dev)
model = model.to(memory_format=torch.channels_last_3d)
opt = torch.optim.AdamW(model.parameters(), lr=1e-4, fused=True)
loss_fn = DiceCELoss(to_onehot_y=True, softmax=True)
x = torch.randn(B, 4, 128, 128, 128, device=dev).contiguous(memory_format=torch.channels_last_3d)
y = torch.randint(0, 4, (B, 1, 128, 128, 128), device=dev)


def step():
    opt.zero_grad(set_to_none=True)
    loss_fn(model(x), y).backward()
    opt.step()


step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
             with_stack=True) as prof:
    step()
    torch.cuda.synchronize()


def origin(ev):
    p = ev
    while p is not None:
        if p.name.startswith("autograd::engine::evaluate_function"):
            return p.name.split(": ", 1)[-1]
        p = p.cpu_parent
    frames = [s.split("/")[-1] for s in (ev.stack or []) if "waveformer_amd" in s][:3]
    return " < ".join(frames) or "?"


agg = collections.defaultdict(lambda: [0.0, 0])
total = 0.0
for ev in prof.events():
    t = getattr(ev, "self_device_time_total", None)
    if t is None:
        t = ev.self_cuda_time_total
    if t <= 0 or not ev.name.startswith("aten::"):
        continue
    key = (ev.name, str(ev.input_shapes)[:90], origin(ev))
    agg[key][0] += t
    agg[key][1] += 1
    total += t
print(f"# ATen ops with device time of their own, B = {B}: {total / 1e3:.2f} ms in one step")
for (name, shapes, org), (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:45]:
    print(f"{t / 1e3:8.3f} ms x{n:3d}  {name:24s} {org[:70]:70s} {shapes}")
