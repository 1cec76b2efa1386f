"""Which library GEMMs (aten::mm / addmm / linear / matmul) a config-4 train step still issues:
one step at B (default 4) under torch.profiler with shapes and Python stacks."""
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
loss_fn = DiceCELoss(to_onehot_y=True, softmax=True)
x = torch.randn(B, 4, 128, 128, 128, device=dev).contiguous(memory_format=torch.channels_last_3d)
y = torch.randint(0, 4, (B, 1, 128, 128, 128), device=dev)
loss_fn(model(x), y).backward()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
             with_stack=True) as prof:
    model.zero_grad(set_to_none=True)
    loss_fn(model(x), y).backward()
    torch.cuda.synchronize()
seen = set()
for ev in prof.events():
    if ev.name in ("aten::mm", "aten::addmm", "aten::bmm", "aten::matmul", "aten::linear"):
        stack = [s for s in (ev.stack or []) if "waveformer_amd" in s or "torch/nn" in s][:4]
        key = (ev.name, str(ev.input_shapes), tuple(stack))
        if key in seen:
            continue
        seen.add(key)
        print(ev.name, ev.input_shapes, "\n    " + "\n    ".join(stack), flush=True)

print("\n# aten ops by device time (the framework's own kernels in the step)")
print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_device_time_total",
                                                         row_limit=30, max_name_column_width=40,
                                                         max_shapes_column_width=60))
