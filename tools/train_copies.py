"""Which framework ops (layout copies, adds, fills) run inside one config-4 train step, and from
where: torch.profiler with stacks over one step after warm-up, aggregated by (op, shapes, the
innermost waveformer_amd frame).
    python tools/train_copies.py [BATCH]"""
import collections
import sys

import torch

sys.path.insert(0, ".")
import waveformer_amd.network_models as NM  # noqa: E402
from waveformer_amd import _lib  # noqa: E402
from waveformer_amd.losses import DiceCELoss  # noqa: E402

_lib.load()
dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
torch.manual_seed(0)
model = NM.Waveformer(img_size=(128,) * 3, in_chans=4, out_chans=4, depths=[2] * 4,
                      feat_size=[48, 96, 192, 384], num_heads=[3, 6, 12, 24]).train().to(dev)
x = torch.randn(B, 4, 128, 128, 128, device=dev)
y = torch.randint(0, 4, (B, 1, 128, 128, 128), device=dev)
lf = DiceCELoss(to_onehot_y=True, softmax=True)
opt = torch.optim.AdamW(model.parameters(), lr=1e-4)


def step():
    opt.zero_grad(set_to_none=True)
    loss = lf(model(x), y)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 12)
    opt.step()


for _ in range(2):
    step()
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
agg = collections.defaultdict(lambda: [0, 0.0])
for ev in prof.events():
    if ev.name not in ("aten::copy_", "aten::add_", "aten::add", "aten::fill_", "aten::zero_",
                       "aten::clone", "aten::contiguous", "aten::gelu", "aten::gelu_backward",
                       "aten::mul", "aten::sum", "aten::native_group_norm",
                       "aten::native_group_norm_backward"):
        continue
    frames = [f for f in (ev.stack or []) if "waveformer_amd" in f or "torch/autograd" in f]
    where = frames[0] if frames else "?"
    t = ev.device_time_total if hasattr(ev, "device_time_total") else ev.cuda_time_total
    key = (ev.name, str(ev.input_shapes)[:80], where)
    agg[key][0] += 1
    agg[key][1] += t
tot = sum(v[1] for v in agg.values())
print(f"framework ops: {tot / 1e3:.2f} ms of device time in one step")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{v[1] / 1e3:7.2f} ms {v[0]:4d}x  {k[0]:14s} {k[1]:80s} {k[2]}")
