"""Config-4 step timing probe: encoder fwd, full fwd, DiceCE + backward per iteration.
    python tools/train_probe.py [BATCH] [ITERS]
env: WF_CL3D=1 -> channels_last_3d model/input (MIOpen NDHWC solvers for the decoder convs);
     WF_CUDNN_BENCH=1 -> torch.backends.cudnn.benchmark (MIOpen find instead of immediate)."""
import os
import sys
import time

import torch

sys.path.insert(0, '.')
import waveformer_amd.network_models as NM  # noqa: E402
from waveformer_amd.losses import DiceCELoss  # noqa: E402
from waveformer_amd import _lib  # noqa: E402

_lib.load()
torch.backends.cudnn.benchmark = os.environ.get("WF_CUDNN_BENCH", "0") == "1"
cl = os.environ.get("WF_CL3D", "0") == "1"
dev = torch.device('cuda', 0)
torch.manual_seed(0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
model = NM.Waveformer(img_size=(128,) * 3, in_chans=4, out_chans=4, depths=[2] * 4,
                      feat_size=[48, 96, 192, 384], num_heads=[3, 6, 12, 24]).train().to(dev)
x = torch.randn(B, 4, 128, 128, 128, device=dev)
y = torch.randint(0, 4, (B, 1, 128, 128, 128), device=dev)
if cl:
    model = model.to(memory_format=torch.channels_last_3d)
    x = x.contiguous(memory_format=torch.channels_last_3d)
lf = DiceCELoss()
print(f"B={B} channels_last_3d={cl} cudnn.benchmark={torch.backends.cudnn.benchmark}", flush=True)


def T():
    torch.cuda.synchronize()
    return time.perf_counter()


for it in range(iters):
    t0 = T()
    with torch.no_grad():
        model.waveformer_encoder(x)
    t1 = T()
    out = model(x)
    t2 = T()
    loss = lf(out, y)
    loss.backward()
    t3 = T()
    print(f"it {it}: enc fwd {t1-t0:.3f}s, full fwd {t2-t1:.3f}s, loss+bwd {t3-t2:.3f}s, "
          f"loss {loss.item():.4f}", flush=True)
    model.zero_grad(set_to_none=True)
print("peak GB", torch.cuda.max_memory_allocated() / 2 ** 30)
