import sys, time, torch
sys.path.insert(0, '.')
import waveformer_amd.network_models as NM
from waveformer_amd.losses import DiceCELoss
from waveformer_amd import _lib; _lib.load()
dev = torch.device('cuda', 0)
torch.manual_seed(0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
model = NM.Waveformer(img_size=(128,)*3, in_chans=4, out_chans=4, depths=[2]*4, feat_size=[48,96,192,384], num_heads=[3,6,12,24]).train().to(dev)
x = torch.randn(B, 4, 128, 128, 128, device=dev)
y = torch.randint(0, 4, (B, 1, 128, 128, 128), device=dev)
lf = DiceCELoss()
def T(): torch.cuda.synchronize(); return time.perf_counter()
for it in range(3):
    t0 = T()
    enc = model.waveformer_encoder(x)
    t1 = T()
    out = model(x)
    t2 = T()
    loss = lf(out, y)
    loss.backward()
    t3 = T()
    print(f"it {it}: enc fwd {t1-t0:.3f}s, full fwd {t2-t1:.3f}s, loss+bwd {t3-t2:.3f}s, loss {loss.item():.4f}", flush=True)
    model.zero_grad(set_to_none=True)
print("peak GB", torch.cuda.max_memory_allocated()/2**30)
