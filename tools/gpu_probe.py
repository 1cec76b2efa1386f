"""Quick op-level sanity probe of libwaveformer_hip.so against plain torch (dev tool)."""
import math
import sys
import os

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from waveformer_amd import ops  # noqa: E402

torch.manual_seed(0)
dev = "cuda"
res = {}


def rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


# DWT
x = torch.randn(2, 16, 12, 20, 48, device=dev)
bands = ops.dwt3d_haar(x)
xr = x.permute(0, 4, 1, 2, 3)
def haar_ref(v):
    s = 1 / math.sqrt(2)
    out = {}
    a = v
    def split(t, dim):
        e = t.narrow(dim, 0, t.shape[dim]).unfold(dim, 2, 2)
        return (e[..., 0] + e[..., 1]) * s, (e[..., 0] - e[..., 1]) * s
    az, dz = split(v, 2)
    res = {}
    for zn, zt in (("a", az), ("d", dz)):
        ay, dy = split(zt, 3)
        for yn, yt in (("a", ay), ("d", dy)):
            ax, dx = split(yt, 4)
            res[zn + yn + "a"] = ax
            res[zn + yn + "d"] = dx
    return res
ref = haar_ref(xr)
ll, det = ops.bands_to_coeffs(bands)
res["dwt_ll"] = rel(ll, ref["aaa"])
for k in ops.DETAIL_KEYS:
    res["dwt_" + k] = rel(det[k], ref[k])
# IDWT round trip 2 levels
b2 = ops.dwt3d_haar(bands[0].contiguous())
ll2, det2 = ops.bands_to_coeffs(b2)
rec = ops.idwt3d_haar(ll2.contiguous(), [det2, det])
res["idwt_roundtrip"] = rel(rec, xr)

# attention: plain token batch (ws^3 = N, one window per batch)
B_, ws, C, heads = 6, 8, 48, 3
N = ws ** 3
xt = torch.randn(B_, N, C, device=dev)
wqkv = torch.randn(3 * C, C, device=dev) * 0.1
bqkv = torch.randn(3 * C, device=dev) * 0.1
wproj = torch.randn(C, C, device=dev) * 0.1
bproj = torch.randn(C, device=dev) * 0.1
table = torch.randn((2 * ws - 1) ** 3, heads, device=dev)
idx = torch.randint(0, table.shape[0], (N, N), device=dev)
bias = ops.rel_pos_bias(table, idx)
res["bias"] = rel(bias, table[idx.view(-1)].view(N, N, heads).permute(2, 0, 1))
scale = (C // heads) ** -0.5
out = ops.window_attention(xt.view(B_, ws, ws, ws, C), wqkv, bqkv, bias, wproj, bproj, ws, heads, scale)
qkv = (xt @ wqkv.t() + bqkv).reshape(B_, N, 3, heads, C // heads).permute(2, 0, 3, 1, 4)
q, k, v = qkv[0] * scale, qkv[1], qkv[2]
a = (q @ k.transpose(-2, -1) + bias.unsqueeze(0)).softmax(-1)
ref_o = ((a @ v).transpose(1, 2).reshape(B_, N, C)) @ wproj.t() + bproj
res["attn"] = rel(out.view(B_, N, C), ref_o)

# msfuse
sc = torch.randn(2, 16, 16, 16, 48, device=dev)
s1 = torch.randn(2, 8, 8, 8, 48, device=dev)
s2 = torch.randn(2, 4, 4, 4, 48, device=dev)
o, st = ops.msfuse([s1, s2], sc, 1e-6)
up = lambda t: F.interpolate(t.permute(0, 4, 1, 2, 3), size=(16, 16, 16), mode="trilinear").permute(0, 2, 3, 4, 1)
ref_m = sc + (up(s1) + up(s2))
res["msfuse"] = rel(o, ref_m)
res["msfuse_mean"] = rel(st[:, 0], ref_m.reshape(-1, 48).mean(-1))

# proj_out
po = ops.proj_out(sc, True)
res["proj_out"] = rel(po, F.layer_norm(sc, [48]).permute(0, 4, 1, 2, 3))

# patch embed
xin = torch.randn(2, 4, 16, 16, 16, device=dev)
w = torch.randn(48, 4, 2, 2, 2, device=dev)
bb = torch.randn(48, device=dev)
pe = ops.patch_embed(xin, w, bb)
res["patch_embed"] = rel(pe, F.conv3d(xin, w, bb, stride=2).permute(0, 2, 3, 4, 1))

for k, v in res.items():
    print(f"{k:20s} {v:.3e}")
bad = {k: v for k, v in res.items() if not v < 2e-2}
print("FAIL" if bad else "OK", bad)
