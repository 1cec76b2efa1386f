"""Fused up-sample + depthwise conv vs the two-kernel path: max difference and where (developer
diagnostic)."""
import torch
import torch.nn.functional as F
from oracle.weight_rule import seeded_randn
from waveformer_amd import ops, _lib
_lib.load()
for B, C_, src, s, ac in [(2, 32, (5, 6, 7), 2, True), (1, 192, (6, 5, 7), 4, True),
                          (1, 96, (3, 9, 12), 2, False), (1, 32, (2, 2, 20), 2, True)]:
    dst = tuple(a * s for a in src)
    x = seeded_randn((B, C_) + src, 12).cuda().contiguous(memory_format=torch.channels_last_3d)
    w = seeded_randn((C_, 1, 3, 3, 3), 13).cuda() * 0.3
    b = seeded_randn((C_,), 14).cuda()
    got, gst = ops.upsample_dwconv3d_cl(x, dst, w, b, 1e-5, ac)
    up = ops.upsample_cl(x, dst, ac)
    want, wst = ops.dwconv3d_cl(up, w, b, norm_eps=1e-5)
    ref = F.conv3d(F.interpolate(x.double().cpu(), size=dst, mode="trilinear", align_corners=ac),
                   w.double().cpu(), b.double().cpu(), padding=1, groups=C_)
    d = (got - want).abs()
    i = int(d.argmax())
    idx = torch.unravel_index(torch.tensor(i), d.shape)
    rel = lambda a: float((a.double().cpu() - ref).norm() / ref.norm())
    print(B, C_, src, s, ac, "maxdiff", float(d.max()), "at", [int(t) for t in idx],
          "n!=", int((d > 0).sum()), "/", d.numel(), "rel fused", rel(got), "rel 2k", rel(want),
          "stats maxdiff", float((gst - wst).abs().max()))
