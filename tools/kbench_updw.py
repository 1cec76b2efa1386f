"""Fused up-sample + depthwise conv (ProjectionUpsample.conv1) vs the two-kernel path at the
config-5 shapes (img 192, B 2: learnable_up4 192 ch 24^3 -> 96^3, learnable_up3 96 ch 48^3 ->
96^3), HIP-event timed (developer tool).  Env WF_UPDW_PF picks the fused kernel variant."""
import torch
from waveformer_amd import ops, _lib

_lib.load()
ITERS = 20
for C_, src, s in [(192, 24, 4), (96, 48, 2)]:
    x = torch.randn((2, C_, src, src, src), device="cuda").contiguous(
        memory_format=torch.channels_last_3d)
    w = torch.randn((C_, 1, 3, 3, 3), device="cuda") * 0.3
    b = torch.randn((C_,), device="cuda")
    dst = (src * s,) * 3

    def fused():
        return ops.upsample_dwconv3d_cl(x, dst, w, b, 1e-5)

    def two():
        return ops.dwconv3d_cl(ops.upsample_cl(x, dst, True), w, b, norm_eps=1e-5)
    res = {}
    for name, f in (("fused", fused), ("two", two)):
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(ITERS):
            f()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / ITERS * 1e3
    a, bb = fused(), two()
    out_gb = 2 * C_ * dst[0] ** 3 * 4 / 1e9
    print(f"C {C_} {src}^3 x{s}: fused {res['fused']:.1f} us ({out_gb / res['fused'] * 1e6:.0f} GB/s "
          f"of output), two-kernel {res['two']:.1f} us, bitwise {torch.equal(a[0], bb[0])}")
