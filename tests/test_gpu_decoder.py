"""GPU parity of the decoder convolution stack: the channel-last implicit-GEMM
3x3x3 convolution (csrc/conv3d.hip), the InstanceNorm statistics / fused norm + residual +
LeakyReLU pass (csrc/instnorm.hip) and the MONAI blocks that use them, against the oracle's
fp32 PyTorch arithmetic on the CPU (F.conv3d / F.instance_norm / F.leaky_relu, the reference's
ops, monai/networks/blocks/dynunet_block.py:98-185).

Tolerances: convolution rel-L2 <= 1e-5 in the fp32-faithful bf16x3 mode (operand error 2^-17,
fp32 accumulation over up to 2592 terms; measured against fp32 CPU convolution), <= 1e-2 in
plain bf16; InstanceNorm / norm_act rel-L2 <= 1e-6 (fp64 statistics); whole blocks rel-L2
<= 2e-5 (bf16x3; InstanceNorm renormalises every conv output).  The full model's parity
(tests/test_gpu_parity.py: full32 / full32hf rel-L2 1e-4, 128^3 and 192^3 Dice) runs through
these kernels as well.
"""
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_waveformer as R
from oracle.weight_rule import seeded_randn
from tests import cases as C

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from waveformer_amd import _lib
    _lib.load()
    yield


@pytest.mark.parametrize("prec,tol", [("bf16x3", 1e-5), ("bf16", 1e-2)])
@pytest.mark.parametrize("B,Cin,Cout,S", [
    (1, 4, 48, (20, 18, 70)),     # encoder1's first conv (Cin 4), W > 64: two x tiles, ragged
    (2, 96, 48, (9, 13, 33)),     # decoder conv_block conv1 (2C -> C), W in (32, 64]
    (1, 48, 48, (8, 5, 17)),      # W in (16, 32]
    (1, 192, 96, (6, 7, 11)),     # Cout 96 = 2 workgroup column blocks, W <= 16
    (1, 384, 192, (8, 8, 8)),     # decoder4.conv_lf_block shape
    (1, 20, 32, (3, 4, 5)),       # Cin not a multiple of 16, Cout not a multiple of 48
])
def test_conv3d_k3_vs_cpu(B, Cin, Cout, S, prec, tol):
    from waveformer_amd import ops
    x = seeded_randn((B, Cin) + S, 1) * 2 + 0.1
    w = seeded_randn((Cout, Cin, 3, 3, 3), 2) * (Cin * 27) ** -0.5
    b = seeded_randn((Cout,), 3)
    want = F.conv3d(x.double(), w.double(), b.double(), padding=1)
    with ops.precision(prec):
        got = ops.conv3d_k3(x.cuda(), w.cuda(), b.cuda())
    assert got.is_contiguous(memory_format=torch.channels_last_3d)
    assert C.rel_l2(got, want) <= tol


def test_conv3d_k3_channel_slices():
    """Input = channels [8, 56) of a wider channel-last buffer, output into channels [16, 64)
    of another: the ld arguments of the C-ABI."""
    from waveformer_amd import ops
    xb = seeded_randn((2, 72, 6, 9, 20), 4).cuda().contiguous(memory_format=torch.channels_last_3d)
    ob = torch.zeros((2, 80, 6, 9, 20), device="cuda").contiguous(
        memory_format=torch.channels_last_3d)
    w = (seeded_randn((48, 48, 3, 3, 3), 5) * 0.03).cuda()
    ops.conv3d_k3(xb[:, 8:56], w, None, out=ob[:, 16:64])
    want = F.conv3d(xb[:, 8:56].double().cpu(), w.double().cpu(), padding=1)
    assert C.rel_l2(ob[:, 16:64], want) <= 1e-5
    assert float(ob[:, :16].abs().max()) == 0.0 and float(ob[:, 64:].abs().max()) == 0.0


@pytest.mark.parametrize("shape", [(2, 48, 16, 16, 16), (1, 4, 7, 9, 5), (3, 96, 4, 4, 4)])
def test_instnorm_and_norm_act(shape):
    from waveformer_amd import ops
    a = (seeded_randn(shape, 6) * 3 + 5).cuda().contiguous(memory_format=torch.channels_last_3d)
    r = (seeded_randn(shape, 7) - 2).cuda().contiguous(memory_format=torch.channels_last_3d)
    sa = ops.instnorm_stats(a, 1e-5)
    sr = ops.instnorm_stats(r, 1e-5)
    ad, rd = a.double().cpu(), r.double().cpu()
    na, nr = F.instance_norm(ad, eps=1e-5), F.instance_norm(rd, eps=1e-5)
    assert C.rel_l2(ops.norm_act(a, sa, slope=1.0), na) <= 1e-6
    assert C.rel_l2(ops.norm_act(a, sa, r, sr), F.leaky_relu(na + nr, 0.01)) <= 1e-6
    assert C.rel_l2(ops.norm_act(a, sa, r), F.leaky_relu(na + rd, 0.01)) <= 1e-6
    out = a.clone(memory_format=torch.channels_last_3d)
    ops.norm_act(out, ops.instnorm_stats(out, 1e-5), slope=0.01, out=out)  # in place
    assert C.rel_l2(out, F.leaky_relu(na, 0.01)) <= 1e-6


@pytest.mark.parametrize("cin,cout,S", [(4, 48, 24), (96, 48, 16), (48, 48, 12)])
def test_unet_res_block_fast_path(cin, cout, S):
    """UnetResBlock (downsample residual when cin != cout) on the HIP path vs the oracle."""
    from waveformer_amd.blocks import UnetResBlock
    torch.manual_seed(0)
    blk = UnetResBlock(3, cin, cout, 3, 1, "instance").eval()
    sd = {k: v.clone() for k, v in blk.state_dict().items()}
    x = seeded_randn((1, cin, S, S, S), 8)
    want = R.unet_res_block(sd, "", x)
    with torch.no_grad():
        got = blk.cuda()(x.cuda())
    assert C.rel_l2(got, want) <= 2e-5


def test_unet_basic_block_fast_path():
    from waveformer_amd.blocks import UnetBasicBlock
    torch.manual_seed(1)
    blk = UnetBasicBlock(3, 32, 16, 3, 1, "instance").eval()
    x = seeded_randn((2, 32, 10, 12, 14), 9)
    with torch.no_grad():
        want = blk(x)                      # CPU: the PyTorch modules
        got = blk.cuda()(x.cuda())         # GPU: the HIP fast path
    assert C.rel_l2(got, want) <= 2e-5


@pytest.mark.parametrize("ac", [True, False])
@pytest.mark.parametrize("src,dst", [((4, 5, 6), (16, 20, 24)), ((8, 8, 8), (16, 16, 16)),
                                     ((3, 1, 7), (5, 4, 14))])
def test_upsample_cl_vs_interpolate(src, dst, ac):
    from waveformer_amd import ops
    x = seeded_randn((2, 12) + src, 10)
    want = F.interpolate(x, size=dst, mode="trilinear", align_corners=ac)
    got = ops.upsample_cl(x.cuda(), dst, ac)
    assert C.rel_l2(got, want) <= 1e-6


@pytest.mark.parametrize("cin,cout,stride,double", [(192, 48, 4, True), (96, 48, 2, False)])
def test_projection_upsample_fast_path(cin, cout, stride, double):
    """learnable_up4 / learnable_up3 (wave_helper.py:33-81) on the HIP path (channel-last
    upsample + depthwise conv + folded GroupNorm + GEMMs, residual 1x1 conv before its
    upsample) vs the PyTorch modules on the CPU.  fp32 throughout: rel-L2 <= 1e-5."""
    from waveformer_amd.network_models.wave_helper import ProjectionUpsample
    torch.manual_seed(2)
    m = ProjectionUpsample(cin, cout, stride=stride, residual=True, use_double_conv=double).eval()
    with torch.no_grad():
        for p in m.parameters():   # non-trivial GroupNorm affine
            p.add_(0.05 * torch.randn_like(p))
    x = seeded_randn((2, cin, 6, 5, 7), 11)
    with torch.no_grad():
        want = m(x)
        got = m.cuda()(x.cuda())
    assert tuple(got.shape) == tuple(want.shape)
    assert C.rel_l2(got, want) <= 1e-5


def test_unetr_up_block_fast_path():
    """decoder1 (monai UnetrUpBlock, unetr_block.py:22-86): ConvTranspose3d(k2, s2) as a GEMM
    scattered into the channel-last concatenation buffer, then the UnetResBlock, vs the CPU
    modules."""
    from waveformer_amd.blocks import UnetrUpBlock
    torch.manual_seed(3)
    m = UnetrUpBlock(3, 144, 48, 3, 2, "instance", res_block=True).eval()
    x = seeded_randn((2, 144, 5, 6, 7), 12)
    skip = seeded_randn((2, 48, 10, 12, 14), 13)
    with torch.no_grad():
        want = m(x, skip)
        got = m.cuda()(x.cuda(), skip.cuda())
    assert C.rel_l2(got, want) <= 2e-5


@pytest.mark.parametrize("B,Cin,Cout,S", [(2, 48, 48, (12, 9, 70)), (1, 384, 192, (8, 8, 8)),
                                          (1, 20, 32, (5, 6, 19))])
def test_conv3d_k3_fused_instnorm_stats(B, Cin, Cout, S):
    """The InstanceNorm statistics accumulated in the conv epilogue (and, for split-K small
    grids, by the follow-up pass) equal mean / rstd of the conv output: rel err <= 1e-5."""
    from waveformer_amd import ops
    x = (seeded_randn((B, Cin) + S, 14) + 0.5).cuda()
    w = (seeded_randn((Cout, Cin, 3, 3, 3), 15) * (Cin * 27) ** -0.5).cuda()
    b = seeded_randn((Cout,), 16).cuda()
    out, st = ops.conv3d_k3(x, w, b, norm_eps=1e-5)
    o = out.double().cpu()
    mean = o.mean(dim=(2, 3, 4))
    rstd = 1.0 / torch.sqrt(o.var(dim=(2, 3, 4), unbiased=False) + 1e-5)
    assert C.rel_l2(st[:, 0], mean) <= 1e-5
    assert C.rel_l2(st[:, 1], rstd) <= 1e-5


@pytest.mark.parametrize("src,s", [((4, 5, 6), 4), ((8, 7, 3), 2)])
def test_upsample_cl_autograd_adjoint(src, s):
    """Training path of ProjectionUpsample's nn.Upsample(align_corners=True): the HIP adjoint
    (three separable gather passes) vs PyTorch's autograd of F.interpolate on the CPU."""
    from waveformer_amd import autograd as wfa
    x = seeded_randn((2, 8) + src, 17)
    size = tuple(v * s for v in src)
    g = seeded_randn((2, 8) + size, 18)
    xc = x.clone().requires_grad_(True)
    F.interpolate(xc, size=size, mode="trilinear", align_corners=True).backward(g)
    xg = x.cuda().requires_grad_(True)
    y = wfa.upsample_cl(xg, size)
    want_y = F.interpolate(x, size=size, mode="trilinear", align_corners=True)
    assert C.rel_l2(y, want_y) <= 1e-6
    y.backward(g.cuda())
    assert C.rel_l2(xg.grad, xc.grad) <= 1e-6


@pytest.mark.parametrize("cin,cout,S", [(48, 48, (6, 7, 20)), (4, 48, (5, 5, 9)), (96, 16, (4, 6, 5))])
def test_conv3d_k3_autograd(cin, cout, S):
    """Training path of the decoder conv (wfa.Conv3dK3): forward on the MFMA kernel, input
    gradient on the same kernel with flipped / transposed weights (or the framework's when
    Cin % 16 != 0), weight / bias gradients from the framework; vs CPU autograd, rel-L2 1e-5."""
    from waveformer_amd import autograd as wfa
    x = seeded_randn((2, cin) + S, 19)
    w = seeded_randn((cout, cin, 3, 3, 3), 20) * (cin * 27) ** -0.5
    b = seeded_randn((cout,), 21)
    g = seeded_randn((2, cout) + S, 22)
    xc, wc, bc = (t.clone().requires_grad_(True) for t in (x, w, b))
    F.conv3d(xc, wc, bc, padding=1).backward(g)
    xg, wg, bg = (t.cuda().requires_grad_(True) for t in (x, w, b))
    y = wfa.conv3d_k3(xg, wg, bg)
    y.backward(g.cuda())
    assert C.rel_l2(y, F.conv3d(x, w, b, padding=1)) <= 1e-5
    assert C.rel_l2(xg.grad, xc.grad) <= 1e-5
    assert C.rel_l2(wg.grad, wc.grad) <= 1e-5
    assert C.rel_l2(bg.grad, bc.grad) <= 1e-5


@pytest.mark.parametrize("M,N,K,pad", [(100000, 192, 48, 0), (4097, 48, 32, 8),
                                       (3000, 384, 96, 0), (777, 20, 70, 4), (64, 1536, 384, 0),
                                       (33, 5, 3, 0)])
def test_gemm_tn_vs_fp64(M, N, K, pad):
    """wf_gemm_tn (the training path's weight gradients dW = dY^T X, ABI 14): bf16x3 MFMAs over
    M rows dealt to many workgroups, partials summed in a fixed order -- against the fp64
    product, rel-L2 <= 1e-5; strided rows (lda > N), ragged N / K / M; accumulate mode; two
    calls bitwise equal (deterministic).  Bar 1e-5: the split's 2^-17 product rounding is the
    same relative error whatever M (random-sign terms: measured 4.4e-6 at M = 10^5)."""
    from waveformer_amd import ops
    a = seeded_randn((M, N + pad), 40)[:, :N].cuda()
    b = seeded_randn((M, K), 41).cuda()
    want = a.double().t().mm(b.double())
    got = ops.gemm_tn(a, b)
    assert C.rel_l2(got, want) <= 1e-5
    assert torch.equal(got, ops.gemm_tn(a, b))
    acc = torch.ones((N, K), device="cuda")
    ops.gemm_tn(a, b, out=acc, accumulate=True)
    assert C.rel_l2(acc, want + 1) <= 1e-5


@pytest.mark.parametrize("cin,cout,S,bias", [(96, 48, (6, 5, 7), True), (48, 4, (8, 8, 8), True),
                                             (384, 192, (4, 4, 4), False), (4, 48, (5, 6, 7), True)])
def test_conv1x1_and_convtranspose2_autograd(cin, cout, S, bias):
    """The decoder's 1x1 convs (wfa.Conv1x1Fn) and 2^3 transposed convs (wfa.ConvT2Fn) in
    training: forward and input gradient on the streaming MFMA GEMM (bf16x3 operands; K < 8 --
    the 48 -> 4 head's input gradient, the 4 -> 48 stem conv's forward -- on the small-K fp32
    kernel wf_linear_smallk_fwd), weight gradient on
    wf_gemm_tn, bias by column sums -- against fp64 CPU autograd: rel-L2 <= 1e-5 for the bf16x3
    products (operands carried to 16 mantissa bits, fp32 accumulation; round 5 held the fp32
    GEMMs to 2e-6), 2e-6 for the bias column sums."""
    from waveformer_amd import autograd as wfa
    x = seeded_randn((2, cin) + S, 50)
    conv = torch.nn.Conv3d(cin, cout, 1, bias=bias)
    convt = torch.nn.ConvTranspose3d(cin, cout, 2, stride=2, bias=bias)
    for m, seed in ((conv, 51), (convt, 52)):
        with torch.no_grad():
            for prm in m.parameters():
                prm.copy_(seeded_randn(tuple(prm.shape), seed) * 0.1)
        md = m.double()
        xd = x.double().requires_grad_(True)
        yd = md(xd)
        g = seeded_randn(tuple(yd.shape), seed + 10)
        yd.backward(g.double())
        mc = type(m)(*([cin, cout, 1] if m is conv else [cin, cout, 2]),
                     **({} if m is conv else {"stride": 2}), bias=bias).cuda()
        mc.load_state_dict({k: v.float() for k, v in md.state_dict().items()})
        xg = x.cuda().requires_grad_(True)
        y = wfa.conv_train(mc, xg)
        y.backward(g.cuda())
        assert C.rel_l2(y, yd.detach()) <= 1e-5
        assert C.rel_l2(xg.grad, xd.grad) <= 1e-5
        assert C.rel_l2(mc.weight.grad, md.weight.grad) <= 1e-5
        if bias:
            assert C.rel_l2(mc.bias.grad, md.bias.grad) <= 2e-6
        m.float()


@pytest.mark.parametrize("C_,B,S", [(192, 2, (9, 10, 17)), (96, 1, (16, 16, 16)), (8, 3, (2, 3, 5))])
def test_group_norm_cl_autograd(C_, B, S):
    """ProjectionUpsample.norm (GroupNorm(C, C), affine) in training on the channel-last path
    (wfa.GroupNormCLFn: HIP statistics, one-pass affine apply, the norm_act backward with
    slope 1): output, input / weight / bias gradients against fp64 CPU autograd, rel-L2 1e-5."""
    from waveformer_amd import autograd as wfa
    x = seeded_randn((B, C_) + S, 70) * 2 + 0.5
    norm = torch.nn.GroupNorm(C_, C_)
    with torch.no_grad():
        norm.weight.copy_(seeded_randn((C_,), 71))
        norm.bias.copy_(seeded_randn((C_,), 72))
    g = seeded_randn((B, C_) + S, 73)
    nd = torch.nn.GroupNorm(C_, C_).double()
    nd.load_state_dict({k: v.double() for k, v in norm.state_dict().items()})
    xd = x.double().requires_grad_(True)
    yd = nd(xd)
    yd.backward(g.double())
    ng = norm.cuda()
    xg = x.cuda().contiguous(memory_format=torch.channels_last_3d).requires_grad_(True)
    y = wfa.group_norm_cl(ng, xg)
    assert y.is_contiguous(memory_format=torch.channels_last_3d)
    y.backward(g.cuda())
    assert C.rel_l2(y, yd.detach()) <= 1e-5
    assert C.rel_l2(xg.grad, xd.grad) <= 1e-5
    assert C.rel_l2(ng.weight.grad, nd.weight.grad) <= 1e-5
    assert C.rel_l2(ng.bias.grad, nd.bias.grad) <= 1e-5


@pytest.mark.parametrize("C_,B,S", [(192, 2, (9, 20, 17)), (32, 1, (3, 5, 40)), (96, 1, (12, 9, 8)),
                                    (48, 2, (5, 6, 7)), (64, 1, (1, 1, 1))])
def test_dwconv3d_autograd(C_, B, S):
    """Depthwise 3^3 conv in training (wfa.DWConv3dK3: ProjectionUpsample.conv1, CCF_FFN.dwconv
    backward): forward and input gradient on the z-streaming LDS kernel (the gradient with the
    taps mirrored, round 5), weight gradient on the z-streaming partial-tile kernel summed in a
    fixed order (C % 32 == 0; the per-position kernels otherwise, C = 48 here) -- against fp64
    CPU autograd, rel-L2 <= 2e-6 (exact fp32 arithmetic); the weight gradient bitwise
    repeatable; ragged tiles, a single-position volume."""
    from waveformer_amd import autograd as wfa
    x = seeded_randn((B, C_) + S, 60)
    w = seeded_randn((C_, 1, 3, 3, 3), 61) * 0.3
    b = seeded_randn((C_,), 62)
    g = seeded_randn((B, C_) + S, 63)
    xd, wd, bd = (t.double().requires_grad_(True) for t in (x, w, b))
    yd = F.conv3d(xd, wd, bd, padding=1, groups=C_)
    yd.backward(g.double())
    xg, wg, bg = (t.cuda().requires_grad_(True) for t in (x, w, b))
    y = wfa.DWConv3dK3.apply(xg, wg, bg)
    y.backward(g.cuda())
    assert C.rel_l2(y, yd.detach()) <= 2e-6
    assert C.rel_l2(xg.grad, xd.grad) <= 2e-6
    assert C.rel_l2(wg.grad, wd.grad) <= 2e-6
    assert C.rel_l2(bg.grad, bd.grad) <= 2e-6
    w1 = wg.grad.clone()
    wg.grad = None
    wfa.DWConv3dK3.apply(xg, wg, bg).backward(g.cuda())
    assert torch.equal(wg.grad, w1)


@pytest.mark.parametrize("C_,B,S,sig", [
    (48, 2, (12, 12, 12), True),    # decoder2 level shapes (C 48)
    (96, 1, (6, 7, 9), True),       # ragged planes / rows, z not a multiple of the 8-plane tile
    (192, 2, (3, 3, 3), True),      # decoder4 (C 192), fewer positions than one workgroup
    (48, 1, (17, 5, 4), False),     # hf_refinement.use_sigmoid False
    (24, 1, (4, 9, 10), True),      # C / 4 not dividing 256 evenly
])
def test_hf_refinement_fused_vs_module(C_, B, S, sig):
    """ops.hf_refine (csrc/hfref.hip, two passes over the 7 detail tensors of a level) against
    HFRefinementRes's own PyTorch forward in fp64 on the CPU (idwt_upsample.py:39-50), detail
    tensors as the DWT hands them over: channel-last views of one (8, B, D, H, W, C) band
    buffer.  All-fp32 kernel arithmetic: rel-L2 <= 1e-5."""
    import waveformer_amd.network_models as NM
    from waveformer_amd import ops
    cfg = None if sig else {"hf_refinement": {"use_sigmoid": False}}
    m = NM.HFRefinementRes(C_, network_config=cfg)
    with torch.no_grad():
        for i, p in enumerate(m.parameters()):
            p.copy_(seeded_randn(tuple(p.shape), 40 + i) * (0.5 if p.dim() > 1 else 0.2)
                    + (1.0 if p.dim() == 1 and i == 2 else 0.0))
    bands = (seeded_randn((8, B) + S + (C_,), 7) * 1.5 + 0.2)
    det = {k: bands[i + 1].permute(0, 4, 1, 2, 3) for i, k in enumerate(ops.DETAIL_KEYS)}
    md = m.double()
    with torch.no_grad():
        want = {k: md(v.double()) for k, v in det.items()}
    m = m.float().cuda()
    bc = bands.cuda()
    dc = {k: bc[i + 1].permute(0, 4, 1, 2, 3) for i, k in enumerate(ops.DETAIL_KEYS)}
    with torch.no_grad():
        assert m.fast_ok(dc["aad"])
        got = ops.hf_refine(dc, m)
    for k in ops.DETAIL_KEYS:
        assert C.rel_l2(got[k], want[k]) <= 1e-5, k


@pytest.mark.parametrize("B,Cin,Cout,S", [
    (1, 4, 48, (20, 18, 70)),     # encoder1's first conv (Cin 4: one partial 16-channel slice)
    (2, 96, 48, (9, 13, 33)),     # decoder conv_block conv1 (2C -> C), ragged x / y tiles
    (1, 48, 48, (8, 5, 17)),
    (1, 192, 96, (6, 7, 11)),     # Cout 96 = two 48-channel blocks
    (1, 384, 192, (8, 8, 8)),     # decoder4.conv_lf_block shape
    (1, 20, 32, (3, 4, 5)),       # Cin % 16 != 0, Cout % 48 != 0 (16-channel blocks)
])
def test_conv3d_k3_wgrad_vs_cpu(B, Cin, Cout, S):
    """wf_conv3d_k3_wgrad (csrc/conv3d_wgrad.hip) against torch.nn.grad.conv3d_weight in fp64
    on the CPU: bf16x3 operands, fp32 accumulation over B*D*H*W positions: rel-L2 <= 1e-5;
    two runs bit-identical (no atomics)."""
    from waveformer_amd import ops
    x = seeded_randn((B, Cin) + S, 11) * 2 + 0.1
    g = seeded_randn((B, Cout) + S, 12)
    want = torch.nn.grad.conv3d_weight(x.double(), (Cout, Cin, 3, 3, 3), g.double(), padding=1)
    xc = x.cuda().contiguous(memory_format=torch.channels_last_3d)
    gc = g.cuda().contiguous(memory_format=torch.channels_last_3d)
    got = ops.conv3d_k3_wgrad(xc, gc, (Cout, Cin, 3, 3, 3))
    assert C.rel_l2(got, want) <= 1e-5
    assert torch.equal(got, ops.conv3d_k3_wgrad(xc, gc, (Cout, Cin, 3, 3, 3)))


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("B,C_,S", [(2, 48, (9, 10, 11)), (1, 96, (4, 5, 6)), (2, 16, (16, 3, 7))])
def test_norm_act_autograd_vs_torch(mode, B, C_, S):
    """autograd.NormActFn (InstanceNorm3d(affine=False) + residual (none / plain / normed) +
    LeakyReLU, forward wf_instnorm_stats_cl + wf_norm_act_cl, backward wf_norm_act_bwd_cl)
    against the framework's InstanceNorm3d / LeakyReLU in fp64 on the CPU: forward and both
    input gradients rel-L2 <= 1e-5."""
    from waveformer_amd import autograd as wfa
    a = seeded_randn((B, C_) + S, 61) * 2 + 0.3
    r = seeded_randn((B, C_) + S, 62) * 1.5 - 0.2
    gy = seeded_randn((B, C_) + S, 63)
    ad, rd = a.double().requires_grad_(True), r.double().requires_grad_(True)
    z = F.instance_norm(ad, eps=1e-5)
    if mode == 1:
        z = z + rd
    elif mode == 2:
        z = z + F.instance_norm(rd, eps=1e-5)
    want = F.leaky_relu(z, 0.01)
    want.backward(gy.double())
    ac = a.cuda().contiguous(memory_format=torch.channels_last_3d).requires_grad_(True)
    rc = r.cuda().contiguous(memory_format=torch.channels_last_3d).requires_grad_(True)
    got = wfa.norm_act(ac, rc if mode else None, 0.01, 1e-5, 1e-5, normed_residual=mode == 2)
    got.backward(gy.cuda())
    assert C.rel_l2(got, want) <= 1e-5
    assert C.rel_l2(ac.grad, ad.grad) <= 1e-5
    if mode:
        assert C.rel_l2(rc.grad, rd.grad) <= 1e-5


def test_channel_last_copy_cat_and_subvoxel_scatter():
    """layout.hip: wf_copy_cl (channel slices of channels_last_3d tensors), ops.cat_cl (mixed
    layouts) and wf_subvoxel_scatter_cl (ConvTranspose3d k = s = 2 placement + bias) against
    the torch ops they replace, bit for bit."""
    from waveformer_amd import ops
    cl = torch.channels_last_3d
    a = seeded_randn((2, 8, 5, 6, 7), 41).cuda().contiguous(memory_format=cl)
    b = seeded_randn((2, 12, 5, 6, 7), 42).cuda().contiguous(memory_format=cl)
    c = seeded_randn((2, 4, 5, 6, 7), 43).cuda()  # NCDHW: the torch-copy fallback
    got = ops.cat_cl([a, b, c])
    assert got.is_contiguous(memory_format=cl)
    assert torch.equal(got, torch.cat([a, b, c], 1))
    buf = torch.full((2, 20, 5, 6, 7), 3.0, device="cuda").contiguous(memory_format=cl)
    ops.copy_cl(b, buf[:, 4:16])
    assert torch.equal(buf[:, 4:16], b) and torch.all(buf[:, :4] == 3) and torch.all(buf[:, 16:] == 3)
    # transposed conv k = s = 2 as rows @ W, scattered into the first Cout channels
    B, Cin, Cout, d, h, w = 2, 16, 12, 3, 4, 5
    x = seeded_randn((B, Cin, d, h, w), 44).cuda()
    tc = torch.nn.ConvTranspose3d(Cin, Cout, 2, 2).cuda()
    with torch.no_grad():
        tc.bias.copy_(seeded_randn((Cout,), 45).cuda())
        want = tc(x)
    rows = x.permute(0, 2, 3, 4, 1).reshape(-1, Cin)
    g = rows @ tc.weight.detach().permute(0, 2, 3, 4, 1).reshape(Cin, 8 * Cout)
    dst = torch.full((B, Cout + 4, 2 * d, 2 * h, 2 * w), 5.0, device="cuda").contiguous(memory_format=cl)
    ops.subvoxel_scatter_cl(g, tc.bias.detach(), dst)
    assert C.rel_l2(dst[:, :Cout], want) <= 1e-5
    assert torch.all(dst[:, Cout:] == 5.0)


@pytest.mark.parametrize("B,Cin,Cout,d,h,w", [(2, 16, 12, 3, 4, 5), (1, 144, 48, 6, 6, 6),
                                              (2, 8, 4, 1, 1, 3), (1, 96, 48, 5, 7, 9)])
def test_convtranspose2_gemm_subvoxel_epilogue(B, Cin, Cout, d, h, w):
    """wf_convtranspose2_cl: ConvTranspose3d(k = s = 2) as one streaming MFMA GEMM whose
    epilogue stores the sub-voxels + bias into a channel slice of a wider channel-last buffer,
    against torch's fp32 transposed conv (bf16x3 operands: fp32-faithful, rel-L2 <= 1e-5);
    ragged row counts (M % 16 != 0) and one- and multi-chunk column splits included."""
    from waveformer_amd import ops
    cl = torch.channels_last_3d
    x = seeded_randn((B, Cin, d, h, w), 51).cuda()
    tc = torch.nn.ConvTranspose3d(Cin, Cout, 2, 2).cuda()
    with torch.no_grad():
        tc.weight.copy_(seeded_randn(tuple(tc.weight.shape), 52).cuda() * 0.1)
        tc.bias.copy_(seeded_randn((Cout,), 53).cuda())
        want = tc(x)
    dst = torch.full((B, Cout + 8, 2 * d, 2 * h, 2 * w), 5.0, device="cuda").contiguous(memory_format=cl)
    ops.convtranspose2_cl(x, tc.weight.detach(), tc.bias.detach(), dst)
    assert C.rel_l2(dst[:, :Cout], want) <= 1e-5
    assert torch.all(dst[:, Cout:] == 5.0)
    dst2 = ops.empty_cl(B, Cout, 2 * d, 2 * h, 2 * w, x.device)  # dense, no bias, cl input
    ops.convtranspose2_cl(x.contiguous(memory_format=cl), tc.weight.detach(), None, dst2)
    assert C.rel_l2(dst2 + tc.bias.detach().view(1, -1, 1, 1, 1), want) <= 1e-5


def test_unetr_up_block_skip_in_place():
    """UnetrUpBlock's fast path with the skip produced into its concat buffer (opt-in
    `skip_in_place=True`, as the backbone's encoder1 does) and with a free-standing skip: the
    same result as the reference composition torch.cat((ConvTranspose3d(x), skip), 1) -> conv
    block.  Without the flag a skip that merely views such a buffer leaves the caller's storage
    untouched."""
    from waveformer_amd import ops
    from waveformer_amd.blocks import UnetrUpBlock
    torch.manual_seed(0)
    blk = UnetrUpBlock(3, 24, 8, 3, 2, "instance", res_block=True).cuda().eval()
    x = seeded_randn((1, 24, 4, 4, 4), 61).cuda()
    skip = seeded_randn((1, 8, 8, 8, 8), 62).cuda()
    buf = ops.empty_cl(1, 16, 8, 8, 8, x.device)
    buf[:, 8:].copy_(skip)
    view = buf[:, 8:]
    assert ops.cl_parent(view, 8) is buf or ops.cl_parent(view, 8).data_ptr() == buf.data_ptr()
    with torch.no_grad():
        before = buf.clone()
        got_view = blk(x, view)                       # no opt-in: buf must not be written
        assert torch.equal(buf, before)
        got_inplace = blk(x, view, skip_in_place=True)
        got_free = blk(x, skip)
        tc = blk.transp_conv.conv
        ref_in = torch.cat((tc(x), skip), 1)
        want = blk.conv_block(ref_in)
    assert C.rel_l2(got_free, want) <= 1e-5
    assert C.rel_l2(got_inplace, want) <= 1e-5
    assert C.rel_l2(got_view, want) <= 1e-5


def test_norm_act_linear_residual_fold():
    """ops.norm_act_lin (wf_moments_cl + wf_norm_act_lin_cl): the norm3'ed 4 -> 48 1x1
    residual of encoder1 folded into per-sample weights from x's fp64 moments, against the
    materialised composition in fp64 (B = 2 samples with different means / scales, written into
    a channel slice of a wider buffer); and UnetResBlock(4 -> 48) writing through `out=`."""
    from waveformer_amd import ops
    from waveformer_amd.blocks import UnetResBlock
    B, K, Cc, S = 2, 4, 48, 10
    x = seeded_randn((B, K, S, S, S), 71)
    x[0] = x[0] * 3.0 + 1.5
    x[1] = x[1] * 0.5 - 2.0
    a = seeded_randn((B, Cc, S, S, S), 72)
    w = seeded_randn((Cc, K, 1, 1, 1), 73) * 0.3
    bias = seeded_randn((Cc,), 74)
    xd, ad = x.double(), a.double()
    r = F.conv3d(xd, w.double(), bias.double())
    want = F.leaky_relu(F.instance_norm(ad, eps=1e-5) + F.instance_norm(r, eps=1e-5), 0.01)
    cl = torch.channels_last_3d
    ac = a.cuda().contiguous(memory_format=cl)
    buf = torch.full((B, Cc + 8, S, S, S), 7.0, device="cuda").contiguous(memory_format=cl)
    got = ops.norm_act_lin(ac, ops.instnorm_stats(ac, 1e-5), x.cuda(), w.cuda(), bias.cuda(),
                           1e-5, slope=0.01, out=buf[:, 8:])
    assert got.data_ptr() == buf[:, 8:].data_ptr()
    assert C.rel_l2(got.double().cpu(), want) <= 2e-6
    assert torch.all(buf[:, :8] == 7.0)
    torch.manual_seed(0)
    blk = UnetResBlock(3, K, Cc, 3, 1, "instance").cuda().eval()
    with torch.no_grad():
        free = blk(x.cuda())
        into = blk(x.cuda(), out=buf[:, 8:])
    assert into.data_ptr() == buf[:, 8:].data_ptr()
    # the conv epilogue's InstanceNorm sums are fp64 atomics: last-bit run-to-run differences
    assert C.rel_l2(into, free) <= 1e-6


@pytest.mark.parametrize("B,K,N,S", [(2, 48, 3, 9), (1, 8, 16, 17), (1, 96, 1, 5)])
def test_unet_out_block_head_kernel(B, K, N, S):
    """wf_conv1x1_head_cl (UnetOutBlock's 1x1x1 conv, channel-last in -> NCDHW logits) vs
    torch's fp32 conv3d; ragged last position tile (S^3 % 256 != 0); the module's fast path."""
    from waveformer_amd import ops
    from waveformer_amd.blocks import UnetOutBlock
    x = seeded_randn((B, K, S, S, S), 81).cuda().contiguous(memory_format=torch.channels_last_3d)
    blk = UnetOutBlock(3, K, N).cuda().eval()
    with torch.no_grad():
        want = F.conv3d(x.contiguous(), blk.conv.conv.weight, blk.conv.conv.bias)
        got = blk(x)
    assert got.is_contiguous()
    assert C.rel_l2(got, want) <= 1e-6
    got2 = ops.conv1x1_head(x, blk.conv.conv.weight, None)
    assert C.rel_l2(got2 + blk.conv.conv.bias.view(1, -1, 1, 1, 1), want) <= 1e-6


@pytest.mark.parametrize("src,dst,ac", [((3, 4, 5), (6, 8, 10), True), ((4, 4, 4), (16, 16, 16), True),
                                        ((5, 3, 4), (7, 9, 8), False)])
def test_upsample_add_cl(src, dst, ac):
    """wf_upsample_trilinear_add_cl: out += F.interpolate(x, trilinear), channel-last."""
    from waveformer_amd import ops
    cl = torch.channels_last_3d
    x = seeded_randn((2, 8) + src, 82).cuda().contiguous(memory_format=cl)
    base = seeded_randn((2, 8) + dst, 83).cuda().contiguous(memory_format=cl)
    want = base + F.interpolate(x, size=dst, mode="trilinear", align_corners=ac)
    got = ops.upsample_add_cl(x, base.clone(memory_format=cl), ac)
    assert C.rel_l2(got, want) <= 1e-6
    assert C.rel_l2(ops.upsample_cl(x, dst, ac),
                    F.interpolate(x, size=dst, mode="trilinear", align_corners=ac)) <= 1e-6


@pytest.mark.parametrize("B,C_,S", [(2, 48, 48), (1, 96, 9), (1, 16, 37)])
def test_conv3d_k3_fp16_input_bitwise(B, C_, S):
    """fp16 policy: conv1's norm1 + lrelu stored fp16 (wf_norm_act_h_cl) and conv2 on the
    fp16-input kernel (wf_conv3d_k3_fwd_xh) give bitwise the output of the fp32 path, whose
    staging rounds the same values to fp16; the stored operands are torch's fp16 rounding."""
    from waveformer_amd import ops
    from waveformer_amd.blocks import UnetResBlock
    cl = torch.channels_last_3d
    a = seeded_randn((B, C_, S, S, S), 91).cuda().contiguous(memory_format=cl)
    w = seeded_randn((48, C_, 3, 3, 3), 92).cuda() * 0.05
    bias = seeded_randn((48,), 93).cuda()
    st = ops.instnorm_stats(a, 1e-5)
    with ops.precision("fp16"):
        h32 = ops.norm_act(a, st, slope=0.01)
        h16 = ops.norm_act_h(a, st, slope=0.01)
        assert h16.dtype == torch.float16 and torch.equal(h16, h32.half())
        y32, s32 = ops.conv3d_k3(h32, w, bias, norm_eps=1e-5)
        y16, s16 = ops.conv3d_k3(h16, w, bias, norm_eps=1e-5)
    # no split-K with 4- or 8-row tiles (the fp16-input path uses 8 rows at W > 32; split-K's
    # fp32 atomics add in any order): bitwise
    if B * S * ((S + 7) // 8) >= 512:
        assert torch.equal(y32, y16)
    assert C.rel_l2(y16, y32) <= 1e-6
    assert C.rel_l2(s16, s32) <= 1e-6
    # the block's fast path at fp16 (norm_act_h inside) vs the same block at bf16x3
    torch.manual_seed(0)
    blk = UnetResBlock(3, C_, 48, 3, 1, "instance").cuda().eval()
    with torch.no_grad():
        ref = blk(a)
        with ops.precision("fp16"):
            got = blk(a)
    assert C.rel_l2(got, ref) <= 5e-3


@pytest.mark.parametrize("B,C_,S", [(2, 64, 12), (1, 96, 9), (1, 32, 17)])
def test_dwconv3d_fused_channel_stats(B, C_, S):
    """wf_dwconv3d_stats_cl: the depthwise conv's output (same kernel as wf_dwconv3d_cl, bit
    for bit) and its per-(sample, channel) mean / rstd from the epilogue vs instnorm_stats of
    the stored output (fp64 sums both ways)."""
    from waveformer_amd import ops
    cl = torch.channels_last_3d
    x = seeded_randn((B, C_, S, S, S), 97).cuda().contiguous(memory_format=cl)
    w = seeded_randn((C_, 1, 3, 3, 3), 98).cuda() * 0.2
    b = seeded_randn((C_,), 99).cuda()
    y0 = ops.dwconv3d_cl(x, w, b)
    y1, st = ops.dwconv3d_cl(x, w, b, norm_eps=1e-5)
    assert torch.equal(y0, y1)
    ref = ops.instnorm_stats(y1, 1e-5)
    assert C.rel_l2(st, ref) <= 1e-6
    want = F.conv3d(x.contiguous(), w, b, padding=1, groups=C_)
    assert C.rel_l2(y1, want) <= 1e-6




# (precision, Cin, Cout, (B, D, H, W), fp16 input, statistics): shapes that take the wide-chunk
# kernel (W > 32, Cout % 48 == 0, >= 512 workgroups of the 4-row plan; every Cin with
# WF_CONV_WIDE_MINCIN=1); Cin 40 / 104 = an odd number of 8-channel chunks, Cout 96 = two column
# blocks, W 70 / 100 = ragged x tiles
_WIDE_CASES = (("fp16", 96, 48, (2, 24, 32, 70), False, True),
               ("bf16", 48, 96, (1, 32, 24, 100), False, False),
               ("fp16", 40, 48, (2, 32, 32, 36), False, True),
               ("fp16", 48, 48, (2, 64, 48, 40), True, True),
               ("bf16x3", 96, 48, (2, 24, 32, 70), False, True),
               ("bf16x3", 104, 96, (1, 20, 40, 100), False, False))
_WIDE_CHILD = r"""
import sys, torch
sys.path.insert(0, '.')
from tests.test_gpu_decoder import _wide_outputs
torch.save(_wide_outputs(), sys.argv[1])
print("WIDE_CHILD_OK")
"""


def _wide_outputs():
    from waveformer_amd import ops
    outs = []
    for i, (prec, cin, cout, shp, xh, stats) in enumerate(_WIDE_CASES):
        B, D, H, W = shp
        x = (seeded_randn((B, cin, D, H, W), 150 + i) + 0.25).cuda()
        x = x.contiguous(memory_format=torch.channels_last_3d)
        if xh:
            x = x.half().contiguous(memory_format=torch.channels_last_3d)
        w = (seeded_randn((cout, cin, 3, 3, 3), 160 + i) * (cin * 27) ** -0.5).cuda()
        b = seeded_randn((cout,), 170 + i).cuda()
        with ops.precision(prec):
            r = ops.conv3d_k3(x, w, b, norm_eps=1e-5 if stats else None)
        outs.append(tuple(t.cpu() for t in r) if stats else (r.cpu(),))
    return outs


def _wide_child(tmp_path, name, **env_over):
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = str(tmp_path / name)
    env = dict(os.environ, PYTHONPATH=repo, **env_over)
    r = subprocess.run([sys.executable, "-c", _WIDE_CHILD, dst], cwd=repo, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "WIDE_CHILD_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    return torch.load(dst, weights_only=True)


def test_conv3d_k3_wide_chunks_bitwise(tmp_path):
    """conv3d_k3w_kernel (16 channels per 64-B load, 8-wave workgroups of 8 x 64 outputs; one
    8-channel chunk's hi / lo per step under bf16x3) runs each output's K reduction in the
    8-channel kernels' order on the same operands: outputs bitwise equal to WF_CONV_WIDE=0, the
    fused InstanceNorm statistics equal to fp32 summation-order level (both sides in child
    processes: the switches are read once per process); the fp64 CPU convolution at the bars."""
    wide = _wide_child(tmp_path, "wide.pt", WF_CONV_WIDE="1", WF_CONV_WIDE_MINCIN="1")
    narrow = _wide_child(tmp_path, "narrow.pt", WF_CONV_WIDE="0")
    for case, g, want in zip(_WIDE_CASES, wide, narrow):
        assert torch.equal(g[0], want[0]), (case, float((g[0] - want[0]).abs().max()))
        if len(g) > 1:
            assert C.rel_l2(g[1], want[1]) <= 1e-6, case
    for i in (1, 5):  # bf16 and bf16x3 against the fp64 convolution
        prec, cin, cout, (B, D, H, W), _, _ = _WIDE_CASES[i]
        x = seeded_randn((B, cin, D, H, W), 150 + i) + 0.25
        w = seeded_randn((cout, cin, 3, 3, 3), 160 + i) * (cin * 27) ** -0.5
        b = seeded_randn((cout,), 170 + i)
        want = F.conv3d(x.double(), w.double(), b.double(), padding=1)
        assert C.rel_l2(wide[i][0], want) <= (1e-5 if prec == "bf16x3" else 1e-2), prec


@pytest.mark.parametrize("ac", [True, False])
@pytest.mark.parametrize("B,C_,src,s", [(2, 32, (5, 6, 7), 2), (1, 192, (6, 5, 7), 4),
                                         (1, 96, (3, 9, 12), 2), (2, 64, (4, 4, 5), (2, 3, 4)),
                                         (1, 32, (2, 2, 20), 2), (1, 32, (3, 4, 4), (1, 2, 2))])
def test_upsample_dwconv3d_fused_bitwise(B, C_, src, s, ac):
    """ProjectionUpsample.conv1 fused (wf_upsample_dwconv3d_stats_cl): bitwise the two-kernel
    path (wf_upsample_trilinear_cl, then wf_dwconv3d_stats_cl) in the output and in the
    GroupNorm statistics, and within fp32 rounding of F.interpolate + F.conv3d in fp64."""
    from waveformer_amd import ops
    st = (s,) * 3 if isinstance(s, int) else s
    dst = tuple(a * b for a, b in zip(src, st))
    x = seeded_randn((B, C_) + src, 12).cuda().contiguous(memory_format=torch.channels_last_3d)
    w = seeded_randn((C_, 1, 3, 3, 3), 13).cuda() * 0.3
    b = seeded_randn((C_,), 14).cuda()
    got, gst = ops.upsample_dwconv3d_cl(x, dst, w, b, 1e-5, ac)
    up = ops.upsample_cl(x, dst, ac)
    want, wst = ops.dwconv3d_cl(up, w, b, norm_eps=1e-5)
    assert torch.equal(got, want)
    assert torch.equal(gst, wst)
    ref = F.conv3d(F.interpolate(x.double().cpu(), size=dst, mode="trilinear", align_corners=ac),
                   w.double().cpu(), b.double().cpu(), padding=1, groups=C_)
    assert C.rel_l2(got, ref) <= 1e-6


def test_upsample_dwconv3d_declines_unsupported():
    from waveformer_amd import ops
    x = torch.zeros((1, 48, 4, 4, 4), device="cuda")
    w, b = torch.zeros((48, 1, 3, 3, 3), device="cuda"), torch.zeros(48, device="cuda")
    assert ops.upsample_dwconv3d_cl(x, (8, 8, 8), w, b, 1e-5) is None      # C % 32
    x = torch.zeros((1, 32, 4, 4, 4), device="cuda")
    w, b = torch.zeros((32, 1, 3, 3, 3), device="cuda"), torch.zeros(32, device="cuda")
    assert ops.upsample_dwconv3d_cl(x, (8, 8, 6), w, b, 1e-5) is None      # x factor < 2
    assert ops.upsample_dwconv3d_cl(x, (8, 6, 8), w, b, 1e-5) is None      # y factor < 2
    assert ops.upsample_dwconv3d_cl(x, (5, 8, 8), w, b, 1e-5) is not None  # any z factor
