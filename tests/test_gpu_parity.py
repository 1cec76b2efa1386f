"""GPU parity: the HIP path (libwaveformer_hip.so through waveformer_amd) against the oracle
and against the reference's own outputs (tests/golden/ref_fixtures.npz).

Tolerances (stated per check):
  * fp32-only kernels (DWT, IDWT, multi-scale fuse, proj_out LayerNorm, PatchEmbed):
    rel-L2 <= 1e-5 against the oracle in fp32 -- they do the reference's arithmetic in fp32.
  * kernels with MFMA operands (qkv / proj / QK^T / PV / pwconv / fc / PatchMerging
    reduction; fp32 accumulation, fp32 LayerNorm / softmax / residual):
      - default precision "bf16x3" (split hi/lo bf16 operands, fp32-faithful): rel-L2 <= 5e-5
        per op and per Block, <= 1e-4 through the encoder and the full model;
      - fast precision "bf16": rel-L2 <= 1e-2 for a single op, <= 2e-2 through a Block,
        <= 3e-2 through the encoder (bf16 rounds to 2^-9 = 2e-3 relative per operand);
      - config 5's "fp16" (fp16 operands on the f16 MFMA pipes, fp32 accumulation and fp32
        LayerNorm / softmax / residual; window attention and the skip-feature convolutions keep
        the bf16x3 split, ops.FP16_SPLIT_OPS): rel-L2 <= 2e-3 for a single op, <= 3e-3 through a
        Block, <= 5e-3 through the encoder and the full model (fp16 rounds to 2^-12 = 2.4e-4
        relative per operand, 8x finer than bf16).
  * end-to-end metric (BASELINE.json north_star): Dice of TC / WT / ET of the full model's
    argmax labels at 128^3 x 4 >= 1 - 1e-3 against the reference's labels.
"""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_waveformer as R
from oracle.weight_rule import seeded_randn
from tests import cases as C

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from waveformer_amd import _lib
    _lib.load()  # fail loudly if the HIP library is missing
    torch.backends.cuda.matmul.allow_tf32 = False
    yield


def cuda(t):
    return t.to(DEV)


# ------------------------------------------------------------------------------ op level
@pytest.mark.parametrize("C_", [8, 24, 48, 96, 192, 384, 40])
@pytest.mark.parametrize("ln", [False, True])
def test_dwt_haar_vs_oracle(C_, ln):
    from waveformer_amd import ops
    x = seeded_randn((2, 8, 6, 10, C_), 1) * 3 + 0.5
    lw, lb = seeded_randn((C_,), 2) * 0.2 + 1, seeded_randn((C_,), 3) * 0.1
    xin = F.layer_norm(x, [C_], lw, lb, 1e-6) if ln else x
    ll_ref, det_ref = R.dwt3_level(xin.permute(0, 4, 1, 2, 3), "db1")
    bands = ops.dwt3d_haar(cuda(x), (cuda(lw), cuda(lb), 1e-6) if ln else None)
    ll, det = ops.bands_to_coeffs(bands)
    assert C.rel_l2(ll, ll_ref) <= 1e-5
    for k in R.DETAIL_KEYS:
        assert C.rel_l2(det[k], det_ref[k]) <= 1e-5, k


@pytest.mark.parametrize("C_", [8, 48, 96, 192, 40])
@pytest.mark.parametrize("ln", [False, True])
def test_dwt_haar_ll_only_bitwise(C_, ln):
    """wf_dwt3d_haar_fwd_ll (the Blocks whose detail bands are discarded) is bitwise band 0 of
    the 8-band kernel, with and without the fused norm1."""
    from waveformer_amd import ops
    x = cuda(seeded_randn((2, 8, 6, 10, C_), 11) * 3 + 0.5)
    lnp = (cuda(seeded_randn((C_,), 12) * 0.2 + 1), cuda(seeded_randn((C_,), 13) * 0.1), 1e-6)
    bands = ops.dwt3d_haar(x, lnp if ln else None)
    ll = ops.dwt3d_haar_ll(x, lnp if ln else None)
    assert ll.shape == bands[0].shape and torch.equal(ll, bands[0])


@pytest.mark.parametrize("B,cin,S", [(2, 4, (32, 16, 128)), (1, 1, (20, 12, 36))])
def test_patch_embed_ll_fused(B, cin, S):
    """wf_patch_embed_ll_fwd: the stage-1 activation -- Cin = 4 on the matrix cores (bf16x3
    products: rel-L2 <= 1e-5 against the fp64 convolution and the fp32-FMA wf_patch_embed_fwd),
    Cin = 1 bitwise equal to wf_patch_embed_fwd -- and the first Block's level-1 LL equal to the
    LL-only DWT of that activation (norm1 fused) up to the LayerNorm moments' summation order
    (rel-L2 <= 1e-6)."""
    from waveformer_amd import ops
    x = cuda(seeded_randn((B, cin) + S, 15))
    w = cuda(seeded_randn((48, cin, 2, 2, 2), 16) * 0.2)
    bias = cuda(seeded_randn((48,), 17))
    ln = (cuda(seeded_randn((48,), 18) * 0.2 + 1), cuda(seeded_randn((48,), 19) * 0.1), 1e-6)
    out, ll = ops.patch_embed_ll(x, w, bias, ln)
    ref = ops.patch_embed(x, w, bias)
    if cin == 1:
        assert torch.equal(out, ref)
    else:
        exact = torch.nn.functional.conv3d(x.double().cpu(), w.double().cpu(), bias.double().cpu(),
                                           stride=2).permute(0, 2, 3, 4, 1)
        assert C.rel_l2(out.double().cpu(), exact) <= 1e-5
        assert C.rel_l2(out, ref) <= 1e-5
    assert C.rel_l2(ll, ops.dwt3d_haar_ll(out, ln)) <= 1e-6


def test_encoder_block_hf_skip_keeps_outputs():
    """The encoder runs every Block but a stage's last on the LL-only DWT in inference (the
    first one on the LL the fused PatchEmbed kernel forms); its outputs and the returned hf
    dicts (the last Blocks') equal a run that computes every Block's detail bands (the flag
    forced off) up to the fused kernel's LayerNorm-moment rounding, carried through the four
    stages (rel-L2 <= 1e-5; measured 1.6e-6; the encoder's bar against the oracle is 1e-4)."""
    import waveformer_amd.network_models as NM
    from waveformer_amd.network_models import wave_helper as WH
    torch.manual_seed(0)
    m = NM.MultiscaleTransformer(img_size=(32, 32, 32), in_chans=4,
                                 num_heads=[1, 1, 1, 1]).eval().to(DEV)
    x = cuda(seeded_randn((1, 4, 32, 32, 32), 14))
    with torch.no_grad():
        outs, hf = m(x)
        orig = WH.Block._ll_levels
        calls = []

        def spy(self, *a):
            calls.append(1)
            return orig(self, *a)
        WH.Block._ll_levels = spy
        try:
            m(x)
        finally:
            WH.Block._ll_levels = orig
        assert calls, "the LL-only path did not run"
        saved = WH.Block.__dict__["_hf_unused"]
        WH.Block._hf_unused = property(lambda self: False)  # every Block: all 8 bands
        try:
            outs2, hf2 = m(x)
        finally:
            WH.Block._hf_unused = saved
    for a, b in zip(outs, outs2):
        assert C.rel_l2(a, b) <= 1e-5
    for da, db in zip(hf, hf2):
        for ta, tb in zip(da, db):
            for k in ta:
                assert C.rel_l2(ta[k], tb[k]) <= 1e-5, k


@pytest.mark.parametrize("levels,C_,base", [(1, 192, (2, 2, 2)), (2, 96, (2, 3, 2)),
                                            (3, 48, (1, 2, 2)), (3, 8, (2, 2, 2)),
                                            (4, 16, (1, 1, 1))])
def test_idwt_multilevel_vs_oracle_and_roundtrip(levels, C_, base):
    from waveformer_amd import ops
    B = 2
    full = tuple(b * 2 ** levels for b in base)
    x = seeded_randn((B, C_) + full, 5)
    co = R.wavedec3(x, "db1", levels)                 # NCDHW contiguous details
    ref = R.waverec3(co, "db1")
    assert C.rel_l2(ref, x) <= 1e-6
    ll = cuda(co[0])
    dets = [{k: cuda(v) for k, v in d.items()} for d in co[1:]]
    out = ops.idwt3d_haar(ll, dets)
    assert C.rel_l2(out, ref) <= 1e-5
    # channel-last detail views (what Block returns) + writing into a concat buffer
    dets_cl = [{k: v.permute(0, 2, 3, 4, 1).contiguous().permute(0, 4, 1, 2, 3) for k, v in d.items()}
               for d in dets]
    buf = torch.full((B, C_ + 3) + full, 7.0, device=DEV)
    ops.idwt3d_haar(ll, dets_cl, out=buf)
    assert C.rel_l2(buf[:, :C_], ref) <= 1e-5
    assert torch.all(buf[:, C_:] == 7.0)
    # channel-last concat buffer (the decoder's, ABI 12 wf_idwt3d_haar_cl), with the LL read
    # channel-last too: the same values bit for bit, the skip channels untouched
    if C_ % 4 == 0:
        bcl = torch.full((B, C_ + 4) + full, 7.0, device=DEV).contiguous(
            memory_format=torch.channels_last_3d)
        llcl = ll.contiguous(memory_format=torch.channels_last_3d)
        ops.idwt3d_haar(llcl, dets_cl, out=bcl)
        assert torch.equal(bcl[:, :C_], buf[:, :C_])
        assert torch.all(bcl[:, C_:] == 7.0)


@pytest.mark.parametrize("levels,C_,base", [(1, 48, (4, 4, 8)), (3, 16, (1, 2, 3)), (2, 12, (2, 1, 2))])
def test_idwt_vector_paths_match_scalar(levels, C_, base):
    """The 16-B kernels (channel-last output: idwt3d_haar_cl4; NCDHW output:
    idwt3d_haar_nc4) against the one-channel-per-lane kernel (WF_IDWT_SCALAR=1), bit for bit:
    the same additions in the same order."""
    from waveformer_amd import ops
    B = 2
    full = tuple(b * 2 ** levels for b in base)
    co = R.wavedec3(seeded_randn((B, C_) + full, 11), "db1", levels)
    ll = cuda(co[0])
    dets = [{k: cuda(v).permute(0, 2, 3, 4, 1).contiguous().permute(0, 4, 1, 2, 3)
             for k, v in d.items()} for d in co[1:]]
    llcl = ll.contiguous(memory_format=torch.channels_last_3d)

    def run():
        nc = torch.full((B, C_ + 4) + full, 3.0, device=DEV)
        ops.idwt3d_haar(ll, dets, out=nc)
        cl = torch.full((B, C_ + 4) + full, 3.0, device=DEV).contiguous(
            memory_format=torch.channels_last_3d)
        ops.idwt3d_haar(llcl, dets, out=cl)
        return nc, cl

    nc, cl = run()
    os.environ["WF_IDWT_SCALAR"] = "1"
    try:
        nc0, cl0 = run()
    finally:
        del os.environ["WF_IDWT_SCALAR"]
    assert torch.equal(nc, nc0) and torch.equal(cl, cl0)
    assert torch.equal(nc, cl)
    assert torch.all(nc[:, C_:] == 3.0) and torch.all(cl[:, C_:] == 3.0)


@pytest.mark.parametrize("levels,C_,base", [(1, 48, (4, 4, 8)), (2, 12, (2, 1, 2))])
def test_idwt_fused_concat(levels, C_, base):
    """wf_idwt3d_haar_cl_cat (ABI 13): the IDWT into channels [0, C) and the skip into [C, 2C)
    of the decoder's channel-last concat buffer in one kernel -- bit-identical to the IDWT
    followed by the copy (idwt_upsample.py:160-163), the skip copied exactly."""
    from waveformer_amd import ops
    B = 2
    full = tuple(b * 2 ** levels for b in base)
    co = R.wavedec3(seeded_randn((B, C_) + full, 13), "db1", levels)
    ll = cuda(co[0]).contiguous(memory_format=torch.channels_last_3d)
    dets = [{k: cuda(v).permute(0, 2, 3, 4, 1).contiguous().permute(0, 4, 1, 2, 3)
             for k, v in d.items()} for d in co[1:]]
    skip = cuda(seeded_randn((B, C_) + full, 14)).contiguous(memory_format=torch.channels_last_3d)
    want = torch.full((B, 2 * C_) + full, 5.0, device=DEV).contiguous(
        memory_format=torch.channels_last_3d)
    ops.idwt3d_haar(ll, dets, out=want)
    ops.copy_cl(skip, want[:, C_:])
    got = torch.full((B, 2 * C_) + full, 5.0, device=DEV).contiguous(
        memory_format=torch.channels_last_3d)
    ops.idwt3d_haar(ll, dets, out=got, skip=skip)
    assert torch.equal(got, want)
    assert torch.equal(got[:, C_:], skip)
    # under the scalar debug switch the fused entry does not apply; the op must
    # fall back to IDWT + copy instead of raising
    os.environ["WF_IDWT_SCALAR"] = "1"
    try:
        sc = torch.full((B, 2 * C_) + full, 5.0, device=DEV).contiguous(
            memory_format=torch.channels_last_3d)
        ops.idwt3d_haar(ll, dets, out=sc, skip=skip)
    finally:
        del os.environ["WF_IDWT_SCALAR"]
    assert torch.equal(sc, want)


def test_encoder_hf_feed_idwt_roundtrip():
    """DWT bands of the forward kernel, re-synthesised by the IDWT kernel, give back the input
    (Haar is orthonormal): the property that holds at full 128^3 sizes."""
    from waveformer_amd import ops
    x = cuda(seeded_randn((1, 64, 64, 64, 48), 9))
    cur, dets = x, []
    for _ in range(3):
        b = ops.dwt3d_haar(cur)
        dets.append(ops.bands_to_coeffs(b)[1])
        cur = b[0]
    rec = ops.idwt3d_haar(cur.permute(0, 4, 1, 2, 3), dets[::-1])
    assert C.rel_l2(rec, x.permute(0, 4, 1, 2, 3)) <= 1e-5


@pytest.mark.parametrize("shapes", [[(8, 8, 8), (4, 4, 4), (2, 2, 2)], [(16, 16, 16)],
                                    [(4, 4, 4)], [(3, 5, 6)]])
def test_msfuse_vs_trilinear(shapes):
    from waveformer_amd import ops
    B, Cc, D = 2, 48, 16
    sc = seeded_randn((B, D, D, D, Cc), 3)
    srcs = [seeded_randn((B,) + s + (Cc,), 10 + i) for i, s in enumerate(shapes)]
    ref = 0
    for s in srcs:
        ref = ref + F.interpolate(s.permute(0, 4, 1, 2, 3), size=(D, D, D), mode="trilinear")
    ref = sc + ref.permute(0, 2, 3, 4, 1)
    out, st = ops.msfuse([cuda(s) for s in srcs], cuda(sc), 1e-6)
    assert C.rel_l2(out, ref) <= 1e-6
    mean = ref.mean(-1).reshape(-1)
    rstd = torch.rsqrt(ref.var(-1, unbiased=False) + 1e-6).reshape(-1)
    assert C.rel_l2(st[:, 0], mean) <= 1e-5
    assert C.rel_l2(st[:, 1], rstd) <= 1e-5


@pytest.mark.parametrize("C_,S", [(48, 4096), (96, 512), (192, 64), (384, 8), (384, 1000)])
def test_proj_out_layernorm_ncdhw(C_, S):
    from waveformer_amd import ops
    x = seeded_randn((2, S, 1, 1, C_), 4) * 2 + 1
    out = ops.proj_out(cuda(x), True)
    ref = F.layer_norm(x, [C_]).permute(0, 4, 1, 2, 3)
    assert C.rel_l2(out, ref) <= 1e-5
    out = ops.proj_out(cuda(x), False)
    assert torch.equal(out.cpu(), x.permute(0, 4, 1, 2, 3))


@pytest.mark.parametrize("C_,S", [(48, 4096), (96, 512), (192, 64), (384, 8), (384, 1000),
                                  (40, 333), (8, 65)])
def test_proj_out_channel_last_bitwise(C_, S):
    """wf_proj_out_cl_fwd: proj_out's values (bitwise) as an NCDHW-shaped channels_last_3d
    tensor the UnetResBlocks read without a transpose."""
    from waveformer_amd import ops
    x = cuda(seeded_randn((2, S, 1, 1, C_), 5) * 2 + 1)
    for norm in (True, False):
        cl = ops.proj_out_cl(x, norm)
        assert cl.shape == (2, C_, S, 1, 1) and ops.cl_ld(cl) == C_
        assert torch.equal(cl.contiguous(), ops.proj_out(x, norm))


def test_full_model_channel_last_outs_bitwise():
    """The full model's inference hands the encoder's stage outputs over channel-last (no
    NCDHW write + transpose back); its logits are bitwise those of the NCDHW hand-over."""
    import waveformer_amd.network_models as NM
    from waveformer_amd.network_models import network_backbone as NB
    torch.manual_seed(0)
    m = NM.Waveformer(img_size=(32,) * 3, in_chans=4, out_chans=4,
                      num_heads=[1, 1, 1, 1]).eval().to(DEV)
    x = cuda(seeded_randn((1, 4, 32, 32, 32), 15))
    saved = NB._CL_OUTS
    try:
        with torch.no_grad():
            NB._CL_OUTS = True
            a = m(x)
            NB._CL_OUTS = False
            b = m(x)
    finally:
        NB._CL_OUTS = saved
    assert torch.equal(a, b)


@pytest.mark.parametrize("cin,S", [(4, 32), (1, 32), (4, 128)])
def test_patch_embed(cin, S):
    from waveformer_amd import ops
    x = seeded_randn((1, cin, S, S, S), 6)
    w = seeded_randn((48, cin, 2, 2, 2), 7) * 0.3
    b = seeded_randn((48,), 8)
    out = ops.patch_embed(cuda(x), cuda(w), cuda(b))
    ref = F.conv3d(x, w, b, stride=2).permute(0, 2, 3, 4, 1)
    assert C.rel_l2(out, ref) <= 1e-5


@pytest.mark.parametrize("ws,heads,dim,B_", [(8, 3, 48, 2), (8, 24, 384, 1), (2, 1, 48, 5),
                                             (2, 1, 384, 2), (4, 2, 64, 3), (8, 1, 96, 1),
                                             (8, 1, 192, 1), (12, 3, 48, 1), (4, 1, 128, 2),
                                             (4, 2, 64, 1)])
def test_attention_vs_oracle(ws, heads, dim, B_):
    import waveformer_amd.network_models as NM
    from oracle.weight_rule import rule_state_dict
    m = NM.Attention(dim, num_heads=heads, qkv_bias=True, window_size=ws)
    sd = rule_state_dict(m.state_dict())
    m.load_state_dict(sd)
    m = m.eval().to(DEV)
    from waveformer_amd import ops
    x = seeded_randn((B_, ws ** 3, dim), 12)
    ref = R.attention(sd, "", x, heads, ws)
    for prec, tol in (("bf16x3", 5e-5), ("bf16", 1e-2), ("fp16", 2e-3)):
        with torch.no_grad(), ops.precision(prec):
            out = m(cuda(x))
        assert C.rel_l2(out, ref) <= tol, prec


@pytest.mark.parametrize("shape", [(2, 8, 8, 8), (1, 5, 6, 11), (1, 16, 16, 16), (1, 3, 12, 9),
                                   (1, 20, 8, 8), (3, 7, 4, 9)])
@pytest.mark.parametrize("block", [False, True])
def test_ccf_ffn_stage1_fused_vs_oracle(shape, block):
    """C = 48, hidden = 192: the fused dwconv + LN2 + GELU + fc + residual kernel
    (ffn_dwfc.hip), ragged tiles included, z segments shorter than the volume at (1, 20, 8, 8);
    Block form (norm2 + Q4 double residual, per-sample DropPath factors) and bare
    CCF_FFN.forward."""
    import waveformer_amd.network_models as NM
    from oracle.weight_rule import rule_state_dict
    from waveformer_amd import ops
    B = shape[0]
    mlp = NM.CCF_FFN(48, 192, img_size=shape[1:])
    sd = rule_state_dict(mlp.state_dict())
    mlp.load_state_dict(sd)
    mlp = mlp.eval().to(DEV)
    norm2 = torch.nn.LayerNorm(48, eps=1e-6)
    with torch.no_grad():
        norm2.weight.copy_(seeded_randn((48,), 31) * 0.2 + 1)
        norm2.bias.copy_(seeded_randn((48,), 32) * 0.1)
    norm2 = norm2.to(DEV)
    x = seeded_randn(shape + (48,), 33)
    bs = torch.tensor([0.5, 2.0, 1.0][:B])
    if block:
        n2 = F.layer_norm(x, [48], norm2.weight.detach().cpu(), norm2.bias.detach().cpu(), 1e-6)
        ref = x + R.ccf_ffn(sd, "", n2) * bs.view(-1, 1, 1, 1, 1)
    else:
        ref = x + (R.ccf_ffn(sd, "", x) - x) * bs.view(-1, 1, 1, 1, 1)
    for prec, tol in (("bf16x3", 5e-5), ("bf16", 1e-2), ("fp16", 2e-3)):
        with torch.no_grad(), ops.precision(prec):
            xc = cuda(x)
            stats = ops.msfuse([], xc, 1e-6)[1] if block else None
            out = ops.ccf_ffn(xc, stats, norm2 if block else None, mlp, cuda(bs))
        assert C.rel_l2(out, ref) <= tol, prec


def test_ccf_ffn_stage1_batch_beyond_tb4_range():
    """the default stage-1 back half (ffn_dwfc_tb4) addresses its output through
    32-bit buffer offsets (2 GiB).  At 64^3 x 48 that is B >= 43 (inference with a large
    sw_batch_size): the launcher must take the unlimited SIMD-balanced kernel instead of failing.
    Samples 0 and B-1 of a B = 44 call against the same samples run at B = 2 (tb4)."""
    import waveformer_amd.network_models as NM
    from oracle.weight_rule import rule_state_dict
    from waveformer_amd import ops
    S, B = 64, 44
    mlp = NM.CCF_FFN(48, 192, img_size=(S,) * 3)
    mlp.load_state_dict(rule_state_dict(mlp.state_dict()))
    mlp = mlp.eval().to(DEV)
    assert B * S ** 3 * 48 * 4 >= 2 ** 31
    with torch.no_grad(), ops.precision("bf16x3"):
        x = torch.randn((B, S, S, S, 48), device=DEV, generator=torch.Generator(DEV).manual_seed(5))
        out = ops.ccf_ffn(x, None, None, mlp, None)
        pair = torch.stack([x[0], x[-1]])
        ref = ops.ccf_ffn(pair, None, None, mlp, None)
    torch.cuda.synchronize()
    assert C.rel_l2(out[0], ref[0]) <= 1e-6 and C.rel_l2(out[-1], ref[1]) <= 1e-6
    del x, out


@pytest.mark.parametrize("shape", [(2, 8, 8, 8), (1, 5, 6, 11), (3, 7, 4, 9), (1, 20, 8, 8),
                                   (1, 16, 16, 16)])
@pytest.mark.parametrize("block", [False, True])
def test_ccf_ffn_stage2_vs_oracle(shape, block):
    """C = 96, hidden = 384 (encoder stage 2): the pwconv + LN1 + GELU GEMM (pw2.hip's
    resident-weight kernel for bf16x3 / fp16, gemm_lnw.hip for bf16; rows not a multiple of the
    16-row tile included), then
    the fused back half (ffn_dwfc.hip's ffn_dwfc2_kernel: depthwise conv, LN2 + GELU, fc and
    the Q4 residual with h2 on chip; ragged 4 x 4 tiles, z segments shorter than the volume
    at (1, 20, 8, 8)) -- same bars as stage 1."""
    import waveformer_amd.network_models as NM
    from oracle.weight_rule import rule_state_dict
    from waveformer_amd import ops
    B = shape[0]
    mlp = NM.CCF_FFN(96, 384, img_size=shape[1:])
    sd = rule_state_dict(mlp.state_dict())
    mlp.load_state_dict(sd)
    mlp = mlp.eval().to(DEV)
    norm2 = torch.nn.LayerNorm(96, eps=1e-6)
    with torch.no_grad():
        norm2.weight.copy_(seeded_randn((96,), 34) * 0.2 + 1)
        norm2.bias.copy_(seeded_randn((96,), 35) * 0.1)
    norm2 = norm2.to(DEV)
    x = seeded_randn(shape + (96,), 36)
    bs = torch.tensor([0.5, 2.0, 1.0][:B])
    if block:
        n2 = F.layer_norm(x, [96], norm2.weight.detach().cpu(), norm2.bias.detach().cpu(), 1e-6)
        ref = x + R.ccf_ffn(sd, "", n2) * bs.view(-1, 1, 1, 1, 1)
    else:
        ref = x + (R.ccf_ffn(sd, "", x) - x) * bs.view(-1, 1, 1, 1, 1)
    for prec, tol in (("bf16x3", 5e-5), ("bf16", 1e-2), ("fp16", 2e-3)):
        with torch.no_grad(), ops.precision(prec):
            xc = cuda(x)
            stats = ops.msfuse([], xc, 1e-6)[1] if block else None
            out = ops.ccf_ffn(xc, stats, norm2 if block else None, mlp, cuda(bs))
        assert C.rel_l2(out, ref) <= tol, prec


@pytest.mark.parametrize("C_,shape", [(192, (2, 8, 8, 8)), (192, (1, 5, 6, 11)),
                                      (192, (1, 20, 4, 4)), (384, (2, 4, 4, 4)),
                                      (384, (1, 3, 5, 2))])
@pytest.mark.parametrize("block", [False, True])
def test_ccf_ffn_stage34_vs_oracle(C_, shape, block):
    """C = 192 / 384, hidden = 4C (encoder stages 3 / 4), the default path: the pwconv on
    gemm_kc, the LN1 + GELU pass (ln_act_fwd), the depthwise conv (ragged tiles, z segments and
    volume edges whose zero padding must stay zero), then the fc with LN2 + GELU in its loader
    and the Q4 residual -- same bars as stages 1 / 2.  The opt-in LN1-fused variant
    (WF_FFN_LN1_FUSE=1, read once per process) is covered by
    test_ccf_ffn_stage34_ln1_fuse_subprocess."""
    import waveformer_amd.network_models as NM
    from oracle.weight_rule import rule_state_dict
    from waveformer_amd import ops
    B = shape[0]
    mlp = NM.CCF_FFN(C_, 4 * C_, img_size=shape[1:])
    sd = rule_state_dict(mlp.state_dict())
    mlp.load_state_dict(sd)
    mlp = mlp.eval().to(DEV)
    norm2 = torch.nn.LayerNorm(C_, eps=1e-6)
    with torch.no_grad():
        norm2.weight.copy_(seeded_randn((C_,), 37) * 0.2 + 1)
        norm2.bias.copy_(seeded_randn((C_,), 38) * 0.1)
    norm2 = norm2.to(DEV)
    x = seeded_randn(shape + (C_,), 39)
    bs = torch.tensor([0.5, 2.0, 1.0][:B])
    if block:
        n2 = F.layer_norm(x, [C_], norm2.weight.detach().cpu(), norm2.bias.detach().cpu(), 1e-6)
        ref = x + R.ccf_ffn(sd, "", n2) * bs.view(-1, 1, 1, 1, 1)
    else:
        ref = x + (R.ccf_ffn(sd, "", x) - x) * bs.view(-1, 1, 1, 1, 1)
    for prec, tol in (("bf16x3", 5e-5), ("bf16", 1e-2), ("fp16", 2e-3)):
        with torch.no_grad(), ops.precision(prec):
            xc = cuda(x)
            stats = ops.msfuse([], xc, 1e-6)[1] if block else None
            out = ops.ccf_ffn(xc, stats, norm2 if block else None, mlp, cuda(bs))
        assert C.rel_l2(out, ref) <= tol, prec


_LN1_FUSE_CHILD = r"""
import sys, torch, torch.nn.functional as F
sys.path.insert(0, '.')
import waveformer_amd.network_models as NM
from oracle import ref_waveformer as R
from oracle.weight_rule import rule_state_dict, seeded_randn
from tests import cases as C
from waveformer_amd import ops
worst = 0.0
for C_, shape in ((192, (1, 5, 6, 11)), (384, (2, 4, 4, 4))):
    mlp = NM.CCF_FFN(C_, 4 * C_, img_size=shape[1:])
    sd = rule_state_dict(mlp.state_dict())
    mlp.load_state_dict(sd)
    mlp = mlp.eval().cuda()
    x = seeded_randn(shape + (C_,), 39)
    bs = torch.tensor([0.5, 2.0, 1.0][:shape[0]])
    ref = x + (R.ccf_ffn(sd, "", x) - x) * bs.view(-1, 1, 1, 1, 1)
    with torch.no_grad(), ops.precision("bf16x3"):
        out = ops.ccf_ffn(x.cuda(), None, None, mlp, bs.cuda())
    worst = max(worst, C.rel_l2(out, ref))
print("LN1FUSE_WORST", worst)
"""


def test_ccf_ffn_stage34_ln1_fuse_subprocess():
    """the opt-in LN1-fused stage-3/4 path (WF_FFN_LN1_FUSE=1: LN1 partials in the
    pwconv epilogue, ln_stats_finalize, dwconv3d_kernel<float, true> applying LN1 + GELU while
    it stages) is read once per process, so it runs in a child process with the switch set,
    against the oracle at the bf16x3 bar."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WF_FFN_LN1_FUSE="1", PYTHONPATH=repo)
    r = subprocess.run([sys.executable, "-c", _LN1_FUSE_CHILD], cwd=repo, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    worst = float(r.stdout.split("LN1FUSE_WORST")[1].split()[0])
    assert worst <= 5e-5, worst


_MERGE_SHAPES = ((2, 8, 8, 8), (1, 6, 10, 6), (1, 64, 64, 64))


def _merge48_outputs(prec):
    """PatchMerging 1 -> 2 (C = 48: merge.hip's resident-weight kernel unless WF_MERGE_RES=0)
    over _MERGE_SHAPES, with the oracle's fp64 outputs."""
    import waveformer_amd.network_models as NM
    from oracle.weight_rule import rule_state_dict
    from waveformer_amd import ops
    outs = []
    for i, shape in enumerate(_MERGE_SHAPES):
        m = NM.PatchMerging(48, norm_layer=C._ln6())
        sd = rule_state_dict(m.state_dict())
        m.load_state_dict(sd)
        m = m.to(DEV)
        x = seeded_randn(shape + (48,), 60 + i) * 1.5 + 0.25
        ref = R.patch_merging({k: v.double() for k, v in sd.items()}, "", x.double())
        with torch.no_grad(), ops.precision(prec):
            out = ops.patch_merging(x.to(DEV), m.norm, m.reduction)
        outs.append((out.cpu(), ref))
    return outs


@pytest.mark.parametrize("prec,tol", [("bf16x3", 1e-5), ("fp16", 2e-3)])
def test_patch_merging_c48_resident_vs_oracle(prec, tol):
    """The stage 1 -> 2 merge on merge.hip (weight resident in LDS, persistent 12-wave
    workgroups, no barrier after the staging): ragged row count (45 rows: a partial 16-row
    tile) and a 64^3 volume (2048 tiles over 256 workgroups), against the fp64 oracle
    (wave_helper.py:173-194 with quirk Q3)."""
    for out, ref in _merge48_outputs(prec):
        assert out.shape == ref.shape
        assert C.rel_l2(out, ref.float()) <= tol


_MERGE_CHILD = r"""
import sys, torch
sys.path.insert(0, '.')
from tests import test_gpu_parity as T
outs = T._merge48_outputs(sys.argv[1])
torch.save([o for o, _ in outs], sys.argv[2])
print("MERGE_CHILD_OK")
"""


@pytest.mark.parametrize("prec", ["bf16x3", "fp16"])
def test_patch_merging_c48_resident_bitwise_vs_gemm_kc(prec, tmp_path):
    """merge.hip keeps gemm_kc's LN_COMPUTE arithmetic and order (shifted one-pass moments,
    k-step MFMA accumulation, fp16 operands rounded from the fp32 value): bit-identical outputs
    to gemm_kc (8-wave workgroups at the small shapes, 16-wave at 64^3).  WF_MERGE_RES=0 (read
    once per process) runs gemm_kc in a child process."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = str(tmp_path / "kc.pt")
    env = dict(os.environ, WF_MERGE_RES="0", PYTHONPATH=repo)
    r = subprocess.run([sys.executable, "-c", _MERGE_CHILD, prec, dst], cwd=repo, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "MERGE_CHILD_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    kc = torch.load(dst, weights_only=True)
    for (out, _), o_kc in zip(_merge48_outputs(prec), kc):
        d = (out - o_kc).abs()
        rows = (d.reshape(-1, out.shape[-1]) > 0).any(-1)
        assert torch.equal(out, o_kc), (tuple(out.shape), int((d > 0).sum()), float(d.max()),
                                        int(rows.sum()), rows.nonzero()[:8].flatten().tolist())


_FFN2_SHAPES = ((2, 8, 8, 8), (1, 5, 6, 11), (8, 32, 32, 32))


def _stage2_ffn_outputs(prec):
    """The stage-2 CCF_FFN inside a Block (norm2 statistics given, Q4 residual) over
    _FFN2_SHAPES; the last is the B = 8 bench shape (262,144 rows: 16,384 tiles over 256
    persistent workgroups)."""
    import waveformer_amd.network_models as NM
    from oracle.weight_rule import rule_state_dict
    from waveformer_amd import ops
    outs = []
    for i, shape in enumerate(_FFN2_SHAPES):
        mlp = NM.CCF_FFN(96, 384, img_size=shape[1:])
        mlp.load_state_dict(rule_state_dict(mlp.state_dict()))
        mlp = mlp.eval().to(DEV)
        norm2 = torch.nn.LayerNorm(96, eps=1e-6)
        with torch.no_grad():
            norm2.weight.copy_(seeded_randn((96,), 34) * 0.2 + 1)
            norm2.bias.copy_(seeded_randn((96,), 35) * 0.1)
        norm2 = norm2.to(DEV)
        x = seeded_randn(shape + (96,), 70 + i).to(DEV)
        bs = torch.linspace(0.5, 2.0, shape[0]).to(DEV)
        with torch.no_grad(), ops.precision(prec):
            stats = ops.msfuse([], x, 1e-6)[1]
            outs.append(ops.ccf_ffn(x, stats, norm2, mlp, bs).cpu())
    return outs


_FFN2_CHILD = r"""
import sys, torch
sys.path.insert(0, '.')
from tests import test_gpu_parity as T
torch.save(T._stage2_ffn_outputs(sys.argv[1]), sys.argv[2])
print("FFN2_CHILD_OK")
"""


@pytest.mark.parametrize("prec", ["bf16x3", "fp16"])
def test_stage2_pwconv_resident_bitwise_vs_gemm_lnw(prec, tmp_path):
    """pw2.hip (weight resident, whole rows per wave) keeps gemm_lnw<3, 3, 8, 8>'s arithmetic
    and order -- split products per column tile, the row moments as its 8 waves' partials in its
    tree order: the stage-2 FFN outputs are bit-identical.  WF_PW2_RES=0 (read once per
    process) runs gemm_lnw in a child process."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = str(tmp_path / "lnw.pt")
    env = dict(os.environ, WF_PW2_RES="0", PYTHONPATH=repo)
    r = subprocess.run([sys.executable, "-c", _FFN2_CHILD, prec, dst], cwd=repo, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "FFN2_CHILD_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    ref = torch.load(dst, weights_only=True)
    for out, o_ref in zip(_stage2_ffn_outputs(prec), ref):
        d = (out - o_ref).abs()
        assert torch.equal(out, o_ref), (tuple(out.shape), int((d > 0).sum()), float(d.max()))


@pytest.mark.parametrize("shape", [(2, 8, 8, 8), (1, 5, 6, 11)])
@pytest.mark.parametrize("block", [False, True])
def test_ccf_ffn_stage2_staged_path_vs_oracle(shape, block, monkeypatch):
    """The unfused stage-2 back half (WF_FFN_NO_DWFC=1: z-marching depthwise conv with LN2
    moments, then the fc with LN2 + GELU in its loader) -- the path training keeps, since its
    backward needs h2."""
    monkeypatch.setenv("WF_FFN_NO_DWFC", "1")
    test_ccf_ffn_stage2_vs_oracle(shape, block)


@pytest.mark.parametrize("shape", [(2, 8, 8, 8), (1, 5, 6, 11), (1, 16, 16, 16), (1, 3, 12, 9)])
@pytest.mark.parametrize("block", [False, True])
def test_ccf_ffn_stage1_whole_kernel_vs_oracle(shape, block, monkeypatch):
    """The opt-in whole-FFN kernel (WF_FFN_FUSED=1, ffn_fused.hip: pw + LN1 + GELU recomputed
    on chip per haloed plane, dwconv, LN2, GELU, fc, Q4 residual) on the same cases and bars as
    the staged path above, ragged tiles and volume edges included."""
    monkeypatch.setenv("WF_FFN_FUSED", "1")
    test_ccf_ffn_stage1_fused_vs_oracle(shape, block)


def test_window_attention_q1_layout_on_raster():
    """Raster attention == window_partition -> Attention -> plain reshape (quirk Q1)."""
    import waveformer_amd.network_models as NM
    from oracle.weight_rule import rule_state_dict
    m = NM.Attention(48, num_heads=3, qkv_bias=True, window_size=4)
    sd = rule_state_dict(m.state_dict())
    m.load_state_dict(sd)
    m = m.eval().to(DEV)
    x = seeded_randn((2, 8, 12, 16, 48), 21)
    with torch.no_grad():
        out = m.forward_raster(cuda(x))
    win = R.window_partition(x, 4).view(-1, 64, 48)
    ref = R.attention(sd, "", win, 3, 4).reshape(2, 8, 12, 16, 48)
    assert C.rel_l2(out, ref) <= 5e-5


# ------------------------------------------------------------------------------ module level
# Dice bound of the fp16 path (see test_full_model_128_dice_vs_reference for why reduced-
# precision operands move Dice at all with these weights)
FP16_DICE = 1e-3  # the north star's bound; fp16 policy (ops.FP16_SPLIT_OPS): 192^3 HF 6.7e-4

# rel-L2 bounds per precision (measured: bf16x3 2.5e-6..2.6e-5, bf16 1.5e-3..1e-2)
TOL = {"bf16x3": {"tensor": 5e-5, "block": 5e-5, "encoder": 1e-4, "full": 1e-4},
       "bf16": {"tensor": 1e-2, "block": 2e-2, "encoder": 3e-2, "full": 3e-2},
       "fp16": {"tensor": 2e-3, "block": 3e-3, "encoder": 5e-3, "full": 5e-3}}


@pytest.mark.parametrize("prec", ["bf16x3", "bf16", "fp16"])
@pytest.mark.parametrize("name", ["attn_ws8", "attn_ws2_h1", "attn_ws4_h2", "merge", "ccf_ffn",
                                  "block_l3", "block_l1", "block_l0", "block_ss_l2", "enc32",
                                  "full32", "full32hf"])
def test_module_vs_reference_golden_and_oracle(name, prec):
    from waveformer_amd import ops
    case = C.cases()[name]
    m, sd = C.build(case, DEV)
    x = C.case_input(case)
    with torch.no_grad(), ops.precision(prec):
        out = m(cuda(x))
    with torch.no_grad():
        ora = case.oracle(sd, x)
    got = C.flatten_output(case, out)
    want_oracle = C.flatten_output(case, ora)
    keys = [k for k in C.golden().files if (k == name or k.startswith(name + "_")) and "__" not in k]
    assert set(got) == set(keys)
    tol = TOL[prec][case.kind]
    for k in keys:
        ref = C.g(k)
        assert tuple(got[k].shape) == tuple(ref.shape), k
        e_ref = C.rel_l2(got[k], ref)
        e_ora = C.rel_l2(got[k], want_oracle[k])
        # high-pass bands of deep encoder stages are differences of neighbouring voxels
        # (cancellation): the same absolute error is ~10x larger relative to them
        t = tol * (10 if "_hf" in k and case.kind == "encoder" else 1)
        assert e_ref <= t, (k, e_ref)
        assert e_ora <= t, (k, e_ora)


def test_encoder128_vs_reference_summaries():
    case = C.cases()["enc128"]
    m, _ = C.build(case, DEV)
    with torch.no_grad():
        outs, hfs = m(cuda(C.case_input(case)))
    flat = C.flatten_output(case, (outs, hfs))
    for k, t in flat.items():
        assert tuple(t.shape) == tuple(C.golden()[k + "__shape"]), k
        sums, sample = C.summary(t)
        ref = C.golden()[k + "__sum"]
        tol = 2e-3 if "_hf" in k else 2e-4  # bf16x3 (default precision)
        assert abs(math.sqrt(sums[1]) / math.sqrt(ref[1]) - 1) <= tol, k
        assert abs(sums[2] - ref[2]) <= 10 * tol * math.sqrt(ref[1]), k
        assert C.rel_l2(sample, C.g(k + "__sample")) <= tol, (k, C.rel_l2(sample, C.g(k + "__sample")))


def test_encoder192_vs_reference_summaries():
    """config 5 widths at 192^3 x 4: window 12 (N = 1728 tokens, 23^3-row bias table)."""
    case = C.cases()["enc192"]
    m, _ = C.build(case, DEV)
    with torch.no_grad():
        outs, _ = m(cuda(C.case_input(case)))
    for i, t in enumerate(outs):
        k = f"enc192_out{i}"
        assert tuple(t.shape) == tuple(C.golden()[k + "__shape"]), k
        sums, sample = C.summary(t)
        ref = C.golden()[k + "__sum"]
        assert abs(math.sqrt(sums[1]) / math.sqrt(ref[1]) - 1) <= 2e-4, k
        assert C.rel_l2(sample, C.g(k + "__sample")) <= 2e-4, (k, C.rel_l2(sample, C.g(k + "__sample")))


@pytest.mark.parametrize("prec,bound", [("bf16x3", 1e-3), ("fp16", FP16_DICE)])
def test_full_model_192_hf_refinement_dice_vs_reference(prec, bound):
    """config 5: full model with the HF refinement branch at 192^3 x 4: Dice of the argmax
    labels (TC / WT / ET) against the reference's own labels -- fp32-faithful bf16x3, and the
    fp16 MFMA path config 5 names (fp16 operands, fp32 accumulation / LayerNorm / softmax)."""
    from waveformer_amd import ops
    case = C.cases()["full192hf"]
    m, _ = C.build(case, DEV)
    with torch.no_grad(), ops.precision(prec):
        logits = m(cuda(C.case_input(case)))
    lab = logits.argmax(1).cpu()
    ref = C.g("full192hf_labels").long()
    d = [C.dice(a, b) for a, b in zip(C.brats_regions(lab), C.brats_regions(ref))]
    assert min(d) >= 1 - bound, d


@pytest.mark.parametrize("prec,bound", [("bf16x3", 1e-3), ("bf16", 5e-2), ("fp16", FP16_DICE)])
def test_full_model_128_dice_vs_reference(prec, bound):
    """BASELINE north_star: Dice within 1e-3 of the reference (TC / WT / ET of the argmax
    labels of the full model at 128^3 x 4).  The fp32-faithful default (bf16x3) meets it;
    plain bf16 operands cannot with these weights (every logit margin is uniformly spread near
    zero, so a 1e-2 logit error flips ~1% of voxels -- measured Dice ~0.98; CPU bf16 autocast of
    the reference encoder gives 0.97), hence its looser bound."""
    from waveformer_amd import ops
    case = C.cases()["full128"]
    m, _ = C.build(case, DEV)
    with torch.no_grad(), ops.precision(prec):
        logits = m(cuda(C.case_input(case)))
    lab = logits.argmax(1).cpu()
    ref = C.g("full128_labels").long()
    d = [C.dice(a, b) for a, b in zip(C.brats_regions(lab), C.brats_regions(ref))]
    assert min(d) >= 1 - bound, d
