"""torch.library registration of the hot-path ops (SURVEY 8b "Registration", library.py).

CPU (no GPU needed):
  * the six ops exist under torch.ops.waveformer with Meta (fake) kernels: Blocks and the
    encoder's Blocks + PatchMerging built on the meta device run forward and give the
    reference's output shapes (meta-device shape inference of the drop-in);
  * the fake kernels' workspace sizes (plain SymInt arithmetic) equal the library's own
    wf_*_workspace_bytes queries;
  * CPU tensors fail loudly (no CPU kernel: the product path has no fallback).
GPU (-m gpu):
  * torch.library.opcheck on every op (schema, fake tensor, autograd registration, AOT
    dispatch), inference and train variants;
  * torch.compile(Block, fullgraph=True) equals eager bit for bit (multi-scale, level 0 and
    single-scale Blocks; backend aot_eager: dynamo + fake tensors + AOT autograd, no codegen);
  * a compiled Block in training mode (AOT autograd traces the backward through the
    registered *_backward ops) gives the eager gradients.
"""
from functools import partial

import pytest
import torch
import torch.nn as nn

from oracle.weight_rule import rule_state_dict, seeded_randn

OPS = ["dwt3d", "idwt3d", "window_attn", "msfuse", "ccf_ffn", "patch_merging"]


def _nm():
    import waveformer_amd.network_models as NM
    return NM


def test_ops_registered():
    import waveformer_amd.library  # noqa: F401
    for name in OPS:
        assert hasattr(torch.ops.waveformer, name), name


@pytest.mark.parametrize("level,img,ms", [(3, 16, True), (1, 16, True), (0, 8, True),
                                          (2, 16, False)])
def test_block_meta_shape_inference(level, img, ms):
    NM = _nm()
    with torch.device("meta"), torch.no_grad():
        blk = NM.Block(48, 3, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6),
                       level=level, ms_attention=ms, img_size=(img,) * 3).eval()
        x = torch.empty(2, img, img, img, 48)
        r = blk(x)
    out = r[0] if isinstance(r, tuple) else r
    assert out.device.type == "meta" and tuple(out.shape) == (2, img, img, img, 48)
    if level > 0:
        hfs = r[1]
        n = max(level, 1) if ms else level
        assert len(hfs) == n
        sizes = [img // 2 ** (n - i) for i in range(n)]  # coarse -> fine
        for d, s in zip(hfs, sizes):
            assert sorted(d) == sorted(("aad", "ada", "add", "daa", "dad", "dda", "ddd"))
            assert all(tuple(t.shape) == (2, 48, s, s, s) for t in d.values())


def test_encoder_meta_shape_inference():
    NM = _nm()
    # (the constructor's drop-path schedule calls .item(), as the reference's does: build on
    # the CPU, then move to meta)
    m = NM.MultiscaleTransformer(img_size=(32,) * 3, in_chans=4, qkv_bias=True,
                                 norm_layer=partial(nn.LayerNorm, eps=1e-6)).eval().to("meta")
    with torch.device("meta"), torch.no_grad():
        blocks_out = []
        x = torch.empty(1, 48, 16, 16, 16).permute(0, 2, 3, 4, 1)
        for s in range(4):
            if s > 0:
                x = getattr(m, f"downsample_{s}")(x)
            for blk in getattr(m, f"block{s + 1}"):
                r = blk(x)
                x = r[0] if isinstance(r, tuple) else r
            blocks_out.append(tuple(x.shape))
    assert blocks_out == [(1, 16, 16, 16, 48), (1, 8, 8, 8, 96), (1, 4, 4, 4, 192),
                          (1, 2, 2, 2, 384)]


def test_fake_workspace_sizes_match_library():
    from waveformer_amd import _lib, library
    for (B, C, D, H, W) in [(1, 48, 32, 32, 32), (8, 96, 16, 16, 16), (2, 384, 8, 8, 8)]:
        assert library.attn_workspace_bytes(B, C, D, H, W) == _lib.query(
            "wf_window_attention_workspace_bytes", B, C, D, H, W, library.SPLIT)
        assert library.ffn_workspace_bytes(B, C, 4 * C, D, H, W) == _lib.query(
            "wf_ccf_ffn_workspace_bytes", B, C, 4 * C, D, H, W, library.SPLIT)


def test_cpu_tensors_fail_loudly_through_ops():
    import waveformer_amd.library  # noqa: F401
    x = torch.zeros(1, 4, 4, 4, 8)
    with pytest.raises(RuntimeError, match="GPU only"):
        torch.ops.waveformer.dwt3d(x, None, None, 0.0)


# ------------------------------------------------------------------------------------ GPU
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from waveformer_amd import _lib
    _lib.load()


def _inputs(name, train):
    """Small sample arguments of each op (bf16x3 = WF_PREC 1)."""
    d = "cuda"
    g = lambda shape, seed, scale=1.0: (seeded_randn(shape, seed) * scale).to(d)
    rg = train
    if name == "dwt3d":
        return [g((2, 8, 6, 4, 16), 1).requires_grad_(rg), g((16,), 2, 0.1).add_(1).requires_grad_(rg),
                g((16,), 3, 0.1).requires_grad_(rg), 1e-6]
    if name == "idwt3d":
        ll = g((2, 8, 2, 3, 2), 4).requires_grad_(rg)
        det = [g((2, 8, 2, 3, 2), 10 + k).requires_grad_(rg) for k in range(7)]
        det += [g((2, 8, 4, 6, 4), 20 + k).requires_grad_(rg) for k in range(7)]
        return [ll, det]
    if name == "window_attn":
        from waveformer_amd.network_models.attention import relative_position_index
        C, h, ws = 32, 2, 4
        return [g((1, 8, 4, 8, C), 5).requires_grad_(rg), None, None, 0.0,
                g((3 * C, C), 6, 0.1).requires_grad_(rg), g((3 * C,), 7, 0.1).requires_grad_(rg),
                g(((2 * ws - 1) ** 3, h), 8, 0.1).requires_grad_(rg),
                relative_position_index(ws).to(d), g((C, C), 9, 0.1).requires_grad_(rg),
                g((C,), 10, 0.1).requires_grad_(rg), ws, h, (C // h) ** -0.5, 1, train]
    if name == "msfuse":
        return [[g((2, 2, 2, 2, 16), 11).requires_grad_(rg), g((2, 4, 4, 4, 16), 12).requires_grad_(rg)],
                g((2, 4, 4, 4, 16), 13).requires_grad_(rg), None, 1e-6, True]
    if name == "ccf_ffn":
        C, hid = 16, 64
        xh = g((2, 4, 4, 4, C), 14)
        from waveformer_amd import ops
        st = ops.msfuse([], xh, 1e-6)[1]
        return [xh.requires_grad_(rg), st, g((C,), 15, 0.1).add_(1).requires_grad_(rg),
                g((C,), 16, 0.1).requires_grad_(rg), g((hid, C, 1, 1, 1), 17, 0.2).requires_grad_(rg),
                g((hid,), 18, 0.1).requires_grad_(rg), g((hid,), 19, 0.1).add_(1).requires_grad_(rg),
                g((hid,), 20, 0.1).requires_grad_(rg), g((hid, 1, 3, 3, 3), 21, 0.2).requires_grad_(rg),
                g((hid,), 22, 0.1).requires_grad_(rg), g((hid,), 23, 0.1).add_(1).requires_grad_(rg),
                g((hid,), 24, 0.1).requires_grad_(rg), g((C, hid), 25, 0.1).requires_grad_(rg),
                g((C,), 26, 0.1).requires_grad_(rg), None, 1e-6, 1e-5, 1e-5, 1, train]
    if name == "patch_merging":
        C = 16
        return [g((2, 4, 4, 4, C), 27).requires_grad_(rg), g((8 * C,), 28, 0.1).add_(1).requires_grad_(rg),
                g((8 * C,), 29, 0.1).requires_grad_(rg), 1e-6, g((2 * C, 8 * C), 30, 0.1).requires_grad_(rg),
                False, 1]
    raise KeyError(name)


@pytest.mark.gpu
@pytest.mark.parametrize("train", [False, True])
@pytest.mark.parametrize("name", OPS)
def test_opcheck(name, train):
    _gpu()
    from waveformer_amd import library
    op = getattr(torch.ops.waveformer, name).default
    args = _inputs(name, train)
    tests = ["test_schema", "test_faketensor", "test_autograd_registration"]
    if train:
        tests.append("test_aot_dispatch_dynamic")
    torch.library.opcheck(op, args, test_utils=tests)


def _block(level, img, ms, dim=48, heads=3):
    NM = _nm()
    m = NM.Block(dim, heads, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6),
                 level=level, ms_attention=ms, img_size=(img,) * 3)
    m.load_state_dict(rule_state_dict(m.state_dict()), strict=True)
    return m.cuda()


def _flat(r):
    if isinstance(r, torch.Tensor):
        return [r]
    out, hfs = r
    return [out] + [d[k] for d in hfs for k in sorted(d)]


@pytest.mark.gpu
@pytest.mark.parametrize("level,img,ms", [(3, 16, True), (0, 8, True), (2, 16, False)])
def test_compile_block_fullgraph_matches_eager(level, img, ms):
    _gpu()
    torch._dynamo.reset()
    m = _block(level, img, ms).eval()
    x = seeded_randn((2, img, img, img, 48), 31).cuda()
    cm = torch.compile(m, fullgraph=True, backend="aot_eager")
    with torch.no_grad():
        want = _flat(m(x))
        got = _flat(cm(x))
    assert len(got) == len(want)
    for a, b in zip(got, want):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_compile_block_fullgraph_training_grads():
    _gpu()
    torch._dynamo.reset()
    m = _block(1, 16, True)
    x = seeded_randn((2, 16, 16, 16, 48), 32).cuda()
    cm = torch.compile(m, fullgraph=True, backend="aot_eager")
    grads = []
    for fn in (m, cm):
        m.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        loss = sum((t * seeded_randn(tuple(t.shape), 50 + i).cuda()).sum()
                   for i, t in enumerate(_flat(fn(xi))))
        loss.backward()
        grads.append([xi.grad] + [p.grad for p in m.parameters()])
    # the attention backward accumulates dQ and the bias gradient with fp32 atomics, so two
    # eager runs already differ in the last bits: compared at rel-L2 <= 1e-5 per tensor
    from tests.cases import rel_l2
    for a, b in zip(*grads):
        if b is None:
            assert a is None
            continue
        assert rel_l2(a, b) <= 1e-5
