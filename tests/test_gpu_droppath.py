"""Training-mode DropPath through the HIP kernels.

Block in .train() with drop_path > 0 hands per-sample factors to the fused kernels: msfuse's
branch_scale, the FFN residual epilogue's r_scale (ffn_dwfc's bscale at C = 48), and in the
backward MsFuse's row scaling / the interpolation adjoint's oscale / CCFFFN's df scaling.
`DropPath.sample_scale` is pinned to fixed factors holding both a dropped (0) and a kept
(1 / keep) sample, and the forward outputs and every gradient are compared against the oracle
(oracle/ref_waveformer.block with the same factors: wave_helper.py:507-508, :546-547) on the
CPU in fp32 autograd.  Bars: the module bars of test_train_grads (forward rel-L2 <= 5e-5,
gradients <= 2e-4 per tensor, bf16x3 forward / fp32 backward).
"""
from functools import partial

import pytest
import torch
import torch.nn as nn

from oracle import ref_waveformer as R
from oracle.weight_rule import rule_state_dict, seeded_randn
from tests import cases as C

pytestmark = pytest.mark.gpu

KEEP = 0.75
# (name, dim, heads, level, img, multi-scale): the r1 Block cases at B = 2 plus a stage-1
# width (C = 48, hidden 192: the fused ffn_dwfc kernel) block
CASES = [("block_l3", 32, 2, 3, 16, True), ("block_l0", 32, 2, 0, 8, True),
         ("block_ss_l2", 32, 2, 2, 16, False), ("block48_l1", 48, 3, 1, 16, True)]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from waveformer_amd import _lib
    _lib.load()
    torch.backends.cuda.matmul.allow_tf32 = False
    yield


@pytest.mark.parametrize("name,dim,heads,level,img,ms", CASES)
def test_block_train_droppath_vs_oracle(name, dim, heads, level, img, ms, monkeypatch):
    import waveformer_amd.network_models as NM
    from waveformer_amd.network_models.wave_helper import DropPath
    s_attn = torch.tensor([1 / KEEP, 0.0])
    s_mlp = torch.tensor([0.0, 1 / KEEP])
    calls = []

    def fixed(self, batch, device):
        assert self.training and batch == 2
        calls.append(1)
        return (s_attn if len(calls) % 2 == 1 else s_mlp).to(device)

    monkeypatch.setattr(DropPath, "sample_scale", fixed)
    m = NM.Block(dim, heads, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6),
                 level=level, ms_attention=ms, img_size=(img,) * 3, drop_path=1 - KEEP)
    sd = rule_state_dict(m.state_dict())
    m.load_state_dict(sd, strict=True)
    m = m.train().cuda()
    x = seeded_randn((2, img, img, img, dim), 41)

    xg = x.cuda().requires_grad_(True)
    out = m(xg)
    assert len(calls) == 2, "Block must sample one factor per branch"
    C.grad_loss(C.flat_outputs(out)).backward()
    torch.cuda.synchronize()

    sdg = {k: (v.detach().clone().requires_grad_(True) if v.is_floating_point() else v)
           for k, v in sd.items()}
    xo = x.clone().requires_grad_(True)
    ref = R.block(sdg, "", xo, heads, level, (img,) * 3, ms, drop_scales=(s_attn, s_mlp))
    C.grad_loss(C.flat_outputs(ref)).backward()

    got_f, want_f = C.flat_outputs(out), C.flat_outputs(ref)
    assert len(got_f) == len(want_f)
    for i, (a, b) in enumerate(zip(got_f, want_f)):
        assert C.rel_l2(a, b) <= 5e-5, (name, "output", i, C.rel_l2(a, b))
    bad = []
    want = {"x": xo.grad}
    want.update({k: v.grad for k, v in sdg.items() if v.is_floating_point() and v.grad is not None})
    got = {"x": xg.grad}
    got.update({k: p.grad for k, p in m.named_parameters() if p.grad is not None})
    floor = 1e-5 * max(w.norm().item() for w in want.values())
    for k, w in want.items():
        assert k in got, (name, "no gradient for", k)
        if w.norm().item() < floor:
            assert got[k].norm().item() < 10 * floor, (name, k)
            continue
        e = C.rel_l2(got[k], w)
        if not e <= 2e-4:
            bad.append((k, e))
    assert not bad, (name, bad)
