"""CPU: pin the oracle (oracle/ref_waveformer.py) to the golden vectors.

* PyWavelets 1.1.1 vectors pin the ptwt restatement (wavedec3 / waverec3, 'haar' and 'db2',
  'zero' mode, 1-3 levels, even and odd sizes) to float64 rounding.
* Fixtures produced by running the reference network_models itself (gen_reference_fixtures.py)
  pin Attention / Block (levels 0-3, single- and multi-scale) / PatchMerging / CCF_FFN / the
  encoder (32^3 x 1 with head_dim = C; 128^3 x 4 default) / the full Waveformer (32^3 x 4,
  128^3 x 4 label map).  The oracle recomputes each from the same rule weights and seeded
  input in fp32: agreement is expected at fp32 rounding (rel-L2 <= 2e-6).
"""
import numpy as np
import pytest
import torch

from oracle import ref_waveformer as R
from oracle.weight_rule import seeded_randn
from tests import cases as C

FP32_TOL = 2e-6


def test_pywt_vectors():
    z = np.load(C.PYWT_PATH)
    ncase = len([k for k in z.files if k.endswith("_meta")])
    assert ncase == 6
    for ci in range(ncase):
        x = torch.from_numpy(z[f"c{ci}_x"])
        wav = bytes(z[f"c{ci}_wavelet"]).decode()
        for L in range(1, int(z[f"c{ci}_meta"][0]) + 1):
            co = R.wavedec3(x, wav, L)
            np.testing.assert_allclose(co[0].numpy(), z[f"c{ci}_L{L}_ll"], atol=1e-12, rtol=0)
            assert len(co) == L + 1
            for li, d in enumerate(co[1:]):
                assert tuple(d.keys()) == R.DETAIL_KEYS
                for k, v in d.items():
                    np.testing.assert_allclose(v.numpy(), z[f"c{ci}_L{L}_d{li}_{k}"], atol=1e-12, rtol=0)
            rec = R.waverec3(co, wav)
            np.testing.assert_allclose(rec.numpy(), z[f"c{ci}_L{L}_rec"], atol=1e-12, rtol=0)
            if x.shape[-3:] == rec.shape[-3:]:
                np.testing.assert_allclose(rec.numpy(), x.numpy(), atol=1e-12, rtol=0)


@pytest.mark.parametrize("ws", [2, 4, 8, 12])
def test_relative_position_index_quirk_q2(ws):
    idx = R.relative_position_index(ws)
    N = ws ** 3
    assert idx.shape == (N, N)
    # the depth stride is 3*ws-1, not (2*ws-1)^2 -> distinct offsets collide (Q2)
    assert idx.max().item() == (2 * ws - 2) * (3 * ws - 1) + (2 * ws - 2) * (2 * ws - 1) + 2 * ws - 2
    if ws == 8:
        assert torch.unique(idx).numel() == 547
    for name, w in (("attn_ws8", 8), ("attn_ws2_h1", 2), ("attn_ws4_h2", 4)):
        if w == ws:
            assert torch.equal(idx.to(torch.int16), C.g(name + "__index"))


def test_window_reverse_quirk_q1_is_not_identity():
    # wave_helper.py:498-499: partition then plain reshape != identity when nW > 1
    x = torch.arange(2 * 8 * 8 * 8 * 3, dtype=torch.float32).view(2, 8, 8, 8, 3)
    w = R.window_partition(x, 4).reshape(2, 8, 8, 8, 3)
    assert not torch.equal(w, x)
    w1 = R.window_partition(x, 8).reshape(2, 8, 8, 8, 3)  # nW == 1 -> identity
    assert torch.equal(w1, x)


SMALL = ["attn_ws8", "attn_ws2_h1", "attn_ws4_h2", "block_l3", "block_l1", "block_l0",
         "block_ss_l2", "merge", "ccf_ffn", "enc32", "full32", "full32hf"]


@pytest.mark.parametrize("name", SMALL)
def test_oracle_matches_reference_small(name):
    case = C.cases()[name]
    _, sd = C.build(case)
    with torch.no_grad():
        out = case.oracle(sd, C.case_input(case))
    flat = C.flatten_output(case, out)
    keys = [k for k in C.golden().files if k == name or k.startswith(name + "_")]
    keys = [k for k in keys if "__" not in k]
    assert set(flat) == set(keys), (sorted(set(flat) ^ set(keys)))[:5]
    for k in keys:
        ref = C.g(k)
        got = flat[k]
        assert tuple(got.shape) == tuple(ref.shape), k
        assert C.rel_l2(got, ref) <= FP32_TOL, (k, C.rel_l2(got, ref))


def test_oracle_matches_reference_encoder128():
    case = C.cases()["enc128"]
    _, sd = C.build(case)
    with torch.no_grad():
        out = case.oracle(sd, C.case_input(case))
    flat = C.flatten_output(case, out)
    for k, t in flat.items():
        sums, sample = C.summary(t)
        ref_sums = C.golden()[k + "__sum"]
        assert tuple(t.shape) == tuple(C.golden()[k + "__shape"])
        np.testing.assert_allclose(sums[1], ref_sums[1], rtol=1e-5)           # sum of squares
        np.testing.assert_allclose(sums[2], ref_sums[2], rtol=1e-4, atol=1e-3 * np.sqrt(ref_sums[1]))
        # stage outputs agree to ~2e-7; the high-pass bands are differences of neighbouring
        # voxels (cancellation), so the same absolute fp32 noise is up to ~1e-4 relative there
        tol = 2e-4 if "_hf" in k else 2e-6
        assert C.rel_l2(sample, C.g(k + "__sample")) <= tol, k


@pytest.mark.slow
@pytest.mark.parametrize("name", ["enc192"])
def test_oracle_matches_reference_encoder192_summaries(name):
    case = C.cases()[name]
    _, sd = C.build(case)
    with torch.no_grad():
        outs, _ = case.oracle(sd, C.case_input(case))
    for i, t in enumerate(outs):
        k = f"{name}_out{i}"
        sums, sample = C.summary(t)
        assert tuple(t.shape) == tuple(C.golden()[k + "__shape"])
        np.testing.assert_allclose(sums[1], C.golden()[k + "__sum"][1], rtol=1e-5)
        assert C.rel_l2(sample, C.g(k + "__sample")) <= 2e-6, k


def test_oracle_matches_reference_full128_dice():
    case = C.cases()["full128"]
    _, sd = C.build(case)
    with torch.no_grad():
        logits = case.oracle(sd, C.case_input(case))
    sums, _ = C.summary(logits)
    np.testing.assert_allclose(sums[1], C.golden()["full128__sum"][1], rtol=1e-5)
    lab = logits.argmax(1)
    ref = C.g("full128_labels").long()
    for a, b in zip(C.brats_regions(lab), C.brats_regions(ref)):
        assert C.dice(a, b) >= 0.9999
