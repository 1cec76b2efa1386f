"""GPU parity for config 3 (sliding-window inference + flip TTA) through the C-ABI kernels
wf_importance_map, wf_sliding_window_stitch and wf_tta_merge.

Tolerances (stated per check):
  * stitch / TTA merge on identical patches and map: BIT-EXACT against the oracle -- the
    kernels sum in the reference's order with explicit round-to-nearest adds, multiplies and
    divides (no FMA contraction).
  * gaussian importance map: rel max error <= 2e-6 against the reference's map (expf on the GPU
    vs the CPU exp, 1-2 ulp).
  * whole inference with the toy predictor run by torch on the GPU: rel-L2 <= 1e-6 against
    the reference's own output (predictor ulps + map ulps).
  * whole inference with the Waveformer as predictor (bf16x3 MFMA path): rel-L2 <= 1e-4
    against the oracle's sliding window over the oracle Waveformer, like the full-model
    parity in test_gpu_parity.py.
"""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from gen_sliding_window_fixtures import CASES, TTA, toy_predictor  # noqa: E402

from oracle import ref_sliding_window as RS  # noqa: E402
from oracle import ref_waveformer as R  # noqa: E402
from oracle.weight_rule import seeded_randn  # noqa: E402
from tests import cases as C  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"
FIX = np.load(os.path.join(HERE, "golden", "sw_fixtures.npz"))


def _fx(k):
    return torch.from_numpy(np.array(FIX[k]))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from waveformer_amd import _lib
    _lib.load()
    yield


@pytest.mark.parametrize("roi", [(16, 16, 16), (12, 12, 12), (12, 20, 8)])
def test_importance_map_vs_reference(roi):
    from waveformer_amd import ops
    got = ops.importance_map(roi, "gaussian", (0.125,) * 3).cpu()
    ref = _fx("imap_gauss_" + "x".join(map(str, roi)))
    assert ((got - ref).abs() / ref).max().item() <= 2e-6
    assert torch.equal(ops.importance_map(roi, "constant").cpu(), torch.ones(roi))


def test_importance_map_128_vs_reference():
    from waveformer_amd import ops
    got = ops.importance_map((128,) * 3, "gaussian", (0.125,) * 3).cpu()[::3, ::3, ::3]
    ref = _fx("imap_gauss_128x128x128_s3")
    assert ((got - ref).abs() / ref).max().item() <= 2e-6


@pytest.mark.parametrize("world,sb,B", [(1, 1, 1), (1, 3, 2), (3, 2, 1), (8, 2, 2), (4, 1, 3)])
def test_stitch_bit_exact_vs_oracle(world, sb, B):
    from waveformer_amd import inferers, ops
    img, roi = (30, 26, 21), (12, 10, 9)
    st = inferers.dense_patch_starts(img, roi, inferers.scan_interval(img, roi, (0.5,) * 3))
    total = B * len(st[0]) * len(st[1]) * len(st[2])
    rounds, slots = inferers.shard_plan(total, world, sb)
    patches = seeded_randn((rounds * world * sb, 3) + roi, 7)
    wmap = RS.importance_map(roi, "gaussian", (0.125,) * 3)
    got = ops.sliding_window_stitch(patches.to(DEV), wmap.to(DEV), st, img, B, world, sb)
    ref = RS.stitch(patches, wmap, st, img, B, world, sb)
    assert torch.equal(got.cpu(), ref)


@pytest.mark.parametrize("world,B", [(1, 1), (1, 2), (3, 1), (8, 2)])
def test_stitch_partial_allreduce_vs_oracle(world, B):
    """The all-reduce exchange (wf_sliding_window_stitch_partial + wf_sliding_window_normalize,
    ABI 14): each rank's partial bit-exact against the oracle's partial; the rank partials
    summed (what the all-reduce computes) and normalised against the all-gather stitch --
    bitwise at one rank, rel-L2 <= 1e-6 when the sums meet in rank order."""
    from waveformer_amd import inferers, ops
    img, roi = (30, 26, 21), (12, 10, 9)
    st = inferers.dense_patch_starts(img, roi, inferers.scan_interval(img, roi, (0.5,) * 3))
    total = B * len(st[0]) * len(st[1]) * len(st[2])
    slots = -(-total // world)
    allp = seeded_randn((total, 3) + roi, 8)
    wmap = RS.importance_map(roi, "gaussian", (0.125,) * 3)
    acc = None
    for r in range(world):
        local = torch.zeros((slots, 3) + roi)
        g = torch.arange(r, total, world)
        local[:len(g)] = allp[g]
        got = ops.sliding_window_stitch_partial(local.to(DEV), wmap.to(DEV), st, img, B, world, r)
        assert torch.equal(got.cpu(), RS.stitch_partial(local, wmap, st, img, B, world, r))
        acc = got if acc is None else acc + got
    out = ops.sliding_window_normalize(acc)
    ref = RS.stitch(allp, wmap, st, img, B)
    if world == 1:
        assert torch.equal(out.cpu(), ref)
    else:
        assert C.rel_l2(out, ref) <= 1e-6


def test_stitch_rejects_bad_geometry():
    from waveformer_amd import ops
    p = torch.zeros((2, 1, 4, 4, 4), device=DEV)
    m = torch.ones((4, 4, 4), device=DEV)
    with pytest.raises(RuntimeError, match="span"):
        ops.sliding_window_stitch(p, m, [[0, 2], [0], [0]], (8, 4, 4), 1)  # ends at 6 != 8
    with pytest.raises(RuntimeError, match="ascending"):
        ops.sliding_window_stitch(p, m, [[0, 0], [0], [0]], (4, 4, 4), 1)


def test_tta_merge_bit_exact_vs_oracle():
    from waveformer_amd import inferers, ops
    passes = inferers.mirror_passes([0, 1, 2])
    pred = seeded_randn((8, 3, 9, 7, 6), 8)
    got = ops.tta_merge(pred.to(DEV), passes).cpu()
    assert torch.equal(got, RS.tta_merge(pred, passes))
    passes2 = inferers.mirror_passes([1])
    got2 = ops.tta_merge(pred[:2].contiguous().to(DEV), passes2).cpu()
    assert torch.equal(got2, RS.tta_merge(pred[:2], passes2))


def _toy_gpu(x):
    return toy_predictor(x.cpu()).to(x.device)  # the predictor is the test's, not the product


@pytest.mark.parametrize("name", sorted(CASES))
def test_sliding_window_vs_reference(name):
    from waveformer_amd import inferers
    shape, seed, roi, sb, ov, mode = CASES[name]
    x = seeded_randn(shape, seed).to(DEV)
    y = inferers.sliding_window_inference(x, roi, sb, _toy_gpu, overlap=ov, mode=mode)
    assert y.device.type == "cuda"
    assert C.rel_l2(y, _fx(name + "_y")) <= 1e-6


def test_tta_vs_reference():
    from waveformer_amd import inferers
    name, shape, seed, roi, sb, ov, mode, axes = TTA
    inf = inferers.SlidingWindowInferer(roi, sw_batch_size=sb, overlap=ov, mode=mode,
                                        cache_roi_weight_map=True)
    y = inferers.maybe_mirror_and_predict(seeded_randn(shape, seed).to(DEV), _toy_gpu, inf, axes)
    assert C.rel_l2(y, _fx(name + "_y")) <= 1e-6


def test_sliding_window_waveformer_vs_oracle():
    """The Waveformer (32^3 roi, default widths) as the predictor over a 44 x 40 x 36 x 4 image,
    gaussian, overlap 0.5, sw_batch 2 -> 2 x 2 x 2 windows."""
    from waveformer_amd import inferers
    case = C.cases()["full32"]
    m, sd = C.build(case, DEV)
    x = seeded_randn((1, 4, 44, 40, 36), 41)
    with torch.no_grad():
        y = inferers.sliding_window_inference(x.to(DEV), (32,) * 3, 2, m, overlap=0.5,
                                              mode="gaussian")
        ref = RS.sliding_window_inference(
            x, (32,) * 3, 2, lambda v: R.waveformer(sd, v, heads=[3, 6, 12, 24], depths=[2] * 4),
            overlap=0.5, mode="gaussian")
    assert C.rel_l2(y, ref) <= 1e-4
