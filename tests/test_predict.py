"""Predictor (light_training/prediction.py:29-228): predict_raw_probability's trilinear
resample (csrc/upsample.hip resample_cf_kernel) and predict_noncrop_probability.

CPU: the oracle restatement (oracle/ref_predict.py) against the golden vectors PyTorch's own
interpolate produced (tests/golden/gen_resample_fixtures.py; the reference module itself is
not importable here -- SimpleITK / skimage are absent); the un-crop paste vs the oracle.
GPU: the HIP resample against the same vectors.  Bar: the fp16 outputs equal the golden ones
except where the fp32 value sits on an fp16 rounding boundary -- at most 1 fp16 ulp apart,
>= 99.9% of elements bit-identical; the fp32 output mode against F.interpolate on the GPU at
rel-L2 <= 1e-6.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ref_predict as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "resample_fixtures.npz")
CASES = ["down", "up", "mixed", "single"]


def _gold():
    return np.load(GOLD)


def _close_f16(got: np.ndarray, want: np.ndarray):
    g = got.astype(np.float16).view(np.int16).astype(np.int32)
    w = want.astype(np.float16).view(np.int16).astype(np.int32)
    ulps = np.abs(g - w)
    assert ulps.max() <= 1, ulps.max()
    assert (ulps == 0).mean() >= 0.999, (ulps == 0).mean()


@pytest.mark.parametrize("name", CASES)
def test_oracle_resample_vs_golden(name):
    G = _gold()
    x, want = G[name + "_in"], G[name + "_out"]
    _close_f16(O.predict_raw_probability(x, want.shape[1:]), want)


def test_noncrop_paste_vs_oracle():
    from waveformer_amd.prediction import Predictor
    rng = np.random.default_rng(0)
    pred3 = rng.integers(0, 4, (5, 6, 7)).astype(np.uint8)
    pred4 = rng.integers(0, 2, (3, 5, 6, 7)).astype(np.uint8)
    props = {"shape_before_cropping": [9, 10, 12],
             "bbox_used_for_cropping": [[2, 7], [1, 7], [4, 11]]}
    for p in (pred3, pred4, torch.from_numpy(pred4)):
        got = Predictor.predict_noncrop_probability(p, props)
        want = O.predict_noncrop_probability(np.asarray(p), props["shape_before_cropping"],
                                             props["bbox_used_for_cropping"])
        assert got.dtype == np.uint8 and np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_hip_resample_vs_golden(name):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from waveformer_amd import _lib, ops
    from waveformer_amd.prediction import Predictor
    _lib.load()
    G = _gold()
    x, want = G[name + "_in"], G[name + "_out"]
    xc = torch.from_numpy(x).cuda()
    props = {"shape_after_cropping_before_resample": list(want.shape[1:])}
    got = Predictor.predict_raw_probability(xc[None], props)
    assert got.dtype == torch.float16 and tuple(got.shape) == want.shape
    _close_f16(got.cpu().numpy(), want)
    # fp32 output mode vs the framework's interpolate on the same device
    f32 = ops.resample_trilinear_cf(xc, want.shape[1:], torch.float32)
    ref = torch.nn.functional.interpolate(xc[None], size=want.shape[1:], mode="trilinear")[0]
    assert float((f32 - ref).norm() / ref.norm()) <= 1e-6
