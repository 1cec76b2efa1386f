"""TEST INFRASTRUCTURE ONLY -- CPU restatement of Predictor.predict_raw_probability
(light_training/prediction.py:35-63) and predict_noncrop_probability (:65-104).

predict_raw_probability resamples each class channel with
F.interpolate(mode="trilinear", align_corners=False) into a torch.half buffer; restated here
as PyTorch's upsample_trilinear3d arithmetic in numpy float32: per axis
src = max((dst + 0.5) * in / out - 0.5, 0), i0 = floor(src), i1 = i0 + (i0 < in - 1),
l1 = src - i0, l0 = 1 - l1, combined t0 * (h0 * (w0 a + w1 b) + h1 * (...)) + t1 * (...),
then rounded to fp16.  Pinned by tests/golden/resample_fixtures.npz (PyTorch's own
interpolate, tests/golden/gen_resample_fixtures.py).
"""
from __future__ import annotations

from typing import Sequence

import numpy as np


def _axis(n_in: int, n_out: int):
    """(i0, i1, l0, l1) per output index, float32 arithmetic (align_corners=False)."""
    scale = np.float32(n_in) / np.float32(n_out)
    dst = np.arange(n_out, dtype=np.float32)
    src = np.maximum(scale * (dst + np.float32(0.5)) - np.float32(0.5), np.float32(0))
    i0 = src.astype(np.int64)
    i1 = i0 + (i0 < n_in - 1)
    l1 = (src - i0.astype(np.float32)).astype(np.float32)
    l0 = (np.float32(1) - l1).astype(np.float32)
    return i0, i1, l0, l1


def predict_raw_probability(x: np.ndarray, size: Sequence[int]) -> np.ndarray:
    """(C, D, H, W) float32 -> (C, *size) float16 (prediction.py:44-51)."""
    x = np.asarray(x, dtype=np.float32)
    C, D, H, W = x.shape
    z0, z1, t0, t1 = _axis(D, size[0])
    y0, y1, h0, h1 = _axis(H, size[1])
    x0, x1, w0, w1 = _axis(W, size[2])
    t0, t1 = t0[:, None, None], t1[:, None, None]
    h0, h1 = h0[None, :, None], h1[None, :, None]
    w0, w1 = w0[None, None, :], w1[None, None, :]
    out = np.empty((C,) + tuple(size), dtype=np.float16)
    for c in range(C):
        v = x[c]

        def g(zi, yi, xi):
            return v[zi[:, None, None], yi[None, :, None], xi[None, None, :]]
        a = h0 * (w0 * g(z0, y0, x0) + w1 * g(z0, y0, x1)) + h1 * (w0 * g(z0, y1, x0) + w1 * g(z0, y1, x1))
        b = h0 * (w0 * g(z1, y0, x0) + w1 * g(z1, y0, x1)) + h1 * (w0 * g(z1, y1, x0) + w1 * g(z1, y1, x1))
        out[c] = (t0 * a + t1 * b).astype(np.float32).astype(np.float16)
    return out


def predict_noncrop_probability(pred: np.ndarray, shape_before_cropping, bbox) -> np.ndarray:
    """prediction.py:65-104: the cropped prediction pasted into uint8 zeros."""
    sl = tuple(slice(int(b[0]), int(b[1])) for b in bbox)
    if pred.ndim == 3:
        out = np.zeros([int(s) for s in shape_before_cropping], dtype=np.uint8)
        out[sl] = pred
    else:
        out = np.zeros([pred.shape[0]] + [int(s) for s in shape_before_cropping], dtype=np.uint8)
        out[(slice(None),) + sl] = pred
    return out
