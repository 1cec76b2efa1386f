"""Generate sliding-window / TTA golden fixtures by running the REFERENCE's own code (CPU, fp32).

    python tests/golden/gen_sliding_window_fixtures.py [--reference /root/reference]

Runs the vendored MONAI of mahfuzalhasan/WaveFormer (`monai.inferers.utils.
sliding_window_inference`, `monai.data.utils.dense_patch_slices`, `compute_importance_map`)
and its `light_training.prediction.Predictor.maybe_mirror_and_predict` with
`monai.inferers.SlidingWindowInferer` on seeded inputs and the deterministic, window-position
dependent toy predictor `toy_predictor` below (tests restate it), so the importance weights
matter.  Stand-ins are installed only for modules prediction.py imports but
maybe_mirror_and_predict never calls: SimpleITK, skimage.measure and
light_training.preprocessing.resampling.default_resampling (whose batchgenerators dependency
is absent).  Writes tests/golden/sw_fixtures.npz.  Nothing here runs on the GPU box.
"""
from __future__ import annotations

import argparse
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle.weight_rule import seeded_randn  # noqa: E402


def toy_predictor(x: torch.Tensor) -> torch.Tensor:
    """(n, Cin, d, h, w) -> (n, 3, d, h, w); depends on the position inside the window."""
    n, c, d, h, w = x.shape
    zz = torch.arange(d, dtype=torch.float).view(1, 1, d, 1, 1) / d
    yy = torch.arange(h, dtype=torch.float).view(1, 1, 1, h, 1) / h
    xx = torch.arange(w, dtype=torch.float).view(1, 1, 1, 1, w) / w
    m = x.mean(1, keepdim=True)
    return torch.cat([m + zz, torch.tanh(x[:, :1]) * (1 + yy), m * m - xx], 1)


CASES = {
    # name: (input shape, seed, roi, sw_batch, overlap, mode)
    "sw_gauss": ((1, 2, 40, 36, 30), 31, (16, 16, 16), 3, 0.5, "gaussian"),
    "sw_const_pad": ((2, 1, 20, 12, 24), 32, (16, 16, 16), 2, 0.25, "constant"),
    "sw_gauss_b2": ((2, 2, 24, 20, 28), 33, (12, 12, 12), 4, 0.5, "gaussian"),
}
TTA = ("sw_tta", (1, 2, 24, 20, 18), 34, (12, 12, 12), 2, 0.5, "gaussian", [0, 1, 2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    sys.path.insert(0, args.reference)
    for n in ("SimpleITK", "skimage", "skimage.measure",
              "light_training.preprocessing.resampling.default_resampling"):
        sys.modules[n] = types.ModuleType(n)
    sys.modules["skimage"].measure = sys.modules["skimage.measure"]
    sys.modules["light_training.preprocessing.resampling.default_resampling"] \
        .resample_data_or_seg_to_shape = None
    from monai.data.utils import compute_importance_map, dense_patch_slices
    from monai.inferers import SlidingWindowInferer
    from monai.inferers.utils import sliding_window_inference
    from light_training.prediction import Predictor

    out = {}
    for name, (shape, seed, roi, sb, ov, mode) in CASES.items():
        x = seeded_randn(shape, seed)
        with torch.no_grad():
            y = sliding_window_inference(x, roi, sb, toy_predictor, overlap=ov, mode=mode)
        out[name + "_y"] = y.numpy()
    for roi in ((16, 16, 16), (12, 12, 12), (12, 20, 8)):
        out["imap_gauss_" + "x".join(map(str, roi))] = compute_importance_map(
            roi, mode="gaussian", sigma_scale=0.125).numpy()
    # config 3's 128^3 map, every 3rd voxel per axis (keeps the fixture small)
    out["imap_gauss_128x128x128_s3"] = compute_importance_map(
        (128, 128, 128), mode="gaussian", sigma_scale=0.125).numpy()[::3, ::3, ::3]
    # BraTS geometry of config 3: 240 x 240 x 155, roi 128, overlap 0.5 -> 3 x 3 x 2 windows
    sl = dense_patch_slices((240, 240, 155), (128, 128, 128), (64, 64, 64))
    out["brats_window_starts"] = np.array([[s.start for s in w] for w in sl], dtype=np.int64)

    name, shape, seed, roi, sb, ov, mode, axes = TTA
    x = seeded_randn(shape, seed)
    pred = Predictor(SlidingWindowInferer(roi, sw_batch_size=sb, overlap=ov, mode=mode),
                     mirror_axes=axes)
    class Toy(torch.nn.Module):  # Predictor calls model.to(device)
        def forward(self, v):
            return toy_predictor(v)

    with torch.no_grad():
        out[name + "_y"] = pred.maybe_mirror_and_predict(x, Toy()).numpy()
    path = os.path.join(HERE, "sw_fixtures.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
