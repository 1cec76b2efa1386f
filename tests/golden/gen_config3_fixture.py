"""Generate the config-3 golden fixture by running the REFERENCE itself (CPU, fp32): MONAI's
sliding-window inference over a BraTS-shaped 1 x 4 x 240 x 240 x 155 case with the reference
Waveformer as the predictor, exactly as 4_predict.py:199-205 sets it up (roi 128^3,
sw_batch_size 2, overlap 0.5, mode "gaussian"; config.yaml prediction block).

    python tests/golden/gen_config3_fixture.py [--reference /root/reference]

The vendored MONAI (`monai.inferers.SlidingWindowInferer`, monai/inferers/utils.py:43-321) and
`network_models.Waveformer` are imported from the read-only reference checkout with the same
stand-ins as gen_reference_fixtures.py (ptwt -> the oracle's restatement pinned to PyWavelets,
timm / torchinfo / ptflops init helpers).  Every parameter comes from oracle.weight_rule and the
input from a seeded CPU generator, so the GPU test rebuilds both exactly.

Writes tests/golden/config3_fixture.npz:
  c3__shape / c3__sum / c3__sample   logits summary (sum, sum of squares, seeded dot; a strided
                                     sample of 4096 values), as gen_reference_fixtures._summary
  c3_labels_packed                   argmax labels (classes 0..3) packed 4 per byte, C order
Nothing here runs on the GPU box.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
from oracle.weight_rule import apply_rule, seeded_randn  # noqa: E402

SHAPE = (1, 4, 240, 240, 155)
SEED = 40
ROI, SW_BATCH, OVERLAP = (128, 128, 128), 2, 0.5
MODEL_KW = dict(img_size=(128, 128, 128), in_chans=4, out_chans=4, depths=[2, 2, 2, 2],
                feat_size=[48, 96, 192, 384], num_heads=[3, 6, 12, 24])


def pack_labels(lab: np.ndarray) -> np.ndarray:
    """uint8 labels in 0..3 -> 2-bit codes, 4 per byte (first label in the low bits)."""
    flat = lab.reshape(-1).astype(np.uint8)
    pad = (-flat.size) % 4
    flat = np.concatenate([flat, np.zeros(pad, np.uint8)]).reshape(-1, 4)
    return (flat[:, 0] | (flat[:, 1] << 2) | (flat[:, 2] << 4) | (flat[:, 3] << 6)).astype(np.uint8)


def unpack_labels(packed: np.ndarray, shape) -> np.ndarray:
    p = np.asarray(packed, dtype=np.uint8)
    lab = np.stack([p & 3, (p >> 2) & 3, (p >> 4) & 3, (p >> 6) & 3], 1).reshape(-1)
    return lab[:int(np.prod(shape))].reshape(shape)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    sys.dont_write_bytecode = True
    import gen_reference_fixtures as G
    G._install_standins()
    sys.path.insert(0, args.reference)
    from monai.inferers import SlidingWindowInferer  # the reference's vendored MONAI
    from network_models import Waveformer

    torch.set_num_threads(8)
    torch.set_grad_enabled(False)
    net = apply_rule(Waveformer(**MODEL_KW)).eval()
    x = seeded_randn(SHAPE, SEED)
    inf = SlidingWindowInferer(roi_size=ROI, sw_batch_size=SW_BATCH, overlap=OVERLAP,
                               mode="gaussian")
    t0 = time.time()
    logits = inf(x, net)
    print(f"sliding window {time.time() - t0:.1f}s -> {tuple(logits.shape)}")
    out = {}
    G._summary("c3", logits, out)
    lab = logits.argmax(1).to(torch.uint8).numpy()
    out["c3_labels_packed"] = pack_labels(lab)
    out["c3_labels_shape"] = np.array(lab.shape, dtype=np.int64)
    out["c3_label_counts"] = np.bincount(lab.reshape(-1), minlength=4).astype(np.int64)
    dst = os.path.join(HERE, "config3_fixture.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst, {k: v.shape for k, v in out.items()}, out["c3_label_counts"])


if __name__ == "__main__":
    main()
