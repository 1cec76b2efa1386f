"""Predictor -- the test-time inference helper of light_training/prediction.py (:29-228).

Same class, constructor and static methods, so 4_predict.py-style callers switch by import:
  * maybe_mirror_and_predict (:110-160): sliding-window inference over the image and its flips
    (inferers.maybe_mirror_and_predict: all passes in ONE sharded window inference, the flip
    merge on HIP);
  * predict_raw_probability (:35-63): every class channel trilinearly resampled to the
    pre-resample shape into a torch.half buffer -- one wf_resample_trilinear_cf launch for all
    channels (HIP, fp32 arithmetic, fp16 store) instead of a framework call per channel;
  * predict_noncrop_probability (:65-104): paste the cropped prediction back into the
    uncropped volume (host numpy, as the reference: its result goes to NIfTI on the host).
The reference's CPU fallback of predict_raw_probability (on a RuntimeError) is not mirrored:
the product path runs on the GPU or fails loudly.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from . import inferers, ops


def _ints(v):
    return [int(t.item()) if isinstance(t, torch.Tensor) else int(t) for t in v]


class Predictor:
    def __init__(self, window_infer, mirror_axes: Optional[Sequence[int]] = None) -> None:
        self.window_infer = window_infer
        self.mirror_axes = mirror_axes

    @staticmethod
    def predict_raw_probability(model_output: torch.Tensor, properties) -> torch.Tensor:
        """(1, C, D, H, W) or (C, D, H, W) probabilities -> (C, d, w, h) fp16 on the GPU at
        properties["shape_after_cropping_before_resample"] (prediction.py:35-63); a host
        tensor is moved to the GPU first."""
        if model_output.dim() == 5:
            model_output = model_output[0]
        if model_output.device.type != "cuda":  # the reference's CPU-returning TTA output
            model_output = model_output.to("cuda", non_blocking=True)
        size = _ints(properties["shape_after_cropping_before_resample"][:3])
        with torch.no_grad():
            return ops.resample_trilinear_cf(model_output, size, torch.float16)

    @staticmethod
    def predict_noncrop_probability(model_output, properties) -> np.ndarray:
        """Paste a (d, h, w) label map or (C, d, h, w) prediction into zeros of
        properties["shape_before_cropping"] at properties["bbox_used_for_cropping"]
        (prediction.py:65-104), uint8 like the reference."""
        if isinstance(model_output, torch.Tensor):
            model_output = model_output.cpu().numpy()
        shape = _ints(properties["shape_before_cropping"][:3])
        bb = [_ints(b) for b in properties["bbox_used_for_cropping"]]
        sl = tuple(slice(b[0], b[1]) for b in bb)
        if model_output.ndim == 3:
            out = np.zeros(shape, dtype=np.uint8)
            out[sl] = model_output
            return out
        if model_output.ndim == 4:
            out = np.zeros([model_output.shape[0]] + shape, dtype=np.uint8)
            out[(slice(None),) + sl] = model_output
            return out
        raise ValueError("predict_noncrop_probability: 3-D or 4-D prediction expected")

    def maybe_mirror_and_predict(self, x, model, device=torch.device("cpu"), **kwargs):
        """prediction.py:110-160: the mean over the flip passes of the window inference."""
        if isinstance(device, str):
            device = torch.device(device)
        model.to(device)
        return inferers.maybe_mirror_and_predict(x.to(device), model, self.window_infer,
                                                 self.mirror_axes, **kwargs)
