"""TEST INFRASTRUCTURE ONLY -- CPU restatement of MONAI's sliding-window inference and the
flip-TTA of WaveFormer's Predictor, as the reference's prediction path runs them.

Restates (paths relative to the reference repo root):
  * monai/inferers/utils.py:43-321 `sliding_window_inference`, non-buffered path: scan
    interval (:355-376), F.pad when the image is smaller than the roi (:171-177), windows of
    `dense_patch_slices` (monai/data/utils.py:171-211) batched sw_batch_size at a time
    (:216-230), output *= importance map, scattered with `+=` into a zero output (:282-292),
    count map of summed weights (:262-269), out /= count (:298-299), padding cropped (:303-316);
  * monai/data/utils.py:1088-1138 `compute_importance_map` ('constant' / 'gaussian');
  * light_training/prediction.py:110-160 `maybe_mirror_and_predict` (8-way flip TTA).
Scatter form and operation order are the reference's.  Pinned against the vendored MONAI
itself by tests/golden/sw_fixtures.npz (tests/golden/gen_sliding_window_fixtures.py).
"""
from __future__ import annotations

import math
from typing import Callable, List, Sequence

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def importance_map(roi: Sequence[int], mode: str = "constant",
                   sigma_scale: Sequence[float] = (0.125,) * 3, device=None) -> Tensor:
    """monai/data/utils.py:1118-1137 (float32, on the CPU)."""
    roi = tuple(int(r) for r in roi)
    if mode == "constant":
        m = torch.ones(roi, dtype=torch.float)
    elif mode == "gaussian":
        sig = [r * s for r, s in zip(roi, sigma_scale)]
        m = None
        for i, n in enumerate(roi):
            x = torch.arange(start=-(n - 1) / 2.0, end=(n - 1) / 2.0 + 1, dtype=torch.float)
            x = torch.exp(x ** 2 / (-2 * sig[i] ** 2))
            m = x if i == 0 else m.unsqueeze(-1) * x[(None,) * i]
    else:
        raise ValueError(mode)
    mn = max(torch.min(m).item(), 1e-3)
    return torch.clamp_(m.to(torch.float), min=mn)


def window_starts(image_size: Sequence[int], roi: Sequence[int],
                  overlap: Sequence[float]) -> List[List[int]]:
    """_get_scan_interval + dense_patch_slices starts per axis."""
    starts = []
    for i, r, o in zip(image_size, roi, overlap):
        s = int(r) if r == i else max(int(r * (1 - o)), 1)
        p = min(i, r)
        num = int(math.ceil(float(i) / s))
        n = next((d for d in range(num) if d * s + p >= i), None)
        n = 1 if n is None else n + 1
        starts.append([k * s - max(k * s + p - i, 0) for k in range(n)])
    return starts


def sliding_window_inference(inputs: Tensor, roi_size: Sequence[int], sw_batch_size: int,
                             predictor: Callable[[Tensor], Tensor], overlap=0.25,
                             mode: str = "constant", sigma_scale=0.125, cval: float = 0.0,
                             roi_weight_map: Tensor = None) -> Tensor:
    ov = (overlap,) * 3 if isinstance(overlap, (int, float)) else tuple(overlap)
    ss = (sigma_scale,) * 3 if isinstance(sigma_scale, (int, float)) else tuple(sigma_scale)
    B = inputs.shape[0]
    image_size_ = list(inputs.shape[2:])
    roi = [int(i) if (r is None or r <= 0) else int(r) for r, i in zip(roi_size, image_size_)]
    image_size = [max(i, r) for i, r in zip(image_size_, roi)]
    pad = []
    for k in (2, 1, 0):
        diff = max(roi[k] - inputs.shape[k + 2], 0)
        pad.extend([diff // 2, diff - diff // 2])
    if any(pad):
        inputs = F.pad(inputs, pad=pad, mode="constant", value=cval)
    st = window_starts(image_size, roi, ov)
    slices = [(slice(z, z + roi[0]), slice(y, y + roi[1]), slice(x, x + roi[2]))
              for z in st[0] for y in st[1] for x in st[2]]
    nwin = len(slices)
    total = nwin * B
    w = roi_weight_map if roi_weight_map is not None else importance_map(roi, mode, ss)
    w = w.reshape(roi)[None, None].float()
    out = None
    count = None
    for g0 in range(0, total, sw_batch_size):
        rng = range(g0, min(g0 + sw_batch_size, total))
        win = torch.cat([inputs[i // nwin: i // nwin + 1, :, slices[i % nwin][0],
                                slices[i % nwin][1], slices[i % nwin][2]] for i in rng])
        pred = predictor(win)
        if out is None:
            out = torch.zeros([B, pred.shape[1]] + image_size, dtype=torch.float)
            count = torch.zeros([1, 1] + image_size, dtype=torch.float)
            for s in slices:
                count[(slice(None), slice(None)) + s] += w
        pred = pred * w
        for i, p in zip(rng, pred):
            out[(slice(i // nwin, i // nwin + 1), slice(None)) + slices[i % nwin]] += p
    out /= count
    if any(pad):
        z0, y0, x0 = pad[4], pad[2], pad[0]
        out = out[:, :, z0:z0 + image_size_[0], y0:y0 + image_size_[1], x0:x0 + image_size_[2]]
    return out


def stitch(patches: Tensor, wmap: Tensor, starts: Sequence[Sequence[int]],
           image_size: Sequence[int], batch: int, world: int = 1,
           slots_per_round: int = 1) -> Tensor:
    """The accumulation half alone, over an already-predicted (rows, C, *roi) patch tensor laid
    out as wf_sliding_window_stitch documents (include/waveformer_hip.h) -- same scatter and
    operation order as sliding_window_inference above."""
    roi = tuple(patches.shape[2:])
    slices = [(slice(z, z + roi[0]), slice(y, y + roi[1]), slice(x, x + roi[2]))
              for z in starts[0] for y in starts[1] for x in starts[2]]
    nwin = len(slices)
    C = patches.shape[1]
    out = torch.zeros((batch, C) + tuple(image_size), dtype=torch.float)
    count = torch.zeros((1, 1) + tuple(image_size), dtype=torch.float)
    w = wmap.reshape(roi).float().cpu()
    for s in slices:
        count[(slice(None), slice(None)) + s] += w
    p_all = patches.cpu()
    for g in range(batch * nwin):
        r, j = g % world, g // world
        row = ((j // slots_per_round) * world + r) * slots_per_round + j % slots_per_round
        out[(slice(g // nwin, g // nwin + 1), slice(None)) + slices[g % nwin]] += p_all[row] * w
    out /= count
    return out


def stitch_partial(patches: Tensor, wmap: Tensor, starts: Sequence[Sequence[int]],
                   image_size: Sequence[int], batch: int, world: int, rank: int) -> Tensor:
    """The same scatter restricted to one rank's windows (g % world == rank, local row
    g // world): (batch, C + 1, *image) = [sum pred * w | sum w], no division -- the CPU
    stand-in of wf_sliding_window_stitch_partial (the all-reduce exchange)."""
    roi = tuple(patches.shape[2:])
    slices = [(slice(z, z + roi[0]), slice(y, y + roi[1]), slice(x, x + roi[2]))
              for z in starts[0] for y in starts[1] for x in starts[2]]
    nwin = len(slices)
    C = patches.shape[1]
    out = torch.zeros((batch, C + 1) + tuple(image_size), dtype=torch.float)
    w = wmap.reshape(roi).float().cpu()
    p_all = patches.cpu()
    for g in range(rank, batch * nwin, world):
        b, s = g // nwin, slices[g % nwin]
        out[(slice(b, b + 1), slice(0, C)) + s] += p_all[g // world] * w
        out[(slice(b, b + 1), slice(C, C + 1)) + s] += w
    return out


def normalize(num: Tensor) -> Tensor:
    C = num.shape[1] - 1
    return num[:, :C] / num[:, C:]


def tta_merge(pred: Tensor, passes) -> Tensor:
    """The merge half of mirror_and_predict over stacked per-pass predictions (pass p on the
    input flipped along tensor dims passes[p]) -- the wf_tta_merge contract."""
    acc = pred[0:1].cpu().clone()
    for p in range(1, len(passes)):
        acc += torch.flip(pred[p:p + 1].cpu(), tuple(passes[p]))
    acc /= len(passes)
    return acc


def mirror_and_predict(x: Tensor, window_infer: Callable[[Tensor], Tensor],
                       mirror_axes=None) -> Tensor:
    """light_training/prediction.py:110-160 (fp32 sums in pass order, then / 2^k)."""
    pred = window_infer(x).cpu()
    if mirror_axes is None:
        return pred
    m = set(mirror_axes)
    n = 2 ** len(mirror_axes)
    for combo in [(0,), (1,), (2,), (0, 1), (0, 2), (1, 2), (0, 1, 2)]:
        if set(combo) <= m:
            dims = tuple(a + 2 for a in combo)
            pred += torch.flip(window_infer(torch.flip(x, dims)), dims).cpu()
    pred /= n
    return pred
