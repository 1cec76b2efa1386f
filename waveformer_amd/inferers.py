"""Sliding-window inference for WaveFormer's prediction path (BASELINE config 3), sharded over
GPUs.

Mirrors the caller side of the hot path:
  * `sliding_window_inference` -- monai/inferers/utils.py:43-321 (non-buffered path), with the
    same argument names, window enumeration (`_get_scan_interval` :355-376,
    `dense_patch_slices` monai/data/utils.py:171-211), padding and cropping;
  * `SlidingWindowInferer` -- monai/inferers/inferer.py:382-536, as 4_predict.py:199-205
    builds it (roi 128^3, sw_batch 2, overlap 0.5, 'gaussian');
  * `maybe_mirror_and_predict` -- the 8-way flip TTA of light_training/prediction.py:110-160.

What is MI355X-specific:
  * `process_group` (default None = one process) deals the B x nW windows round-robin over
    the ranks: rank r runs the predictor on windows r, r + W, r + 2W, ... in rounds of
    `sw_batch_size`, and after every round the per-window logits are all-gathered over RCCL
    (`all_gather_into_tensor`, async, so round k's exchange overlaps round k+1's forward)
    into one (rounds, W, sw_batch, C, *roi) buffer.  Every rank then stitches the full
    output; the padded slots of the last round are zeros and never read.  The alternative
    exchange (exchange="allreduce") stitches each rank's own windows into weighted
    sums + weights and all-reduces those once per case.
  * The importance map and the stitch are HIP kernels (`ops.importance_map`,
    `ops.sliding_window_stitch`): one thread per output voxel gathers the windows covering
    it in the reference's order and divides by the summed weights -- no count-map tensor,
    no atomics, one write per output element.
  * TTA batches the 2^k flipped copies of the image as one window set, so the 8 x 18 = 144
    windows of a BraTS case split evenly over 8 GPUs, and the flip-back + sum is one gather
    kernel (`ops.tta_merge`).

Options of the MONAI function that WaveFormer's path never uses (process_fn, buffer_steps,
with_coord, tuple/dict predictor outputs, predictor outputs of another resolution) raise
NotImplementedError instead of silently doing something else.
"""
from __future__ import annotations

import math
import os
from typing import Any, Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import ops

PAD_MODES = ("constant", "reflect", "replicate", "circular")


# ------------------------------------------------------------------------------------------
# window geometry (host logic; pure Python, identical on every rank)
# ------------------------------------------------------------------------------------------
def _tuple3(v, name) -> tuple:
    if isinstance(v, (int, float)):
        return (v,) * 3
    v = tuple(v)
    if len(v) == 1:
        return v * 3
    if len(v) != 3:
        raise ValueError(f"{name}: expected 1 or 3 values, got {len(v)}")
    return v


def fall_back_roi(roi_size, image_size: Sequence[int]) -> Tuple[int, int, int]:
    """monai.utils.fall_back_tuple: None / non-positive components take the image size."""
    roi = _tuple3(roi_size, "roi_size")
    return tuple(int(i) if (r is None or r <= 0) else int(r) for r, i in zip(roi, image_size))


def scan_interval(image_size: Sequence[int], roi_size: Sequence[int],
                  overlap: Sequence[float]) -> Tuple[int, int, int]:
    """monai/inferers/utils.py:355-376."""
    out = []
    for i, r, o in zip(image_size, roi_size, overlap):
        if r == i:
            out.append(int(r))
        else:
            iv = int(r * (1 - o))
            out.append(iv if iv > 0 else 1)
    return tuple(out)


def dense_patch_starts(image_size: Sequence[int], roi_size: Sequence[int],
                       interval: Sequence[int]) -> List[List[int]]:
    """Per-axis window starts of dense_patch_slices (monai/data/utils.py:171-211); the windows
    are their 'ij' meshgrid product, last axis fastest."""
    patch = [min(i, r or i) for i, r in zip(image_size, roi_size)]  # get_valid_patch_size
    starts = []
    for i, p, s in zip(image_size, patch, interval):
        if s == 0:
            n = 1
        else:
            num = int(math.ceil(float(i) / s))
            n = next((d for d in range(num) if d * s + p >= i), None)
            n = 1 if n is None else n + 1
        st = []
        for k in range(n):
            v = k * s
            st.append(v - max(v + p - i, 0))
        starts.append(st)
    return starts


def window_slices(starts: Sequence[Sequence[int]], roi: Sequence[int]) -> List[tuple]:
    return [(slice(z, z + roi[0]), slice(y, y + roi[1]), slice(x, x + roi[2]))
            for z in starts[0] for y in starts[1] for x in starts[2]]


def shard_plan(total: int, world: int, sw_batch: int) -> Tuple[int, int]:
    """(rounds, slots per rank): window g runs on rank g % world in slot g // world; slots
    are padded to whole rounds of sw_batch windows."""
    slots = -(-total // world)
    rounds = -(-slots // sw_batch)
    return rounds, rounds * sw_batch


def pad_amounts(image_size: Sequence[int], roi: Sequence[int]) -> List[int]:
    """F.pad list (last axis first) of monai/inferers/utils.py:171-177."""
    pad = []
    for k in (2, 1, 0):
        diff = max(roi[k] - image_size[k], 0)
        half = diff // 2
        pad.extend([half, diff - half])
    return pad


# ------------------------------------------------------------------------------------------
# the inference loop
# ------------------------------------------------------------------------------------------
def _group_info(process_group) -> Tuple[int, int]:
    if process_group is None:
        return 1, 0
    if not dist.is_initialized():
        raise RuntimeError("sliding_window_inference: process_group given but torch.distributed "
                           "is not initialised")
    return dist.get_world_size(process_group), dist.get_rank(process_group)


def sliding_window_inference(inputs: torch.Tensor, roi_size, sw_batch_size: int,
                             predictor: Callable[..., torch.Tensor], overlap=0.25,
                             mode: str = "constant", sigma_scale=0.125,
                             padding_mode: str = "constant", cval: float = 0.0,
                             sw_device=None, device=None, progress: bool = False,
                             roi_weight_map: Optional[torch.Tensor] = None,
                             process_fn: Optional[Callable] = None,
                             buffer_steps: Optional[int] = None, buffer_dim: int = -1,
                             with_coord: bool = False, *args: Any,
                             process_group=None, stitch: Optional[Callable] = None,
                             weight_map_fn: Optional[Callable] = None,
                             exchange: Optional[str] = None,
                             partial_stitch: Optional[Callable] = None,
                             normalize: Optional[Callable] = None,
                             **kwargs: Any) -> torch.Tensor:
    """monai.inferers.sliding_window_inference for 3-D NCDHW inputs and a predictor returning
    one tensor of the window's spatial size.  See the module docstring for `process_group`.

    exchange (default: WF_SW_EXCHANGE or "allgather"): how the ranks' windows meet --
      "allgather": every round's window logits are all-gathered and every rank stitches the
        whole case in the reference's window order (bitwise MONAI's sums);
      "allreduce": each rank stitches only its own windows into weighted sums + summed weights
        (ops.sliding_window_stitch_partial), ONE all-reduce of those (C + 1) full-size planes,
        then a division (ops.sliding_window_normalize) -- the cheaper exchange SURVEY 8e names
        (one (C + 1) x D x H x W payload instead of every window's logits); the sums then
        meet in rank order, so the result equals the all-gather one to fp32 rounding.
    `stitch` / `weight_map_fn` / `partial_stitch` / `normalize` default to the HIP kernels;
    tests substitute the CPU oracle to exercise the sharding logic on a CPU (gloo) group."""
    if process_fn is not None or (buffer_steps is not None and buffer_steps > 0) or with_coord:
        raise NotImplementedError("process_fn / buffer_steps / with_coord are not used by "
                                  "WaveFormer's prediction path and are not implemented")
    if inputs.dim() != 5:
        raise ValueError(f"inputs must be NCDHW (5-D), got shape {tuple(inputs.shape)}")
    if sw_batch_size < 1:
        raise ValueError("sw_batch_size must be >= 1")
    ov = _tuple3(overlap, "overlap")
    for o in ov:
        if o < 0 or o >= 1:
            raise ValueError(f"overlap must be >= 0 and < 1, got {ov}.")
    if padding_mode not in PAD_MODES:
        raise ValueError(f"padding_mode must be one of {PAD_MODES}")
    world, rank = _group_info(process_group)
    stitch = stitch or ops.sliding_window_stitch
    weight_map_fn = weight_map_fn or ops.importance_map
    exchange = exchange or os.environ.get("WF_SW_EXCHANGE", "allgather")
    if exchange not in ("allgather", "allreduce"):
        raise ValueError(f"exchange must be 'allgather' or 'allreduce', got {exchange!r}")
    reduce_mode = exchange == "allreduce"
    partial_stitch = partial_stitch or ops.sliding_window_stitch_partial
    normalize = normalize or ops.sliding_window_normalize

    B = inputs.shape[0]
    image_size_ = tuple(int(v) for v in inputs.shape[2:])
    device = device or inputs.device
    sw_device = sw_device or inputs.device
    roi = fall_back_roi(roi_size, image_size_)
    image_size = tuple(max(i, r) for i, r in zip(image_size_, roi))
    pad = pad_amounts(image_size_, roi)
    if any(pad):
        inputs = F.pad(inputs, pad=pad, mode=padding_mode,
                       value=cval if padding_mode == "constant" else None)
    starts = dense_patch_starts(image_size, roi, scan_interval(image_size, roi, ov))
    slices = window_slices(starts, roi)
    nwin = len(slices)
    total = B * nwin
    rounds, slots = shard_plan(total, world, sw_batch_size)

    valid_roi = tuple(min(i, r) for i, r in zip(image_size, roi))
    if roi_weight_map is not None and valid_roi == roi:
        wmap = roi_weight_map.to(device=sw_device, dtype=torch.float32).reshape(roi)
    else:
        wmap = weight_map_fn(valid_roi, mode, _tuple3(sigma_scale, "sigma_scale"), sw_device)

    buf: Optional[torch.Tensor] = None  # (rounds, world, sw_batch, C, *roi)
    pending = []
    C_out = None
    if total < world:
        # ranks past the last window run no predictor: agree on the channel count first
        C_out = _agree_channels(inputs, slices, predictor, rank, total, process_group, sw_device,
                                args, kwargs)
    for k in range(rounds):
        gids = [rank + (k * sw_batch_size + t) * world for t in range(sw_batch_size)]
        live = [g for g in gids if g < total]
        out_k = None
        if live:
            win = torch.cat([inputs[g // nwin: g // nwin + 1, :, slices[g % nwin][0],
                                    slices[g % nwin][1], slices[g % nwin][2]] for g in live])
            out_k = predictor(win.to(sw_device), *args, **kwargs)
            if not isinstance(out_k, torch.Tensor):
                raise NotImplementedError("tuple/dict predictor outputs are not supported")
            if tuple(out_k.shape[2:]) != roi:
                raise NotImplementedError(f"predictor output spatial size {tuple(out_k.shape[2:])} "
                                          f"!= roi {roi} (zoomed outputs are not supported)")
            if out_k.shape[0] != len(live):
                raise ValueError("predictor changed the batch size")
            out_k = out_k.float()
        if buf is None:
            C = out_k.shape[1] if out_k is not None else C_out
            # all-reduce: this rank's windows only, local slot order (slot j = window
            # rank + j * world); all-gather: every rank's, per round
            shape = (rounds, 1 if reduce_mode else world, sw_batch_size, C) + roi
            buf = torch.zeros(shape, dtype=torch.float32, device=sw_device)
        if reduce_mode:
            if out_k is not None:
                buf[k, 0, :len(live)].copy_(out_k)
            continue
        mine = buf[k, rank] if world == 1 else torch.zeros_like(buf[k, rank])
        if out_k is not None:
            mine[:len(live)].copy_(out_k)
        if world > 1:
            dst = buf[k].view((world * sw_batch_size,) + tuple(buf.shape[3:]))
            pending.append((dist.all_gather_into_tensor(dst, mine, group=process_group,
                                                        async_op=True), mine))
    for work, _ in pending:
        work.wait()
    if reduce_mode:
        part = partial_stitch(buf.view((-1,) + tuple(buf.shape[3:])), wmap, starts, image_size,
                              B, world, rank)
        if world > 1:
            dist.all_reduce(part, op=dist.ReduceOp.SUM, group=process_group)
        out = normalize(part)
    else:
        out = stitch(buf.view((-1,) + tuple(buf.shape[3:])), wmap, starts, image_size, B,
                     world, sw_batch_size)
    if any(pad):
        # remove padding (monai/inferers/utils.py:303-316; outputs share the roi's resolution)
        z0, y0, x0 = pad[4], pad[2], pad[0]
        out = out[:, :, z0:z0 + image_size_[0], y0:y0 + image_size_[1], x0:x0 + image_size_[2]]
    return out.to(device)


def _agree_channels(inputs, slices, predictor, rank, total, group, sw_device, args, kwargs):
    nwin = len(slices)
    c = torch.zeros(1, dtype=torch.int64, device=sw_device)
    if rank < total:
        g = rank
        s = slices[g % nwin]
        c[0] = predictor(inputs[g // nwin: g // nwin + 1, :, s[0], s[1], s[2]].to(sw_device),
                         *args, **kwargs).shape[1]
    dist.all_reduce(c, op=dist.ReduceOp.MAX, group=group)
    return int(c.item())


class SlidingWindowInferer:
    """monai.inferers.SlidingWindowInferer (monai/inferers/inferer.py:382-536) with an extra
    `process_group` to shard the windows over the ranks of one node."""

    def __init__(self, roi_size, sw_batch_size: int = 1, overlap=0.25, mode: str = "constant",
                 sigma_scale=0.125, padding_mode: str = "constant", cval: float = 0.0,
                 sw_device=None, device=None, progress: bool = False,
                 cache_roi_weight_map: bool = False, cpu_thresh: Optional[int] = None,
                 buffer_steps: Optional[int] = None, buffer_dim: int = -1,
                 with_coord: bool = False, process_group=None,
                 exchange: Optional[str] = None) -> None:
        if mode not in ops.BLEND_MODES:
            raise ValueError(f"mode must be one of {sorted(ops.BLEND_MODES)}, got {mode!r}")
        self.roi_size = roi_size
        self.sw_batch_size = sw_batch_size
        self.overlap = overlap
        self.mode = mode
        self.sigma_scale = sigma_scale
        self.padding_mode = padding_mode
        self.cval = cval
        self.sw_device = sw_device
        self.device = device
        self.progress = progress
        self.cpu_thresh = cpu_thresh
        self.buffer_steps = buffer_steps
        self.buffer_dim = buffer_dim
        self.with_coord = with_coord
        self.process_group = process_group
        self.exchange = exchange
        self.roi_weight_map = None
        self._cache = cache_roi_weight_map

    def __call__(self, inputs: torch.Tensor, network: Callable[..., torch.Tensor], *args: Any,
                 **kwargs: Any) -> torch.Tensor:
        device = kwargs.pop("device", self.device)
        buffer_steps = kwargs.pop("buffer_steps", self.buffer_steps)
        buffer_dim = kwargs.pop("buffer_dim", self.buffer_dim)
        if device is None and self.cpu_thresh is not None and \
                inputs.shape[2:].numel() > self.cpu_thresh:
            device = "cpu"  # stitched output handed back in host memory (inferer.py:520-521)
        if self._cache and self.roi_weight_map is None and isinstance(self.roi_size, Sequence) \
                and min(self.roi_size) > 0 and inputs.is_cuda:
            self.roi_weight_map = ops.importance_map(
                self.roi_size, self.mode, _tuple3(self.sigma_scale, "sigma_scale"), inputs.device)
        return sliding_window_inference(
            inputs, self.roi_size, self.sw_batch_size, network, self.overlap, self.mode,
            self.sigma_scale, self.padding_mode, self.cval, self.sw_device, device,
            self.progress, self.roi_weight_map, None, buffer_steps, buffer_dim, self.with_coord,
            *args, process_group=self.process_group, exchange=self.exchange, **kwargs)


# ------------------------------------------------------------------------------------------
# flip test-time augmentation (light_training/prediction.py:110-160)
# ------------------------------------------------------------------------------------------
def mirror_passes(mirror_axes: Optional[Sequence[int]]) -> List[Tuple[int, ...]]:
    """The reference's pass order: no flip, then axes 0, 1, 2, (0,1), (0,2), (1,2), (0,1,2)
    restricted to mirror_axes, as tensor dims (+2)."""
    if mirror_axes is None:
        return [()]
    m = set(mirror_axes)
    order = [(0,), (1,), (2,), (0, 1), (0, 2), (1, 2), (0, 1, 2)]
    return [()] + [tuple(a + 2 for a in c) for c in order if set(c) <= m]


def maybe_mirror_and_predict(x: torch.Tensor, model: Callable[..., torch.Tensor],
                             window_infer: SlidingWindowInferer,
                             mirror_axes: Optional[Sequence[int]] = None,
                             merge: Optional[Callable] = None, **kwargs) -> torch.Tensor:
    """Predictor.maybe_mirror_and_predict: the average of the window inference over the
    image and its flips, each flipped back.  All passes go through ONE sharded window
    inference (the flipped copies are extra batch images), so with TTA the windows of every
    pass are spread over all ranks.  Output stays on the input's device."""
    passes = mirror_passes(mirror_axes)
    if mirror_axes is not None and max(mirror_axes) > x.dim() - 3:
        raise ValueError("mirror_axes does not match the dimension of the input!")
    if x.shape[0] != 1:
        raise ValueError("maybe_mirror_and_predict: one case at a time (batch 1), as the "
                         "reference's Predictor")
    with torch.no_grad():
        xs = torch.cat([x if not f else torch.flip(x, f) for f in passes])
        pred = window_infer(xs, model, **kwargs)  # (P, C, D, H, W), pass p still flipped
        merge = merge or ops.tta_merge
        return merge(pred, passes)
