"""Focused driver for the config-3 stitch (wf_sliding_window_stitch): a 240x240x155 case,
roi 128^3, overlap 0.5 (18 windows), 4 classes, gaussian map; ITERS timed launches (HIP
events on the current stream)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from waveformer_amd import inferers, ops  # noqa: E402

ITERS = int(os.environ.get("ITERS", "20"))
dev = torch.device("cuda", 0)
img, roi, C = (240, 240, 155), (128, 128, 128), 4
starts = inferers.dense_patch_starts(img, roi, inferers.scan_interval(img, roi, (0.5,) * 3))
nw = len(starts[0]) * len(starts[1]) * len(starts[2])
torch.manual_seed(0)
patches = torch.randn((nw, C) + roi, device=dev)
wmap = ops.importance_map(roi, "gaussian", (0.125,) * 3, device=dev)
for _ in range(3):
    ops.sliding_window_stitch(patches, wmap, starts, img, 1)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(ITERS):
    ops.sliding_window_stitch(patches, wmap, starts, img, 1)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / ITERS
alg = nw * C * 128 ** 3 * 4 + C * 240 * 240 * 155 * 4
print(f"stitch {nw} windows: {us:.1f} us/launch, {alg / us / 1e3:.0f} GB/s algorithmic")
