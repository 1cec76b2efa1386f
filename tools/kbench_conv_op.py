"""ops.conv3d_k3 as config 5's decoder calls it (96 -> 48 at 192^3, B = 2, fp16 precision,
channel-last input), timed with events around REPS calls, with and without the fused
InstanceNorm statistics -- to compare the op-level time the bench's conv3d_k3 roofline reports
with the kernel's own duration under a kernel trace."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from waveformer_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
B, CI, CO, S = int(os.environ.get("B", "2")), 96, 48, int(os.environ.get("S", "192"))
REPS = 4
ops.set_precision("fp16")
g = torch.Generator(device=dev).manual_seed(0)
x = ops.empty_cl(B, CI, S, S, S, dev).normal_(generator=g)
w = torch.randn(CO, CI, 3, 3, 3, device=dev, generator=g) * 0.05
bias = torch.randn(CO, device=dev, generator=g)
for eps in (None, 1e-5):
    for _ in range(2):
        ops.conv3d_k3(x, w, bias, norm_eps=eps)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        ops.conv3d_k3(x, w, bias, norm_eps=eps)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / REPS * 1e3
    fl = 2 * 27 * CI * CO * B * S ** 3
    print(f"norm_eps={eps}: {us:.1f} us per op, {fl / us / 1e6:.1f} TFLOP/s "
          f"(precision {ops._prec() if hasattr(ops, '_prec') else '?'})", flush=True)

# the same launch replayed from a captured HIP graph (the bench's timed region replays the
# step as a graph), 10 replays of a 2-launch graph
out = ops.empty_cl(B, CO, S, S, S, dev)
st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st):
    for _ in range(2):
        ops.conv3d_k3(x, w, bias, out=out)
torch.cuda.current_stream().wait_stream(st)
torch.cuda.synchronize()
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    ops.conv3d_k3(x, w, bias, out=out)
    ops.conv3d_k3(x, w, bias, out=out)
gr.replay()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    gr.replay()
e.record()
torch.cuda.synchronize()
us = s.elapsed_time(e) / 20 * 1e3
print(f"graph replay: {us:.1f} us per conv, {2 * 27 * CI * CO * B * S ** 3 / us / 1e6:.1f} TFLOP/s",
      flush=True)
