"""wf_conv3d_k3_wgrad at the config-4 decoder shapes (B = 4, 128^3 / 64^3), HIP events, vs the
framework's conv3d_weight (MIOpen) when --miopen 1.  usage: python tools/kbench_wgrad.py [B]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from waveformer_amd import _lib, ops  # noqa: E402

_lib.load()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for Cin, Cout, S in [(4, 48, 128), (48, 48, 128), (96, 48, 128), (96, 96, 64), (192, 192, 16)]:
    x = torch.randn(B, Cin, S, S, S, device="cuda").contiguous(memory_format=torch.channels_last_3d)
    g = torch.randn(B, Cout, S, S, S, device="cuda").contiguous(memory_format=torch.channels_last_3d)
    ops.conv3d_k3_wgrad(x, g, (Cout, Cin, 3, 3, 3))
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        ops.conv3d_k3_wgrad(x, g, (Cout, Cin, 3, 3, 3))
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 5
    fl = 2 * 27 * Cin * Cout * B * S ** 3
    print(f"wgrad B={B} {Cin}->{Cout} {S}^3: {ms * 1e3:9.1f} us  {fl / ms / 1e9:7.1f} TFLOP/s "
          f"(x3 issued {3 * fl / ms / 1e9:7.1f})", flush=True)
    del x, g
