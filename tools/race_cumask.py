"""Concurrent encoder forwards on two streams restricted to DISJOINT halves of the CUs
(hipExtStreamCreateWithCUMask): if they still differ from the sequential reference, the
multi-stream issue is not workgroups of the two forwards sharing a CU."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
hip = ctypes.CDLL("libamdhip64.so")
m1 = bench.build_encoder(128, dev)
m2 = bench.build_encoder(128, dev)
m2.load_state_dict(m1.state_dict())
torch.manual_seed(0)
xa = torch.randn(4, 4, 128, 128, 128, device=dev)
xb = torch.randn(4, 4, 128, 128, 128, device=dev)
with torch.no_grad():
    ra = [o.clone() for o in m1(xa)[0]]
    rb = [o.clone() for o in m2(xb)[0]]
ncu = torch.cuda.get_device_properties(0).multi_processor_count
words = (ncu + 31) // 32


def masked_stream(lo, hi):
    mask = (ctypes.c_uint32 * words)()
    for c in range(lo, hi):
        mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


half = ncu // 2
for name, (sa, sb) in (("disjoint CU halves", (masked_stream(0, half), masked_stream(half, ncu))),
                       ("same CU half", (masked_stream(0, half), masked_stream(0, half)))):
    bad = 0
    for _ in range(int(os.environ.get("REPS", "4"))):
        with torch.no_grad():
            main = torch.cuda.current_stream()
            sa.wait_stream(main)
            sb.wait_stream(main)
            with torch.cuda.stream(sa):
                ga = m1(xa)[0]
            with torch.cuda.stream(sb):
                gb = m2(xb)[0]
            main.wait_stream(sa)
            main.wait_stream(sb)
            torch.cuda.synchronize()
        da = max((a - b).abs().max().item() for a, b in zip(ga, ra))
        db = max((a - b).abs().max().item() for a, b in zip(gb, rb))
        bad += (da > 0) or (db > 0)
    print(f"{name} ({ncu} CUs): {bad} runs differ", flush=True)
