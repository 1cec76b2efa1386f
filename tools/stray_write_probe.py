"""Stray-write probe: all GPU memory the encoder forward does not need is held by ONE live
sentinel tensor filled with a canary; after the forward (default stream, then a side
stream) the sentinel must be intact.  A kernel writing outside its own buffers at a distance
-- harmless in a sequential run if it lands in memory that is free at that moment -- shows up
here (the multi-stream issue of DESIGN.md 6.1 needs two forwards' memory side by side)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
m = bench.build_encoder(128, dev)
B = int(os.environ.get("B", "4"))
torch.manual_seed(0)
x = torch.randn(B, 4, 128, 128, 128, device=dev)
with torch.no_grad():
    ref = [o.clone() for o in m(x)[0]]
torch.cuda.synchronize()
free, total = torch.cuda.mem_get_info()
margin = int(os.environ.get("MARGIN_GB", "24")) << 30
n = max(0, free - margin) // 4
sent = torch.empty(n, dtype=torch.int32, device=dev)
CAN = 0x5A5A5A5A
sent.fill_(CAN)
torch.cuda.synchronize()
print(f"sentinel {n * 4 / 2**30:.1f} GiB of {total / 2**30:.1f} GiB", flush=True)
for name, st in (("default stream", None), ("side stream", torch.cuda.Stream())):
    with torch.no_grad():
        if st is None:
            out = m(x)[0]
        else:
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                out = m(x)[0]
            torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    CH = 1 << 28
    bad, first = 0, []
    for i in range(0, n, CH):
        blk = sent[i:i + CH] != CAN
        c = int(blk.sum().item())
        if c and not first:
            first = [(i + j) * 4 for j in blk.nonzero()[:8].flatten().tolist()]
        bad += c
        del blk
    d = max((a - b).abs().max().item() for a, b in zip(out, ref))
    print(f"{name}: {bad} sentinel words overwritten; output diff vs reference {d:.1e}", flush=True)
    if bad:
        print("  first overwritten word offsets (bytes):", first, flush=True)
        sent.fill_(CAN)
