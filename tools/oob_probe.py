"""Out-of-bounds WRITE probe: every tensor the op wrappers allocate (torch.empty / empty_like /
new_empty inside waveformer_amd.ops and .library) is carved out of a larger buffer whose
64 KB guard bands before and after hold a canary; after every library launch the guards of
every live carve-out are checked, naming the first launch that wrote outside its buffers.
    python tools/oob_probe.py"""
import os
import sys
import weakref

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from waveformer_amd import _lib  # noqa: E402

GUARD = 64 * 1024  # bytes
CANARY = 0x5A
guards = []  # (weakref to carve-out, base buffer, nbytes)


def carve(shape, dtype, device):
    t = torch.empty(0, dtype=dtype)
    n = 1
    for d in shape:
        n *= int(d)
    nbytes = n * t.element_size()
    base = _empty_orig(GUARD * 2 + nbytes + 256, dtype=torch.uint8, device=device)
    base.fill_(CANARY)
    view = base[GUARD:GUARD + nbytes].view(dtype).view(*shape) if n else base[:0].view(dtype)
    guards.append((weakref.ref(view), base, nbytes))
    return view


_empty_orig = torch.empty
_empty_like_orig = torch.empty_like


def empty(*size, dtype=None, device=None, **kw):
    if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)):
        size = tuple(size[0])
    dev = torch.device(device) if device is not None else None
    if dev is None or dev.type != "cuda":
        return _empty_orig(*size, dtype=dtype, device=device, **kw)
    return carve(size, dtype or torch.float32, dev)


def empty_like(t, dtype=None, **kw):
    if not t.is_cuda or kw.get("memory_format") not in (None, torch.contiguous_format):
        return _empty_like_orig(t, dtype=dtype, **kw)
    return carve(tuple(t.shape), dtype or t.dtype, t.device)


def check(after):
    torch.cuda.synchronize()
    live = []
    for ref, base, nbytes in guards:
        if ref() is None:
            continue
        live.append((ref, base, nbytes))
        lo = base[:GUARD]
        hi = base[GUARD + nbytes:]
        if bool((lo != CANARY).any()) or bool((hi != CANARY).any()):
            bad_lo = int((lo != CANARY).sum())
            bad_hi = int((hi != CANARY).sum())
            print(f"OOB WRITE after {after}: buffer of {nbytes} B, {bad_lo} B clobbered before, "
                  f"{bad_hi} after", flush=True)
            raise SystemExit(1)
    guards[:] = live


_new_empty_orig = torch.Tensor.new_empty


def new_empty(self, size, dtype=None, device=None, **kw):
    if not self.is_cuda or device is not None:
        return _new_empty_orig(self, size, dtype=dtype, device=device, **kw)
    size = (size,) if isinstance(size, int) else tuple(size)
    return carve(size, dtype or self.dtype, self.device)


real_call = _lib.call
count = [0]


def call(name, *args):
    r = real_call(name, *args)
    count[0] += 1
    check(name)
    return r


_lib.call = call
dev = torch.device("cuda", 0)
torch.empty = _empty_orig  # model build and input allocation unguarded
torch.empty_like = _empty_like_orig
m = bench.build_encoder(128, dev)
x = torch.randn(int(os.environ.get("B", "2")), 4, 128, 128, 128, device=dev)
torch.empty = empty
torch.empty_like = empty_like
torch.Tensor.new_empty = new_empty
with torch.no_grad():
    out = m(x)
torch.cuda.synchronize()
print(f"no out-of-bounds write in {count[0]} library launches", flush=True)
