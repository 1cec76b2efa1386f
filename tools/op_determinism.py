"""Per-op determinism probe of the encoder forward (the stage-2 corruption hunt).

Every HIP op of one B-volume encoder forward is captured with its inputs and output; then each
captured call is re-issued REPS times on the same inputs and its output compared BITWISE with
the captured one (no op of the encoder forward uses atomics, so any difference is a race or a
read of memory the op never wrote).  Modes per op:
  seq   -- plain repeats on the current stream, the free allocator memory filled with a
           different byte pattern before every repeat (uninitialised-read detector);
  conc  -- each repeat on stream s0 while stream s1 runs the same op on the same inputs.
The CCF_FFN op is also split into its three stage launches with a zeroed workspace, so a
difference is pinned to pwconv (h1), dwconv (h2 + partial stats) or fc (out).
For a differing output the differing rows (last axis = channels) are summarised."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from waveformer_amd import _lib, ops  # noqa: E402

B = int(os.environ.get("B", "8"))
REPS = int(os.environ.get("REPS", "12"))
MODES = os.environ.get("MODES", "seq,conc").split(",")
dev = torch.device("cuda", 0)
_lib.load()
m = bench.build_encoder(128, dev)
x = torch.randn(B, 4, 128, 128, 128, device=dev, generator=torch.Generator(device=dev).manual_seed(7))

NAMES = ["patch_embed", "dwt3d_haar", "window_attention", "msfuse", "ccf_ffn_raw",
         "_patch_merging_raw", "proj_out"]
calls = []
orig = {n: getattr(ops, n) for n in NAMES}


def _clone(o):
    if isinstance(o, torch.Tensor):
        return o.clone()
    if isinstance(o, (tuple, list)):
        return type(o)(_clone(v) for v in o)
    return o


def _hook(n):
    def f(*a, **kw):
        out = orig[n](*a, **kw)
        calls.append((n, a, kw, _clone(out)))
        return out
    return f


for n in NAMES:
    setattr(ops, n, _hook(n))
with torch.no_grad():
    m(x)
torch.cuda.synchronize()
for n in NAMES:
    setattr(ops, n, orig[n])
print(f"captured {len(calls)} op calls at B={B}", flush=True)

_pat = [0]


def poison():
    """Fill most of the allocator's free memory with a pattern that changes every call."""
    _pat[0] += 1
    free = torch.cuda.mem_get_info()[0]
    nbytes = min(int(free * 0.5), 48 << 30)
    try:
        t = torch.empty(nbytes // 4, dtype=torch.int32, device=dev)
    except RuntimeError:
        return
    vals = [0x7fc00000, 0x00000000, 0x4b800000, -1, 0x3f800000]
    t.fill_(vals[_pat[0] % len(vals)])
    del t


def flat_tensors(o):
    if isinstance(o, torch.Tensor):
        return [o]
    if isinstance(o, (tuple, list)):
        r = []
        for v in o:
            r += flat_tensors(v)
        return r
    return []


def describe(a, b):
    d = (a != b)
    if a.is_floating_point():
        d &= ~(torch.isnan(a) & torch.isnan(b))
    if not d.any():
        return None
    rows = d.reshape(-1, a.shape[-1]).any(1) if a.dim() >= 2 else d
    nr = int(rows.sum())
    idx = rows.nonzero().flatten()
    lead = a.shape[:-1]
    coords = []
    for i in idx[:6].tolist():
        c = []
        for s in reversed(lead):
            c.append(i % s)
            i //= s
        coords.append(tuple(reversed(c)))
    mx = (a.double() - b.double()).abs().nan_to_num(0).max().item()
    return (f"{int(d.sum())} elements in {nr} rows of {rows.numel()} (shape {tuple(a.shape)}), "
            f"first rows {coords}, max |diff| {mx:.3e}, chans/row {int(d.sum()) / max(nr, 1):.1f}")


def check(tag, ref, got):
    bad = []
    for i, (r, g) in enumerate(zip(flat_tensors(ref), flat_tensors(got))):
        s = describe(g, r)
        if s:
            bad.append(f"out{i}: {s}")
    if bad:
        print(f"  DIFF {tag}: " + " | ".join(bad), flush=True)
    return not bad


def ffn_stages(a, kw):
    """ccf_ffn_raw with its workspace zeroed and cloned after each stage launch."""
    (xh, stats, n2w, n2b, pww, pwb, l1w, l1b, eps1, dww, dwb, l2w, l2b, eps2, fcw, fcb) = a[:16]
    bs = a[16] if len(a) > 16 else kw.get("branch_scale")
    prec = kw.get("prec", ops.prec_id())
    Bv, D, H, W, C = xh.shape
    hid = pww.shape[0]
    pw = ops.split_weight(pww, (hid, C), prec)
    fc = ops.split_weight(fcw, prec=prec)
    out = torch.zeros_like(xh)
    wsb = _lib.query("wf_ccf_ffn_workspace_bytes", Bv, C, hid, D, H, W, prec)
    work = torch.zeros(wsb, dtype=torch.uint8, device=xh.device)
    args = (xh.data_ptr(), ops._ptr(stats), ops._ptr(n2w), ops._ptr(n2b),
            pw.data_ptr(), ops._ptr(pwb), l1w.data_ptr(), l1b.data_ptr(), float(eps1),
            dww.data_ptr(), dwb.data_ptr(), l2w.data_ptr(), l2b.data_ptr(), float(eps2),
            fc.data_ptr(), ops._ptr(fcb), ops._ptr(bs),
            out.data_ptr(), work.data_ptr(), Bv, C, hid, D, H, W, prec, ops._stream())
    res = []
    for st in (1, 2, 3):
        _lib.call("wf_ccf_ffn_stage", st, *args)
        res.append(work.clone())
    res.append(out.clone())
    return res


s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
summary = {}
with torch.no_grad():
    for ci, (n, a, kw, ref) in enumerate(calls):
        shp = tuple(a[0].shape) if isinstance(a[0], torch.Tensor) else None
        tag = f"#{ci} {n} {shp}"
        nbad = {}
        for mode in MODES:
            bad = 0
            for r in range(REPS):
                if mode == "seq":
                    poison()
                    got = orig[n](*a, **kw)
                else:
                    main = torch.cuda.current_stream()
                    s0.wait_stream(main)
                    s1.wait_stream(main)
                    with torch.cuda.stream(s1):
                        orig[n](*a, **kw)
                    with torch.cuda.stream(s0):
                        got = orig[n](*a, **kw)
                    main.wait_stream(s0)
                    main.wait_stream(s1)
                torch.cuda.synchronize()
                bad += not check(f"{tag} {mode} rep {r}", ref, got)
                del got
            nbad[mode] = bad
        if n == "ccf_ffn_raw":
            st_ref = ffn_stages(a, kw)
            torch.cuda.synchronize()
            bad = 0
            for r in range(REPS):
                poison()
                got = ffn_stages(a, kw)
                torch.cuda.synchronize()
                for k, (g, rr) in enumerate(zip(got, st_ref)):
                    if not torch.equal(g, rr):
                        bad += 1
                        if k < 3:
                            gv, rv = g.view(torch.int32), rr.view(torch.int32)
                            dd = (gv != rv).nonzero().flatten()
                            print(f"  DIFF {tag} ffn stage {k + 1} workspace: {dd.numel()} words, "
                                  f"first word offsets {dd[:8].tolist()} of {gv.numel()}", flush=True)
                        else:
                            print(f"  DIFF {tag} ffn out: {describe(g, rr)}", flush=True)
                        break
            nbad["ffn_stages"] = bad
        summary[tag] = nbad
        print(f"{tag}: " + ", ".join(f"{k} {v}/{REPS}" for k, v in nbad.items()), flush=True)
print("SUMMARY differing:", {k: v for k, v in summary.items() if any(v.values())}, flush=True)
