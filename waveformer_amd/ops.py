"""Python wrappers over the C-ABI (include/waveformer_hip.h).

Each wrapper validates device / dtype / shape / contiguity on the host (the C side re-checks
sizes), allocates outputs with the PyTorch caching allocator, and launches on
torch.cuda.current_stream().  They are the only way the modules in
`waveformer_amd.network_models` reach the GPU kernels; there is no CPU or eager-PyTorch
fallback -- a CPU tensor or a missing library raises.
"""
from __future__ import annotations

import ctypes
import math
import os
import threading
import weakref
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib

DETAIL_KEYS = ("aad", "ada", "add", "daa", "dad", "dda", "ddd")  # ptwt key order, band 1..7


# ------------------------------------------------------------------------------------------
# helpers
# ------------------------------------------------------------------------------------------
def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _check(t: torch.Tensor, name: str, dtype=torch.float32, contiguous=True) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor, got {type(t)}")
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{name}: waveformer_amd kernels run on the GPU only (got a {t.device} tensor); "
            "move the module and inputs to cuda")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if contiguous and not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous tensor")


# ------------------------------------------------------------------------------------------
# precision of the MFMA operands (include/waveformer_hip.h, WF_PREC_*)
# ------------------------------------------------------------------------------------------
PRECISIONS = {"bf16": 0, "bf16x3": 1, "fp16": 2}
FP16 = PRECISIONS["fp16"]
_precision = os.environ.get("WAVEFORMER_PRECISION", "bf16x3")  # the process default
if _precision not in PRECISIONS:
    raise ValueError(f"WAVEFORMER_PRECISION={_precision!r}: expected one of {sorted(PRECISIONS)}")
# Scoped overrides (`precision`, `op_precision`) live in thread-local state: a forward that
# switches an op group to bf16x3 never changes what another thread's forward sees, and
# overlapping scopes of two threads cannot restore each other's value.
_prec_tls = threading.local()


def set_precision(p: str) -> None:
    """'bf16x3' (default): fp32-faithful split-bf16 MFMA operands, fp32 intermediates.
    'bf16': plain bf16 operands and bf16 GEMM-to-GEMM intermediates (fastest).
    'fp16': fp16 operands (10-bit mantissa) on the f16 MFMA pipes, fp32 intermediates
    (config 5's fp16 MFMA path).  Sets the process-wide default; a `precision` scope of the
    calling thread still takes precedence inside it."""
    global _precision
    if p not in PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {p!r}")
    _precision = p


def get_precision() -> str:
    """The precision in effect on this thread: its innermost scope, else the default."""
    o = getattr(_prec_tls, "override", None)
    return _precision if o is None else o


class precision:
    """Context manager: `with ops.precision("bf16"): model(x)` -- for the calling thread only."""

    def __init__(self, p: str):
        if p not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {p!r}")
        self.p = p

    def __enter__(self):
        self.prev = getattr(_prec_tls, "override", None)
        _prec_tls.override = self.p
        return self

    def __exit__(self, *exc):
        _prec_tls.override = self.prev


def _prec() -> int:
    return PRECISIONS[get_precision()]


def prec_id() -> int:
    """WF_PREC_* id of the precision in effect on this thread."""
    return PRECISIONS[get_precision()]


# The fp16 precision policy (config 5).  fp16 operands everywhere except the ops whose rounding
# spends the Dice margin, which keep the fp32-faithful bf16x3 split: measured by
# tools/prec_attrib.py on the 192^3 HF model against the reference's labels, each op group
# alone at fp16 (the rest bf16x3): window attention 2.7e-3, all decoder convolutions 1.5e-3 --
# of which encoder2/3/4's first conv (the convolutions reading the transformer's skip features)
# 1.1e-3 / 7e-4 / 4.5e-4, every other conv <= 2.6e-4 --, PatchMerging 3.2e-4, CCF_FFN 2.3e-4,
# 1x1 GEMMs 1.1e-4.  With attention and those three convolutions split, the whole model lands at
# Dice delta 6.7e-4 (north star: <= 1e-3); they are ~5 % of config 5's MFMA work.
FP16_SPLIT_OPS = frozenset({"attn", "skip_conv"})


def op_prec(kind: str) -> int:
    """WF_PREC_* id an op of `kind` runs at under the precision in effect on this thread."""
    cur = get_precision()
    if cur == "fp16" and kind in FP16_SPLIT_OPS:
        return PRECISIONS["bf16x3"]
    return PRECISIONS[cur]


class op_precision(precision):
    """`with ops.op_precision("skip_conv"): ...` -- the precision an op of `kind` runs at
    (the fp16 policy's exceptions switch this thread to bf16x3 inside; otherwise a no-op)."""

    def __init__(self, kind: str):
        self.kind = kind

    def __enter__(self):
        self.prev = getattr(_prec_tls, "override", None)
        cur = get_precision()
        self.p = "bf16x3" if op_prec(self.kind) != PRECISIONS[cur] else cur
        _prec_tls.override = self.p
        return self


# ------------------------------------------------------------------------------------------
# per-forward weight preparation: the bf16 hi / lo planes (and other derived forms) of the
# fp32 parameters are rebuilt at the start of every top-level forward, never cached across
# forwards -- a cache keyed on (data_ptr, _version) goes stale when a caller writes a weight
# through .data (EMA, weight surgery), which bumps no version.  A model's split weights are
# re-split together in ONE launch (WeightArena); inside a HIP graph that launch is captured
# too, so replays always see the current weights.
# ------------------------------------------------------------------------------------------
class WeightArena:
    """The [2][numel] 16-bit planes of a list of fp32 CUDA weights in one buffer -- bf16
    {hi, lo} (f16=False) or {fp16, 0} (f16=True, WF_PREC_FP16) -- refreshed by one
    wf_split_f32_to_bf16x2_multi / wf_cast_f32_to_f16x2_multi launch.

    Stream safety: the forward that used the arena last records an event on its stream when
    its scope closes; a refresh issued on another stream waits for that event first, so a
    forward on stream B never rewrites planes that stream A's kernels still read (graph
    capture skips the event: a captured graph replays on its own stream, in order).  Arenas
    are per thread (weight_scope), so this ordering is only ever between one thread's
    successive forwards."""

    def __init__(self, params: Sequence[torch.Tensor], f16: bool = False):
        dev = params[0].device
        self.f16 = f16
        self.key = tuple((p.data_ptr(), p.numel()) for p in params)
        pre, dsts, off = [0], [], 0
        blocks = []
        for p in params:
            blocks.append(off)
            off += 2 * p.numel()            # numel % 8 == 0: every plane stays 16-B aligned
        self.buf = torch.empty(max(off, 8), dtype=torch.bfloat16, device=dev)
        self.views: Dict[int, torch.Tensor] = {}
        for p, o in zip(params, blocks):
            v = self.buf[o:o + 2 * p.numel()]
            self.views[p.data_ptr()] = v
            dsts.append(v.data_ptr())
            pre.append(pre[-1] + p.numel())
        self.n, self.total = len(params), pre[-1]
        table = pre + [p.data_ptr() for p in params] + dsts
        self.table = torch.tensor(table, dtype=torch.int64).to(dev)
        self.done: Optional[torch.cuda.Event] = None   # last forward's end, on done_stream
        self.done_stream = None

    def refresh(self) -> None:
        cur = torch.cuda.current_stream(self.buf.device)
        if (self.done is not None and self.done_stream != cur.cuda_stream
                and not torch.cuda.is_current_stream_capturing()):
            cur.wait_event(self.done)
        _lib.call("wf_cast_f32_to_f16x2_multi" if self.f16 else "wf_split_f32_to_bf16x2_multi",
                  self.table.data_ptr(), self.n, self.total, cur.cuda_stream)

    def release(self) -> None:
        """The forward that refreshed the arena has issued its last kernel."""
        if torch.cuda.is_current_stream_capturing():
            return
        cur = torch.cuda.current_stream(self.buf.device)
        if self.done is None:
            self.done = torch.cuda.Event()
        self.done.record(cur)
        self.done_stream = cur.cuda_stream

    def retire(self) -> None:
        """Dropped from its module: wait for the last forward that read the planes (it may
        have run on a stream other than the buffer's allocation stream, whose cache the
        memory returns to)."""
        if self.done is not None:
            self.done.synchronize()


class _Scope:
    def __init__(self, arena: Optional[WeightArena]):
        self.arena = arena
        self.cache: Dict[tuple, torch.Tensor] = {}


_tls = threading.local()  # the open weight_scope of THIS thread (two threads: two scopes)
_arena_lock = threading.Lock()
# module -> {thread: {f16: WeightArena}}; outside the module, so copies / pickles of a model
# carry no arenas, and a dropped model drops its arenas
_ARENAS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def arena_count(module: torch.nn.Module) -> int:
    """The weight arenas `module` holds (one per live thread and operand format)."""
    with _arena_lock:
        return sum(len(per) for per in _ARENAS.get(module, {}).values())


def _cur_scope() -> Optional[_Scope]:
    return getattr(_tls, "scope", None)


def split_params(module: torch.nn.Module) -> List[torch.Tensor]:
    """The fp32 CUDA weights `module` feeds to the MFMA kernels as split operands (each
    module that has some lists them in `_wf_split_params()`)."""
    seen, out = set(), []
    for m in module.modules():
        fn = getattr(m, "_wf_split_params", None)
        if fn is None:
            continue
        for p in fn():
            if (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()
                    and p.numel() % 8 == 0 and p.data_ptr() not in seen):
                seen.add(p.data_ptr())
                out.append(p)
    return out


class weight_scope:
    """`with ops.weight_scope(model): ...` -- one forward of `model`: its split weights are
    re-split in one launch on entry and looked up by every kernel wrapper inside; derived
    forms of other weights (packed conv weights, dense attention biases) are made once per
    scope.  Nested scopes reuse the outer one.  Scopes are per thread."""

    def __init__(self, module: torch.nn.Module):
        self.module = module
        self.owner = False

    def __enter__(self):
        if _cur_scope() is not None:
            return self
        arena = None
        params = split_params(self.module)
        if params:
            # the operand format this forward's kernels read: fp16 for an fp16 inference
            # forward, else bf16 hi / lo (training always runs fp32-faithful bf16x3)
            train = torch.is_grad_enabled() and any(p.requires_grad for p in params)
            f16 = get_precision() == "fp16" and not train
            # one arena per (thread, operand format): two threads running forwards of one
            # model on their own streams never share planes or the done / done_stream pair
            # (ADVICE r3 #3); the dict itself is guarded by a lock.  Keyed by the Thread
            # object (an ident is reused by later threads); the arenas of threads that have
            # ended, and an arena whose parameters moved, are retired at the next scope entry
            # (one weight copy per thread identity, never freed)
            with _arena_lock:
                arenas = _ARENAS.get(self.module)
                if arenas is None:
                    arenas = {}
                    _ARENAS[self.module] = arenas
                for th in [t for t in arenas if not t.is_alive()]:
                    for old in arenas.pop(th).values():
                        old.retire()
                per = arenas.setdefault(threading.current_thread(), {})
                arena = per.get(f16)
                if arena is None or arena.key != tuple((p.data_ptr(), p.numel()) for p in params):
                    if arena is not None:
                        arena.retire()
                    arena = WeightArena(params, f16)
                    per[f16] = arena
            arena.refresh()
        _tls.scope = _Scope(arena)
        self.owner = True
        return self

    def __exit__(self, *exc):
        if self.owner:
            sc = _cur_scope()
            if sc is not None and sc.arena is not None:
                sc.arena.release()
            _tls.scope = None


def per_forward(key: tuple, make):
    """make() once per weight_scope (once per call outside any scope).  The value's producing
    stream is remembered with an event: a Block runs its coarser wavelet levels on a side
    stream (network_models/wave_helper.py), and a consumer on another stream must wait for the
    kernel that made the cached operand (an fp16-policy forward splits the attention weights
    on whichever stream first asks for them)."""
    sc = _cur_scope()
    if sc is None:
        return make()
    hit = sc.cache.get(key)
    if hit is None:
        v = make()
        ev = st = None
        if isinstance(v, torch.Tensor) and v.is_cuda:
            st = torch.cuda.current_stream(v.device)
            ev = torch.cuda.Event()
            ev.record(st)
        sc.cache[key] = (v, ev, st)
        return v
    v, ev, st = hit
    if ev is not None:
        cur = torch.cuda.current_stream(v.device)
        if cur != st:
            cur.wait_event(ev)
    return v


def split_weight(p: torch.Tensor, shape: Optional[Tuple[int, ...]] = None,
                 prec: Optional[int] = None) -> torch.Tensor:
    """[2][N][K] 16-bit operand planes of an fp32 weight for kernels running at `prec`:
    bf16 {hi, lo} (wf_split_f32_to_bf16x2), or {fp16, 0} for WF_PREC_FP16
    (wf_cast_f32_to_f16x2).  The weight arena's view inside a weight_scope, else made now."""
    shp = (2,) + tuple(p.shape if shape is None else shape)
    f16 = (_prec() if prec is None else prec) == FP16
    sc = _cur_scope()
    if sc is not None and sc.arena is not None and sc.arena.f16 == f16:
        v = sc.arena.views.get(p.data_ptr())
        if v is not None and v.numel() == 2 * p.numel():
            return v.view(shp)

    def make():
        src = p.detach()
        _check(src, "weight")
        out = torch.empty(shp, dtype=torch.bfloat16, device=src.device)  # 16-bit words
        _lib.call("wf_cast_f32_to_f16x2" if f16 else "wf_split_f32_to_bf16x2", src.data_ptr(),
                  out.data_ptr(), src.numel(), _stream())
        return out
    return per_forward(("split", p.data_ptr(), shp, f16), make)


# ------------------------------------------------------------------------------------------
# a10: PatchEmbed conv
# ------------------------------------------------------------------------------------------
def patch_embed(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    """Conv3d(k=2, s=2) NCDHW -> channel-last (B, D/2, H/2, W/2, Cout)."""
    _check(x, "x")
    _check(weight, "weight")
    B, Cin, D2, H2, W2 = x.shape
    Cout = weight.shape[0]
    if tuple(weight.shape) != (Cout, Cin, 2, 2, 2):
        raise ValueError(f"patch_embed: weight {tuple(weight.shape)} is not ({Cout},{Cin},2,2,2)")
    if D2 % 2 or H2 % 2 or W2 % 2:
        raise ValueError("patch_embed: spatial sizes must be even (PatchEmbed pads otherwise)")
    if bias is not None:
        _check(bias, "bias")
    out = torch.empty((B, D2 // 2, H2 // 2, W2 // 2, Cout), dtype=torch.float32, device=x.device)
    _lib.call("wf_patch_embed_fwd", x.data_ptr(), weight.data_ptr(), _ptr(bias), out.data_ptr(),
              B, Cin, Cout, D2 // 2, H2 // 2, W2 // 2, _stream())
    return out


def patch_embed_ll(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                   ln: Tuple[torch.Tensor, torch.Tensor, float]
                   ) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
    """patch_embed fused with the first Block's norm1 + Haar LL (wf_patch_embed_ll_fwd):
    (out, LL of LayerNorm(out)), or None when the shape is not the kernel's (Cin 1 / 4, Cout 48,
    even output sizes, output W <= 64, fewer than 2^31 output elements) -- the caller then runs
    patch_embed + the LL-only DWT."""
    B, Cin, D2, H2, W2 = x.shape
    Cout = weight.shape[0]
    D, H, W = D2 // 2, H2 // 2, W2 // 2
    if (Cout != 48 or Cin not in (1, 4) or tuple(weight.shape) != (Cout, Cin, 2, 2, 2)
            or D2 % 2 or H2 % 2 or W2 % 2 or D % 2 or H % 2 or W % 2 or W > 64
            or B * D * H * W * Cout >= 1 << 31):  # the kernel's 32-bit element indexing
        return None
    _check(x, "x")
    _check(weight, "weight")
    lw, lb, eps = ln
    _check(lw, "ln_w")
    _check(lb, "ln_b")
    if bias is not None:
        _check(bias, "bias")
    out = torch.empty((B, D, H, W, Cout), dtype=torch.float32, device=x.device)
    ll = torch.empty((B, D // 2, H // 2, W // 2, Cout), dtype=torch.float32, device=x.device)
    _lib.call("wf_patch_embed_ll_fwd", x.data_ptr(), weight.data_ptr(), _ptr(bias),
              out.data_ptr(), lw.data_ptr(), lb.data_ptr(), float(eps), ll.data_ptr(), B, Cin,
              Cout, D, H, W, _stream())
    return out, ll


# ------------------------------------------------------------------------------------------
# a1: Haar analysis
# ------------------------------------------------------------------------------------------
def dwt3d_haar(x_cl: torch.Tensor, ln: Optional[Tuple[torch.Tensor, torch.Tensor, float]] = None
               ) -> torch.Tensor:
    """1-level Haar DWT of a channel-last (B,D,H,W,C) volume -> bands (8,B,D/2,H/2,W/2,C)."""
    _check(x_cl, "x")
    B, D, H, W, C = x_cl.shape
    bands = torch.empty((8, B, D // 2, H // 2, W // 2, C), dtype=torch.float32, device=x_cl.device)
    lw = lb = None
    eps = 0.0
    if ln is not None:
        lw, lb, eps = ln
        _check(lw, "ln_w")
        _check(lb, "ln_b")
    _lib.call("wf_dwt3d_haar_fwd", x_cl.data_ptr(), _ptr(lw), _ptr(lb), float(eps),
              bands.data_ptr(), B, C, D, H, W, _stream())
    return bands


def dwt3d_haar_ll(x_cl: torch.Tensor, ln: Optional[Tuple[torch.Tensor, torch.Tensor, float]] = None
                  ) -> torch.Tensor:
    """The LL band of dwt3d_haar alone (wf_dwt3d_haar_fwd_ll): (B,D,H,W,C) -> (B,D/2,H/2,W/2,C),
    bitwise band 0 of dwt3d_haar, for Blocks whose detail bands are never read."""
    _check(x_cl, "x")
    B, D, H, W, C = x_cl.shape
    ll = torch.empty((B, D // 2, H // 2, W // 2, C), dtype=torch.float32, device=x_cl.device)
    lw = lb = None
    eps = 0.0
    if ln is not None:
        lw, lb, eps = ln
        _check(lw, "ln_w")
        _check(lb, "ln_b")
    _lib.call("wf_dwt3d_haar_fwd_ll", x_cl.data_ptr(), _ptr(lw), _ptr(lb), float(eps),
              ll.data_ptr(), B, C, D, H, W, _stream())
    return ll


def bands_to_coeffs(bands) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """(8,B,d,h,w,C) bands (or their 8 unbound (B,d,h,w,C) views) -> (LL, detail dict) as
    NCDHW-shaped (channel-last strided) views, the structure ptwt.wavedec3(level=1) returns
    (wave_helper.py:350-353)."""
    ll = bands[0].permute(0, 4, 1, 2, 3)
    det = {k: bands[i + 1].permute(0, 4, 1, 2, 3) for i, k in enumerate(DETAIL_KEYS)}
    return ll, det


# ------------------------------------------------------------------------------------------
# a11: Haar synthesis
# ------------------------------------------------------------------------------------------
def idwt3d_haar(ll: torch.Tensor, details: Sequence[Dict[str, torch.Tensor]],
                out: Optional[torch.Tensor] = None,
                skip: Optional[torch.Tensor] = None) -> torch.Tensor:
    """ptwt.waverec3((ll,) + tuple(details), 'db1') for NCDHW-shaped tensors of any strides
    inside each (B, C, ...) batch with contiguous spatial (y, x) rows or channel-last layout.

    `details` is coarse -> fine.  If `out` is given (B, >=C, 2^L d, 2^L h, 2^L w) with a
    contiguous (C, D, H, W) block per batch, the result is written into its first C channels
    (this is how the decoder fuses torch.cat((out, skip), 1), idwt_upsample.py:163).  With
    `skip` (B, C, ...) as well, channels [C, 2C) of `out` receive it -- in the same kernel
    (wf_idwt3d_haar_cl_cat) when everything is channel-last, else by a copy."""
    if ll.device.type != "cuda":
        raise RuntimeError("idwt3d_haar: GPU tensors only")
    if ll.dtype != torch.float32:
        raise TypeError("idwt3d_haar: float32 only")
    B, C, d, h, w = ll.shape
    ll_ld = cl_ld(ll)  # a channel-last LL is read in place by the channel-last entry
    if ll_ld is None and ll.stride()[1:] != (d * h * w, h * w, w, 1):
        ll = ll.contiguous()
    L = len(details)
    if not 1 <= L <= 4:
        raise ValueError("idwt3d_haar: 1..4 detail levels supported")
    ptrs: List[int] = []
    strides: List[int] = []
    keep = []
    for l, dct in enumerate(details):
        s = 2 ** l
        exp = (B, C, d * s, h * s, w * s)
        ts = []
        for k in DETAIL_KEYS:
            t = dct[k]
            if tuple(t.shape) != exp:
                raise ValueError(f"idwt3d_haar: level {l} key {k} has shape {tuple(t.shape)}, expected {exp}")
            if t.device != ll.device or t.dtype != torch.float32:
                raise TypeError("idwt3d_haar: detail tensors must be float32 on the same GPU")
            ts.append(t)

        def pattern(t):  # element (b,c,z,y,x) at b*s0 + c*s1 + z*s2 + (y*W_l + x)*s3
            st = t.stride()
            return (st[0], st[1], st[2], st[4]) if st[3] == exp[4] * st[4] else None

        pats = [pattern(t) for t in ts]
        if any(p is None for p in pats) or len(set(pats)) != 1:
            ts = [t.contiguous() for t in ts]
            pats = [pattern(t) for t in ts]
        keep.extend(ts)
        ptrs.extend(t.data_ptr() for t in ts)
        strides.extend(pats[0])
    Do, Ho, Wo = d * 2 ** L, h * 2 ** L, w * 2 ** L
    ldo = None
    if out is None:
        out = torch.empty((B, C, Do, Ho, Wo), dtype=torch.float32, device=ll.device)
    else:
        if out.shape[0] != B or out.shape[1] < C or tuple(out.shape[2:]) != (Do, Ho, Wo):
            raise ValueError(f"idwt3d_haar: out {tuple(out.shape)} does not fit ({B},{C},{Do},{Ho},{Wo})")
        ldo = cl_ld(out)  # channel-last output (channels contiguous, positions ldo apart)
        if ldo is None and out.stride()[1:] != (Do * Ho * Wo, Ho * Wo, Wo, 1):
            raise ValueError("idwt3d_haar: out must be channel-last or contiguous inside each batch")
    arr = (ctypes.c_void_p * len(ptrs))(*ptrs)
    sarr = (ctypes.c_int64 * len(strides))(*strides)
    if ll_ld is not None and ldo is None:
        ll, ll_ld = ll.contiguous(), None  # the NCDHW-output entry reads an NCDHW LL
    if skip is not None and (out is None or out.shape[1] < 2 * C or tuple(skip.shape) != (B, C, Do, Ho, Wo)):
        raise ValueError("idwt3d_haar: skip must be (B, C, ...) of the output and out >= 2C channels")
    skip_ld = cl_ld(skip) if skip is not None else None
    fused = (skip is not None and ldo is not None and ll_ld is not None and skip_ld is not None
             and C % 4 == 0 and skip.device == out.device and skip.dtype == torch.float32
             and skip.stride(0) % 4 == 0 and skip.data_ptr() % 16 == 0
             # the debug switch WF_IDWT_SCALAR (read per call by the library) selects the scalar
             # kernel, which has no fused concat: IDWT + copy then
             and "WF_IDWT_SCALAR" not in os.environ)
    if fused:
        _lib.call("wf_idwt3d_haar_cl_cat", ll.data_ptr(), ll.stride(0), 1, ll_ld, arr, sarr, L,
                  skip.data_ptr(), skip.stride(0), skip_ld, out.data_ptr(), out.stride(0), ldo,
                  B, C, d, h, w, _stream())
    elif ldo is not None:
        ll_cs, ll_ps = (1, ll_ld) if ll_ld is not None else (d * h * w, 1)
        _lib.call("wf_idwt3d_haar_cl", ll.data_ptr(), ll.stride(0), ll_cs, ll_ps, arr, sarr, L,
                  out.data_ptr(), out.stride(0), ldo, B, C, d, h, w, _stream())
    else:
        _lib.call("wf_idwt3d_haar", ll.data_ptr(), ll.stride(0), arr, sarr, L, out.data_ptr(),
                  out.stride(0), B, C, d, h, w, _stream())
    if skip is not None and not fused:
        copy_cl(skip, out[:, C:2 * C])
    del keep
    return out


# ------------------------------------------------------------------------------------------
# C5: general orthogonal wavelets (db1..db4), NCDHW, any sizes
# ------------------------------------------------------------------------------------------
# pywt.Wavelet(name).(dec_lo, dec_hi, rec_lo, rec_hi) -- PyWavelets' filter banks, which ptwt
# 0.1.9 uses (requirements.txt:45); values printed by PyWavelets 1.1.1.
WAVELETS: Dict[str, Tuple[Tuple[float, ...], ...]] = {
    "db1": ((0.7071067811865476, 0.7071067811865476), (-0.7071067811865476, 0.7071067811865476),
            (0.7071067811865476, 0.7071067811865476), (0.7071067811865476, -0.7071067811865476)),
    "db2": ((-0.12940952255126037, 0.2241438680420134, 0.8365163037378079, 0.48296291314453416),
            (-0.48296291314453416, 0.8365163037378079, -0.2241438680420134, -0.12940952255126037),
            (0.48296291314453416, 0.8365163037378079, 0.2241438680420134, -0.12940952255126037),
            (-0.12940952255126037, -0.2241438680420134, 0.8365163037378079, -0.48296291314453416)),
    "db3": ((0.03522629188570953, -0.08544127388202666, -0.13501102001025458,
             0.45987750211849154, 0.8068915093110925, 0.33267055295008263),
            (-0.33267055295008263, 0.8068915093110925, -0.45987750211849154,
             -0.13501102001025458, 0.08544127388202666, 0.03522629188570953),
            (0.33267055295008263, 0.8068915093110925, 0.45987750211849154,
             -0.13501102001025458, -0.08544127388202666, 0.03522629188570953),
            (0.03522629188570953, 0.08544127388202666, -0.13501102001025458,
             -0.45987750211849154, 0.8068915093110925, -0.33267055295008263)),
    "db4": ((-0.010597401785069032, 0.0328830116668852, 0.030841381835560764,
             -0.18703481171909309, -0.027983769416859854, 0.6308807679298589,
             0.7148465705529157, 0.2303778133088965),
            (-0.2303778133088965, 0.7148465705529157, -0.6308807679298589,
             -0.027983769416859854, 0.18703481171909309, 0.030841381835560764,
             -0.0328830116668852, -0.010597401785069032),
            (0.2303778133088965, 0.7148465705529157, 0.6308807679298589,
             -0.027983769416859854, -0.18703481171909309, 0.030841381835560764,
             0.0328830116668852, -0.010597401785069032),
            (-0.010597401785069032, -0.0328830116668852, 0.030841381835560764,
             0.18703481171909309, -0.027983769416859854, -0.6308807679298589,
             0.7148465705529157, -0.2303778133088965)),
}
WAVELETS["haar"] = WAVELETS["db1"]


def _filters(wavelet: str):
    name = str(getattr(wavelet, "name", wavelet))
    if name not in WAVELETS:
        raise NotImplementedError(f"wavelet {name!r}: only {sorted(WAVELETS)} are implemented")
    return [(ctypes.c_float * len(f))(*f) for f in WAVELETS[name]], len(WAVELETS[name][0])


def dwt3d(x: torch.Tensor, wavelet: str) -> torch.Tensor:
    """One level of ptwt.wavedec3(x, wavelet, mode='zero') over the last three axes of an
    NCDHW tensor -> bands (8, B, C, d, h, w), d = (D + L - 1) // 2; band 0 = LL, 1..7 = the
    DETAIL_KEYS (wave_helper.py:350 with a non-Haar wavelet; config 5)."""
    _check(x, "x", contiguous=False)
    if x.dim() != 5:
        raise ValueError(f"dwt3d: expected (B, C, D, H, W), got {tuple(x.shape)}")
    x = x.contiguous()
    (lo, hi, _, _), L = _filters(wavelet)
    B, C, D, H, W = x.shape
    bands = torch.empty((8, B, C, (D + L - 1) // 2, (H + L - 1) // 2, (W + L - 1) // 2),
                        dtype=torch.float32, device=x.device)
    _lib.call("wf_dwt3d_fwd", x.data_ptr(), bands.data_ptr(), B * C, D, H, W, lo, hi, L,
              _stream())
    return bands


def wavedec3(x: torch.Tensor, wavelet: str, level: int) -> List:
    """ptwt.wavedec3(x, wavelet, mode='zero', level=level) -> [LL, dict_coarsest, ...,
    dict_finest] (wave_helper.py:350); every tensor is a view of its level's band buffer."""
    if level < 1:
        raise ValueError("wavedec3: level must be >= 1")
    dets = []
    cur = x
    for _ in range(level):
        bands = dwt3d(cur, wavelet)
        dets.append({k: bands[i + 1] for i, k in enumerate(DETAIL_KEYS)})
        cur = bands[0]
    return [cur] + dets[::-1]


def waverec3(coeffs: Sequence, wavelet: str, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """ptwt.waverec3((LL, dict_coarsest, ..., dict_finest), wavelet) (idwt_upsample.py:160).

    Each level is one wf_idwt3d_level launch reading LL and the 7 details through their own
    strides (an LL one sample longer than the details is cropped to them, pywt's rule).  If
    `out` is given it receives the finest level: a (B, C, Oz, Oy, Ox) view whose (z, y, x) block
    is contiguous, e.g. the first C channels of the decoder's concatenation buffer."""
    (_, _, rlo, rhi), L = _filters(wavelet)
    x = coeffs[0]
    _check(x, "LL", contiguous=False)
    nlev = len(coeffs) - 1
    if nlev < 1:
        raise ValueError("waverec3: need at least one detail level")
    for li, det in enumerate(coeffs[1:]):
        ts = [det[k] for k in DETAIL_KEYS]
        shp = tuple(ts[0].shape)
        for k, t in zip(DETAIL_KEYS, ts):
            _check(t, f"detail {k}", contiguous=False)
            if tuple(t.shape) != shp or t.device != x.device:
                raise ValueError(f"waverec3: level {li} detail {k} has shape {tuple(t.shape)}, "
                                 f"expected {shp}")
        if x.dim() != 5 or tuple(x.shape[:2]) != shp[:2] or any(
                a < b or a > b + 1 for a, b in zip(x.shape[2:], shp[2:])):
            raise ValueError(f"waverec3: LL {tuple(x.shape)} does not fit details {shp}")
        x = x[..., :shp[2], :shp[3], :shp[4]]
        B, C, nz, ny, nx = shp
        O = tuple(2 * n - L + 2 for n in shp[2:])
        last = li == nlev - 1
        if last and out is not None:
            if tuple(out.shape) != (B, C) + O or out.stride()[2:] != (O[1] * O[2], O[2], 1):
                raise ValueError(f"waverec3: out {tuple(out.shape)} / {out.stride()} does not "
                                 f"fit ({B},{C})+{O} with a contiguous (z, y, x) block")
            o = out
        else:
            o = torch.empty((B, C) + O, dtype=torch.float32, device=x.device)
        src = [x] + ts
        ptrs = (ctypes.c_void_p * 8)(*[t.data_ptr() for t in src])
        st = (ctypes.c_int64 * 40)(*[s for t in src for s in t.stride()])
        _lib.call("wf_idwt3d_level", ptrs, st, B, C, nz, ny, nx, rlo, rhi, L, o.data_ptr(),
                  o.stride(0), o.stride(1), _stream())
        x = o
    return x


# ------------------------------------------------------------------------------------------
# decoder convolution stack: channel-last 3x3x3 conv, InstanceNorm, act
# ------------------------------------------------------------------------------------------
def cl_ld(x: torch.Tensor) -> Optional[int]:
    """Position stride of an NCDHW-shaped tensor stored channel-last (a channels_last_3d
    tensor or a channel slice of one), or None if it is not laid out that way."""
    if x.dim() != 5:
        return None
    B, C, D, H, W = x.shape
    s = x.stride()
    ld = s[4] if W > 1 else (s[3] if H > 1 else (s[2] if D > 1 else max(C, 1)))
    if (C > 1 and s[1] != 1) or ld < C or ld % 4 or x.data_ptr() % 16:
        return None
    if (W > 1 and s[4] != ld) or (H > 1 and s[3] != W * ld) or (D > 1 and s[2] != H * W * ld):
        return None
    if B > 1 and s[0] != D * H * W * ld:
        return None
    return ld


def resample_trilinear_cf(x: torch.Tensor, size: Sequence[int], dtype=torch.float16,
                          align_corners: bool = False) -> torch.Tensor:
    """(C, d, h, w) -> (C, *size) trilinear resampling of every channel
    (F.interpolate(x[c][None, None], size, mode='trilinear', align_corners)), output `dtype`
    fp16 or fp32 (wf_resample_trilinear_cf): Predictor.predict_raw_probability's resample."""
    if x.dim() != 4:
        raise ValueError(f"resample_trilinear_cf: (C, d, h, w) expected, got {tuple(x.shape)}")
    if dtype not in (torch.float16, torch.float32):
        raise TypeError("resample_trilinear_cf: fp16 or fp32 output")
    x = x if x.dtype == torch.float32 else x.float()
    if x.stride()[1:] != (x.shape[2] * x.shape[3], x.shape[3], 1):
        x = x.contiguous()
    _check(x, "x", contiguous=False)
    C, d, h, w = x.shape
    D, H, W = (int(v) for v in size)
    out = torch.empty((C, D, H, W), dtype=dtype, device=x.device)
    _lib.call("wf_resample_trilinear_cf", x.data_ptr(), x.stride(0), C, d, h, w, D, H, W,
              int(bool(align_corners)), out.data_ptr(), int(dtype == torch.float16), _stream())
    return out


def hf_refine(details: Dict[str, torch.Tensor], mod) -> Dict[str, torch.Tensor]:
    """HFRefinementRes (idwt_upsample.py:12-50) of the 7 detail tensors of one level in one
    wf_hf_refine_fwd call (two passes: depthwise conv + InstanceNorm moments, then conv +
    norm + ReLU + 1x1 conv + sigmoid + product).  details: {key: (B, C, D, H, W)} channel-last
    views (the DWT's detail bands); returns the refined tensors the same way, as views of one
    (7, B, D, H, W, C) buffer (what idwt3d_haar reads)."""
    ts = [details[k] for k in DETAIL_KEYS]
    B, C, D, H, W = ts[0].shape
    P = D * H * W

    def dense_cl(t):  # (b, c, z, y, x) at b*s0 + ((z*H + y)*W + x)*C + c
        st = t.stride()
        return cl_ld(t) == C and st[2:] == (H * W * C, W * C, C)
    ts = [t if dense_cl(t) else t.contiguous(memory_format=torch.channels_last_3d) for t in ts]
    if len({t.stride(0) for t in ts}) != 1:
        ts = [t.contiguous(memory_format=torch.channels_last_3d) for t in ts]
    for t in ts:
        if tuple(t.shape) != (B, C, D, H, W):
            raise ValueError("hf_refine: the 7 detail tensors must share one shape")
        _check(t, "detail", contiguous=False)
    c1, nrm, c2 = mod.conv1, mod.norm, mod.conv2
    for prm, nm in ((c1.weight, "conv1.weight"), (c1.bias, "conv1.bias"), (nrm.weight, "norm.weight"),
                    (nrm.bias, "norm.bias"), (c2.weight, "conv2.weight"), (c2.bias, "conv2.bias")):
        _check(prm, nm)
    out = torch.empty((7, B, D, H, W, C), dtype=torch.float32, device=ts[0].device)
    ws = torch.empty(_lib.query("wf_hf_refine_workspace_bytes", B, C), dtype=torch.uint8,
                     device=out.device)
    ptrs = (ctypes.c_void_p * 7)(*[t.data_ptr() for t in ts])
    _lib.call("wf_hf_refine_fwd", ptrs, ts[0].stride(0), c1.weight.data_ptr(), c1.bias.data_ptr(),
              nrm.weight.data_ptr(), nrm.bias.data_ptr(), float(nrm.eps), c2.weight.data_ptr(),
              c2.bias.data_ptr(), int(mod.sigmoid is not None), out.data_ptr(), ws.data_ptr(),
              B, C, D, H, W, _stream())
    return {k: out[i].permute(0, 4, 1, 2, 3) for i, k in enumerate(DETAIL_KEYS)}


def to_cl(x: torch.Tensor) -> torch.Tensor:
    """x itself if it is channel-last already, else a channels_last_3d copy."""
    return x if cl_ld(x) is not None else x.contiguous(memory_format=torch.channels_last_3d)


def _cl_ok(t: torch.Tensor) -> bool:
    return (t.is_cuda and t.dtype == torch.float32 and t.dim() == 5 and t.shape[1] % 4 == 0
            and cl_ld(t) is not None)


def copy_cl(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """dst.copy_(src) for two NCDHW-shaped channel-last tensors of one shape (channel slices of
    wider buffers allowed) on wf_copy_cl; other layouts take torch's copy."""
    if tuple(src.shape) != tuple(dst.shape):
        raise ValueError(f"copy_cl: shapes {tuple(src.shape)} and {tuple(dst.shape)} differ")
    if not (_cl_ok(src) and _cl_ok(dst)) or src.device != dst.device:
        return dst.copy_(src)
    B, C, D, H, W = src.shape
    _lib.call("wf_copy_cl", src.data_ptr(), cl_ld(src), dst.data_ptr(), cl_ld(dst),
              B * D * H * W, C, _stream())
    return dst


def cat_cl(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    """torch.cat(tensors, 1) into a channels_last_3d result (the decoder's layout); inputs in
    any layout (channel-last ones are moved by wf_copy_cl, the rest by torch)."""
    t0 = tensors[0]
    B, _, D, H, W = t0.shape
    out = empty_cl(B, sum(t.shape[1] for t in tensors), D, H, W, t0.device)
    c = 0
    for t in tensors:
        copy_cl(t, out[:, c:c + t.shape[1]])
        c += t.shape[1]
    return out


def subvoxel_scatter_cl(g: torch.Tensor, bias: Optional[torch.Tensor], dst: torch.Tensor):
    """ConvTranspose3d(k = s = 2) placement: g (B*d*h*w, 8*C) GEMM rows (column s*C + c, s = dz*4
    + dy*2 + dx) into channels [0, C) of the channel-last dst (B, >=C, 2d, 2h, 2w), + bias."""
    B, _, D2, H2, W2 = dst.shape
    d, h, w = D2 // 2, H2 // 2, W2 // 2
    C = g.shape[1] // 8
    ldd = cl_ld(dst)
    if ldd is None or not g.is_contiguous() or g.shape[0] != B * d * h * w or C % 4:
        raise ValueError("subvoxel_scatter_cl: g must be contiguous (B*d*h*w, 8C), dst channel-last")
    _lib.call("wf_subvoxel_scatter_cl", g.data_ptr(), 0 if bias is None else bias.data_ptr(),
              dst.data_ptr(), ldd, B, C, d, h, w, _stream())
    return dst


def convtranspose2_cl(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                      out: torch.Tensor) -> torch.Tensor:
    """ConvTranspose3d(k = s = 2) of x (B, Cin, d, h, w) into channels [0, Cout) of the
    channel-last out (B, >= Cout, 2d, 2h, 2w) on the streaming MFMA GEMM with the sub-voxel
    store epilogue (wf_convtranspose2_cl).  bf16x3 operands: the fp32-faithful precision the
    fp32 GEMM it replaces had, under every global precision."""
    B, Cin, d, h, w = x.shape
    if tuple(weight.shape) != (Cin, weight.shape[1], 2, 2, 2):
        raise ValueError(f"convtranspose2_cl: weight {tuple(weight.shape)} does not fit Cin={Cin}")
    Cout = weight.shape[1]
    ldo = cl_ld(out)
    if ldo is None or tuple(out.shape) != (B, out.shape[1], 2 * d, 2 * h, 2 * w) \
            or out.shape[1] < Cout:
        raise ValueError("convtranspose2_cl: out must be a channel-last (B, >=Cout, 2d, 2h, 2w)")
    _check(x, "x", contiguous=False)
    if cl_ld(x) != Cin:
        x = x.contiguous(memory_format=torch.channels_last_3d)
    if bias is not None:
        _check(bias, "bias")

    def make():
        wt = weight.detach().permute(2, 3, 4, 1, 0).reshape(8 * Cout, Cin).contiguous()
        wb = torch.empty((2, 8 * Cout, Cin), dtype=torch.bfloat16, device=wt.device)
        _lib.call("wf_split_f32_to_bf16x2", wt.data_ptr(), wb.data_ptr(), wt.numel(), _stream())
        return wb
    wb = per_forward(("ct2", weight.data_ptr(), tuple(weight.shape)), make)
    _lib.call("wf_convtranspose2_cl", x.data_ptr(), wb.data_ptr(), _ptr(bias), out.data_ptr(),
              ldo, B, Cin, Cout, d, h, w, PRECISIONS["bf16x3"], _stream())
    return out


def cl_parent(t: torch.Tensor, c0: int) -> Optional[torch.Tensor]:
    """The channel-last buffer t is the channel slice [c0, c0 + C) of (t._base[:, c0:c0 + C]),
    or None: lets a producer write a decoder's skip features into its concat buffer."""
    base = t._base
    if base is None or base.dim() != 5 or cl_ld(base) != base.shape[1] or c0 < 0:
        return None
    if tuple(base.shape[2:]) != tuple(t.shape[2:]) or base.shape[0] != t.shape[0]:
        return None
    if c0 + t.shape[1] > base.shape[1] or cl_ld(t) != base.shape[1]:
        return None
    if t.data_ptr() != base.data_ptr() + c0 * base.element_size():
        return None
    return base


def empty_cl(B: int, C: int, D: int, H: int, W: int, device) -> torch.Tensor:
    return torch.empty((B, C, D, H, W), dtype=torch.float32, device=device,
                       memory_format=torch.channels_last_3d)


def conv3d_k3_packed(weight: torch.Tensor, prec: Optional[int] = None) -> torch.Tensor:
    """[2][K-steps][Cout][32] 16-bit planes of a (Cout, Cin, 3, 3, 3) conv weight: bf16 hi /
    lo (wf_conv3d_k3_pack), or fp16 for WF_PREC_FP16 (wf_conv3d_k3_pack_f16); made once per
    weight_scope."""
    f16 = (_prec() if prec is None else prec) == FP16

    def make():
        w = weight.detach()
        _check(w, "conv weight", contiguous=False)
        w = w.contiguous()  # a channels_last_3d model keeps its 5-D weights channel-last
        Cout, Cin = w.shape[:2]
        n = _lib.query("wf_conv3d_k3_packed_elems", Cin, Cout)
        out = torch.empty(n, dtype=torch.bfloat16, device=w.device)
        _lib.call("wf_conv3d_k3_pack_f16" if f16 else "wf_conv3d_k3_pack", w.data_ptr(),
                  out.data_ptr(), Cin, Cout, _stream())
        return out
    return per_forward(("conv3", weight.data_ptr(), tuple(weight.shape), f16), make)


def _conv3_workspace(B, Cin, Cout, D, H, W, prec, xh, device) -> Optional[torch.Tensor]:
    """The split-K partial buffer of a small-grid conv3d_k3 (None when the grid is not split)."""
    n = _lib.query("wf_conv3d_k3_workspace_bytes", B, Cin, Cout, D, H, W, prec, int(xh))
    return torch.empty(n, dtype=torch.uint8, device=device) if n > 0 else None


def conv3d_k3(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None, norm_eps: Optional[float] = None):
    """Conv3d(k=3, stride 1, padding 1) of an NCDHW-shaped fp32 tensor on the MFMA implicit-GEMM
    kernel; the result is channels_last_3d (or written into `out`, a channel-last view).
    With `norm_eps` it returns (out, stats): the InstanceNorm (B, 2, C) {mean, rstd} of the
    output, accumulated in the conv's epilogue.  An fp16 channel-last x (from norm_act_h) runs
    the fp16-input kernel (wf_conv3d_k3_fwd_xh; fp16 precision only)."""
    if x.dtype == torch.float16:
        return _conv3d_k3_xh(x, weight, bias, out, norm_eps)
    _check(x, "x", contiguous=False)
    x = to_cl(x)
    B, Cin, D, H, W = x.shape
    Cout = weight.shape[0]
    if tuple(weight.shape) != (Cout, Cin, 3, 3, 3):
        raise ValueError(f"conv3d_k3: weight {tuple(weight.shape)} does not fit Cin={Cin}")
    if bias is not None:
        _check(bias, "bias")
    if out is None:
        out = empty_cl(B, Cout, D, H, W, x.device)
    ldo = cl_ld(out)
    if ldo is None or tuple(out.shape) != (B, Cout, D, H, W):
        raise ValueError("conv3d_k3: out must be a channel-last (B, Cout, D, H, W) tensor")
    acc = None
    if norm_eps is not None:
        acc = torch.zeros((B, Cout, 2), dtype=torch.float64, device=x.device)
    prec = _prec()
    work = _conv3_workspace(B, Cin, Cout, D, H, W, prec, False, x.device)
    _lib.call("wf_conv3d_k3_fwd", x.data_ptr(), cl_ld(x), conv3d_k3_packed(weight, prec).data_ptr(),
              _ptr(bias), out.data_ptr(), ldo, _ptr(acc), _ptr(work), B, Cin, Cout, D, H, W, prec,
              _stream())
    if acc is None:
        return out
    stats = torch.empty((B, 2, Cout), dtype=torch.float32, device=x.device)
    _lib.call("wf_instnorm_finalize", acc.data_ptr(), stats.data_ptr(), B, Cout, D * H * W,
              float(norm_eps), _stream())
    return out, stats


def _conv3d_k3_xh(x, weight, bias, out, norm_eps):
    if _prec() != FP16:
        raise ValueError("conv3d_k3: an fp16 input needs the fp16 precision")
    ld = cl_ld(x)
    if ld is None or not x.is_cuda:
        raise ValueError("conv3d_k3: fp16 input must be a channel-last CUDA tensor")
    B, Cin, D, H, W = x.shape
    Cout = weight.shape[0]
    if tuple(weight.shape) != (Cout, Cin, 3, 3, 3):
        raise ValueError(f"conv3d_k3: weight {tuple(weight.shape)} does not fit Cin={Cin}")
    if bias is not None:
        _check(bias, "bias")
    if out is None:
        out = empty_cl(B, Cout, D, H, W, x.device)
    ldo = cl_ld(out)
    if ldo is None or tuple(out.shape) != (B, Cout, D, H, W):
        raise ValueError("conv3d_k3: out must be a channel-last (B, Cout, D, H, W) tensor")
    acc = None
    if norm_eps is not None:
        acc = torch.zeros((B, Cout, 2), dtype=torch.float64, device=x.device)
    work = _conv3_workspace(B, Cin, Cout, D, H, W, FP16, True, x.device)
    _lib.call("wf_conv3d_k3_fwd_xh", x.data_ptr(), ld, conv3d_k3_packed(weight, FP16).data_ptr(),
              _ptr(bias), out.data_ptr(), ldo, _ptr(acc), _ptr(work), B, Cin, Cout, D, H, W,
              _stream())
    if acc is None:
        return out
    stats = torch.empty((B, 2, Cout), dtype=torch.float32, device=x.device)
    _lib.call("wf_instnorm_finalize", acc.data_ptr(), stats.data_ptr(), B, Cout, D * H * W,
              float(norm_eps), _stream())
    return out, stats


def norm_act_h(a: torch.Tensor, stats_a: torch.Tensor, slope: float = 0.01) -> torch.Tensor:
    """act((a - mean) * rstd) as a dense channel-last fp16 tensor (wf_norm_act_h_cl): the input
    of an fp16 conv3d_k3, rounded exactly as that conv would round the fp32 values."""
    lda = cl_ld(a)
    if lda is None:
        raise ValueError("norm_act_h: channel-last input expected")
    B, C, D, H, W = a.shape
    out = torch.empty((B, C, D, H, W), dtype=torch.float16, device=a.device,
                      memory_format=torch.channels_last_3d)
    _lib.call("wf_norm_act_h_cl", a.data_ptr(), lda, stats_a.data_ptr(), out.data_ptr(), C, B, C,
              D * H * W, float(slope), _stream())
    return out


def conv1x1_cl(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None
               ) -> torch.Tensor:
    """1x1x1 Conv3d of a channel-last tensor as one GEMM over its position rows: the streaming
    MFMA GEMM at bf16x3 (fp32-faithful, under every global precision) when Cin % 8 == 0 and
    Cout % 4 == 0, else torch's fp32 GEMM."""
    x = to_cl(x)
    B, Cin, D, H, W = x.shape
    Cout = weight.shape[0]
    if Cin % 8 == 0 and Cout % 4 == 0 and cl_ld(x) == Cin and x.is_cuda:
        rows = x.permute(0, 2, 3, 4, 1).reshape(-1, Cin)
        y = linear_rows(rows, weight, bias, prec=PRECISIONS["bf16x3"])
        return y.view(B, D, H, W, Cout).permute(0, 4, 1, 2, 3)
    rows = x.permute(0, 2, 3, 4, 1).reshape(-1, Cin)
    w2 = weight.reshape(Cout, Cin)
    y = torch.addmm(bias, rows, w2.t()) if bias is not None else torch.mm(rows, w2.t())
    return y.view(B, D, H, W, Cout).permute(0, 4, 1, 2, 3)


def upsample_cl(x: torch.Tensor, size: Sequence[int], align_corners: bool) -> torch.Tensor:
    """F.interpolate(x, size, mode='trilinear', align_corners) of a channel-last tensor
    (wf_upsample_trilinear_cl); the result is channels_last_3d."""
    x = x if (cl_ld(x) == x.shape[1]) else x.contiguous(memory_format=torch.channels_last_3d)
    B, C, d, h, w = x.shape
    D, H, W = size
    out = empty_cl(B, C, D, H, W, x.device)
    _lib.call("wf_upsample_trilinear_cl", x.data_ptr(), out.data_ptr(), B, C, d, h, w, D, H, W,
              int(bool(align_corners)), _stream())
    return out


def upsample_add_cl(x: torch.Tensor, out: torch.Tensor, align_corners: bool) -> torch.Tensor:
    """out += F.interpolate(x, out.shape[2:], mode='trilinear', align_corners) for channel-last
    x and a dense channel-last out (wf_upsample_trilinear_add_cl)."""
    x = x if (cl_ld(x) == x.shape[1]) else x.contiguous(memory_format=torch.channels_last_3d)
    B, C, d, h, w = x.shape
    if cl_ld(out) != C or tuple(out.shape[:2]) != (B, C):
        raise ValueError("upsample_add_cl: out must be a dense channel-last (B, C, D, H, W)")
    D, H, W = out.shape[2:]
    _lib.call("wf_upsample_trilinear_add_cl", x.data_ptr(), out.data_ptr(), B, C, d, h, w, D, H,
              W, int(bool(align_corners)), _stream())
    return out


def conv1x1_head(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]
                 ) -> torch.Tensor:
    """UnetOutBlock's 1x1x1 conv of a channel-last x (K <= 120 channels) into N <= 16 classes,
    returned NCDHW-contiguous (wf_conv1x1_head_cl, fp32)."""
    ld = cl_ld(x)
    if ld is None:
        raise ValueError("conv1x1_head: channel-last input expected")
    B, K, D, H, W = x.shape
    N = weight.shape[0]
    w2 = weight.detach().reshape(N, K).contiguous()
    if bias is not None:
        _check(bias, "bias")
    out = torch.empty((B, N, D, H, W), dtype=torch.float32, device=x.device)
    _lib.call("wf_conv1x1_head_cl", x.data_ptr(), ld, w2.data_ptr(), _ptr(bias), out.data_ptr(),
              B, K, N, D * H * W, _stream())
    return out


def dwconv3d_cl(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                norm_eps: Optional[float] = None):
    """Depthwise Conv3d(C, C, 3, padding=1, groups=C) of a dense channel-last tensor.  With
    `norm_eps` (bias given, C % 32 == 0) it returns (out, stats): the (B, 2, C) {mean, rstd} of
    the output per (sample, channel), accumulated in the conv's epilogue
    (wf_dwconv3d_stats_cl) -- GroupNorm(C, C) / InstanceNorm statistics without a re-read."""
    x = x if (cl_ld(x) == x.shape[1]) else x.contiguous(memory_format=torch.channels_last_3d)
    B, C, D, H, W = x.shape
    if tuple(weight.shape) != (C, 1, 3, 3, 3):
        raise ValueError(f"dwconv3d_cl: weight {tuple(weight.shape)} is not ({C},1,3,3,3)")
    _check(weight, "weight")
    if bias is not None:
        _check(bias, "bias")
    out = empty_cl(B, C, D, H, W, x.device)
    if norm_eps is not None:
        if bias is None or C % 32:
            raise ValueError("dwconv3d_cl: fused statistics need a bias and C % 32 == 0")
        acc = torch.empty((B, C, 2), dtype=torch.float64, device=x.device)
        _lib.call("wf_dwconv3d_stats_cl", x.data_ptr(), weight.data_ptr(), bias.data_ptr(),
                  out.data_ptr(), acc.data_ptr(), B, C, D, H, W, _stream())
        stats = torch.empty((B, 2, C), dtype=torch.float32, device=x.device)
        _lib.call("wf_instnorm_finalize", acc.data_ptr(), stats.data_ptr(), B, C, D * H * W,
                  float(norm_eps), _stream())
        return out, stats
    _lib.call("wf_dwconv3d_cl", x.data_ptr(), weight.data_ptr(), _ptr(bias), 0, out.data_ptr(),
              B, C, D, H, W, _stream())
    return out


def upsample_dwconv3d_cl(x: torch.Tensor, size, weight: torch.Tensor, bias: torch.Tensor,
                         norm_eps: float, align_corners: bool = True):
    """dwconv3d_cl(upsample_cl(x, size, align_corners), weight, bias, norm_eps) in one kernel
    (wf_upsample_dwconv3d_stats_cl): the up-sampled tensor is never stored.  Returns (out,
    stats) as dwconv3d_cl, or None where the fused kernel does not apply (C % 32, an x or y
    up-sampling factor below 2) -- the caller then takes the two-kernel path."""
    x = x if (cl_ld(x) == x.shape[1]) else x.contiguous(memory_format=torch.channels_last_3d)
    B, C, d, h, w = x.shape
    D, H, W = (int(v) for v in size)
    if C % 32 or W < 2 * w or H < 2 * h or bias is None:  # the kernel's staging spans
        return None
    if tuple(weight.shape) != (C, 1, 3, 3, 3):
        raise ValueError(f"upsample_dwconv3d_cl: weight {tuple(weight.shape)} is not ({C},1,3,3,3)")
    _check(weight, "weight")
    _check(bias, "bias")
    out = empty_cl(B, C, D, H, W, x.device)
    acc = torch.empty((B, C, 2), dtype=torch.float64, device=x.device)
    _lib.call("wf_upsample_dwconv3d_stats_cl", x.data_ptr(), weight.data_ptr(), bias.data_ptr(),
              out.data_ptr(), acc.data_ptr(), B, C, d, h, w, D, H, W, int(bool(align_corners)),
              _stream())
    stats = torch.empty((B, 2, C), dtype=torch.float32, device=x.device)
    _lib.call("wf_instnorm_finalize", acc.data_ptr(), stats.data_ptr(), B, C, D * H * W,
              float(norm_eps), _stream())
    return out, stats


def conv3d_k3_wgrad(x: torch.Tensor, dy: torch.Tensor, wshape) -> torch.Tensor:
    """dW of conv3d_k3 (wf_conv3d_k3_wgrad): x (B, Cin, D, H, W), dy (B, Cout, D, H, W), both
    channel-last (copied to it otherwise) -> (Cout, Cin, 3, 3, 3) fp32."""
    x, dy = to_cl(x), to_cl(dy)
    _check(x, "x", contiguous=False)
    _check(dy, "dy", contiguous=False)
    B, Cin, D, H, W = x.shape
    Cout = dy.shape[1]
    if tuple(wshape) != (Cout, Cin, 3, 3, 3) or tuple(dy.shape) != (B, Cout, D, H, W):
        raise ValueError(f"conv3d_k3_wgrad: x {tuple(x.shape)}, dy {tuple(dy.shape)}, weight "
                         f"{tuple(wshape)} do not match")
    dw = torch.empty(tuple(wshape), dtype=torch.float32, device=x.device)
    ws = torch.empty(_lib.query("wf_conv3d_k3_wgrad_workspace_bytes", B, Cin, Cout, D, H, W),
                     dtype=torch.uint8, device=x.device)
    _lib.call("wf_conv3d_k3_wgrad", x.data_ptr(), cl_ld(x), dy.data_ptr(), cl_ld(dy),
              dw.data_ptr(), 0, ws.data_ptr(), B, Cin, Cout, D, H, W, _stream())
    return dw


def gemm_tn(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None,
            accumulate: bool = False) -> torch.Tensor:
    """a^T b for row matrices a (M, N), b (M, K) (unit column stride, any row stride): the
    weight gradient dW = dY^T X of a Linear over M positions (wf_gemm_tn: bf16x3 MFMAs,
    deterministic split over M).  Returns (N, K) fp32, or adds into / writes `out`."""
    if a.dim() != 2 or b.dim() != 2 or a.shape[0] != b.shape[0]:
        raise ValueError(f"gemm_tn: a {tuple(a.shape)} and b {tuple(b.shape)} do not match")
    a = a if a.stride(1) == 1 and a.dtype == torch.float32 else a.float().contiguous()
    b = b if b.stride(1) == 1 and b.dtype == torch.float32 else b.float().contiguous()
    M, N = a.shape
    K = b.shape[1]
    # rows must not overlap (an expanded stride-0 or short-stride view is copied, not clamped)
    if a.stride(0) < N:
        a = a.contiguous()
    if b.stride(0) < K:
        b = b.contiguous()
    _check(a, "a", contiguous=False)
    _check(b, "b", contiguous=False)
    if b.device != a.device:
        raise ValueError("gemm_tn: a and b must be on the same device")
    if out is None:
        out = torch.empty((N, K), dtype=torch.float32, device=a.device)
        accumulate = False
    # the kernel writes fp32 through out's pointer: a bf16 / fp16 or other-device `out` would be
    # overrun or misread
    if out.dtype != torch.float32 or out.device != a.device:
        raise ValueError(f"gemm_tn: out must be float32 on {a.device}, got {out.dtype} on "
                         f"{out.device}")
    if tuple(out.shape) != (N, K) or out.stride(1) != 1 or out.stride(0) < K:
        raise ValueError("gemm_tn: out must be an (N, K) row matrix")
    ws = torch.empty(max(1, _lib.query("wf_gemm_tn_workspace_bytes", M, N, K)),
                     dtype=torch.uint8, device=a.device)
    _lib.call("wf_gemm_tn", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0),
              out.data_ptr(), out.stride(0), int(accumulate), ws.data_ptr(), M, N, K, _stream())
    return out


def linear_rows(x2d: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
                gelu_in: bool = False, cache: bool = True, prec: Optional[int] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bias + act(x2d) . W^T on the MFMA GEMM family (wf_linear_fwd), act = GELU(erf) when
    gelu_in.  weight (N, K) or (N, K, 1, 1, 1); `cache=False` for per-call weights (no split
    cache on the tensor); `prec` a WF_PREC_* id overriding the global precision; `out` a
    contiguous (M, N) destination (e.g. one sample's row slice of a batch buffer)."""
    _check(x2d, "x")
    M, K = x2d.shape
    N = weight.shape[0]
    w2 = weight.reshape(N, K)
    pr = _prec() if prec is None else prec
    if cache:
        wb = split_weight(weight, (N, K), pr)
    else:
        w2 = w2.contiguous()
        wb = torch.empty((2, N, K), dtype=torch.bfloat16, device=x2d.device)
        _lib.call("wf_cast_f32_to_f16x2" if pr == FP16 else "wf_split_f32_to_bf16x2",
                  w2.data_ptr(), wb.data_ptr(), w2.numel(), _stream())
    if bias is not None:
        _check(bias, "bias")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=x2d.device)
    elif tuple(out.shape) != (M, N) or not out.is_contiguous() or out.dtype != torch.float32:
        raise ValueError(f"linear_rows: out must be a contiguous fp32 ({M}, {N}) tensor")
    _lib.call("wf_linear_fwd", x2d.data_ptr(), wb.data_ptr(), _ptr(bias), out.data_ptr(), M, K, N,
              int(bool(gelu_in)), pr, _stream())
    return out


_GEMM_FALLBACK_TRACE = os.environ.get("WF_GEMM_FALLBACK_TRACE") == "1"  # diagnostics


def mfma_gemm_ok(a: torch.Tensor, K: int, N: int) -> bool:
    """True when a (M, K) row matrix times a (K, N) operand can run on the streaming MFMA GEMM
    (wf_linear_fwd: K % 8 == 0, N % 4 == 0, a contiguous fp32 on the GPU)."""
    ok = (a.is_cuda and a.dtype == torch.float32 and a.dim() == 2 and a.is_contiguous()
          and K % 8 == 0 and K >= 8 and N % 4 == 0 and N >= 4)
    if not ok and _GEMM_FALLBACK_TRACE:
        import traceback
        print(f"[wf] GEMM fallback: a {tuple(a.shape)} stride {a.stride()} {a.dtype} "
              f"contiguous={a.is_contiguous()} K={K} N={N}", flush=True)
        traceback.print_stack(limit=6)
    return ok


def smallk_ok(a: torch.Tensor, K: int, N: int) -> bool:
    """True when a (M, K) row matrix times a (K, N) operand takes the small-K kernel
    (wf_linear_smallk_fwd: K < 8, N % 4 == 0)."""
    return (a.is_cuda and a.dtype == torch.float32 and a.dim() == 2 and a.stride(1) == 1
            and 1 <= K <= 7 and N % 4 == 0 and 4 <= N <= 4096)


def linear_smallk(x2d: torch.Tensor, w_nk: torch.Tensor,
                  bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bias + x2d (M, K) . w_nk (N, K)^T for K < 8 (wf_linear_smallk_fwd, exact fp32 FMAs)."""
    M, K = x2d.shape
    N = w_nk.shape[0]
    w = w_nk.detach().reshape(N, K).contiguous()
    if x2d.stride(1) != 1 or x2d.stride(0) < K:  # overlapping / expanded rows: copy, not clamp
        x2d = x2d.contiguous()
    _check(x2d, "x", contiguous=False)
    _check(w, "w")
    if bias is not None:
        bias = bias.detach().contiguous()
        _check(bias, "bias")
    out = torch.empty((M, N), dtype=torch.float32, device=x2d.device)
    _lib.call("wf_linear_smallk_fwd", x2d.data_ptr(), x2d.stride(0), w.data_ptr(),
              _ptr(bias), out.data_ptr(), N, M, K, N, _stream())
    return out


def _rows_dense(a: torch.Tensor) -> torch.Tensor:
    """A channel slice of a wider channel-last tensor (unit column stride, rows further apart
    than K -- e.g. the gradient of one input of a channel concatenation) as dense rows: one
    copy, instead of handing the product to the platform BLAS (the streaming GEMM reads rows K
    apart)."""
    if a.dim() == 2 and a.stride(1) == 1 and not a.is_contiguous():
        return a.contiguous()
    return a


def mm_rows(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a (M, K) @ b (K, N) -- the data-gradient GEMMs of training (dX = dY W) -- on the
    streaming MFMA GEMM at bf16x3 (fp32-faithful operands, fp32 accumulation; b^T is split
    per call), instead of the platform BLAS (hipBLASLt).  K < 8 (the 4-class head's input
    gradient) runs on the small-K kernel; other shapes neither takes (N % 4 nonzero) fall back
    to torch.mm."""
    K, N = b.shape
    if smallk_ok(a, K, N):
        return linear_smallk(a, b.t())
    a = _rows_dense(a)
    if not mfma_gemm_ok(a, K, N):
        return a.mm(b)
    return linear_rows(a, b.detach().t().contiguous(), None, cache=False,
                       prec=PRECISIONS["bf16x3"])


def linear_rows_any(x2d: torch.Tensor, weight: torch.Tensor,
                    bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bias + x2d @ weight^T (weight (N, K)) at bf16x3 on the streaming MFMA GEMM; K < 8 (the
    4-channel stem's 1x1 residual conv) on the small-K kernel; torch's fp32 addmm for shapes
    neither takes."""
    N, K = weight.shape[0], x2d.shape[1]
    w2 = weight.reshape(N, K)
    if smallk_ok(x2d, K, N):
        return linear_smallk(x2d, w2, bias)
    x2d = _rows_dense(x2d)
    if not mfma_gemm_ok(x2d, K, N):
        return torch.addmm(bias, x2d, w2.t()) if bias is not None else x2d.mm(w2.t())
    return linear_rows(x2d, w2.detach().contiguous(), None if bias is None else bias.detach(),
                       cache=False, prec=PRECISIONS["bf16x3"])


def instnorm_stats(x: torch.Tensor, eps: float) -> torch.Tensor:
    """(B, 2, C) {mean, rstd} of InstanceNorm3d(affine=False) over a channel-last tensor."""
    ld = cl_ld(x)
    if ld is None:
        raise ValueError("instnorm_stats: channel-last input expected")
    B, C = x.shape[:2]
    P = x.shape[2] * x.shape[3] * x.shape[4]
    stats = torch.empty((B, 2, C), dtype=torch.float32, device=x.device)
    ws = torch.empty(_lib.query("wf_instnorm_workspace_bytes", B, C), dtype=torch.uint8,
                     device=x.device)
    _lib.call("wf_instnorm_stats_cl", x.data_ptr(), ld, B, C, P, float(eps), stats.data_ptr(),
              ws.data_ptr(), _stream())
    return stats


def norm_act(a: torch.Tensor, stats_a: torch.Tensor, r: Optional[torch.Tensor] = None,
             stats_r: Optional[torch.Tensor] = None, slope: float = 0.01,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """act((a - mean) * rstd + r') on channel-last tensors (UnetResBlock's norm / add / lrelu);
    r' = InstanceNorm(r) with stats_r, r, or nothing.  `out` may be `a` (in place)."""
    lda = cl_ld(a)
    if lda is None:
        raise ValueError("norm_act: channel-last input expected")
    B, C = a.shape[:2]
    P = a.shape[2] * a.shape[3] * a.shape[4]
    ldr = 0
    if r is not None:
        r = to_cl(r)
        if tuple(r.shape) != tuple(a.shape):
            raise ValueError(f"norm_act: residual {tuple(r.shape)} vs {tuple(a.shape)}")
        ldr = cl_ld(r)
    if out is None:
        out = empty_cl(*a.shape, device=a.device)
    ldo = cl_ld(out)
    if ldo is None or tuple(out.shape) != tuple(a.shape):
        raise ValueError("norm_act: out must be channel-last and shaped like a")
    _lib.call("wf_norm_act_cl", a.data_ptr(), lda, stats_a.data_ptr(), _ptr(r), ldr,
              _ptr(stats_r), out.data_ptr(), ldo, B, C, P, float(slope), _stream())
    return out


def norm_act_lin(a: torch.Tensor, stats_a: torch.Tensor, x: torch.Tensor,
                 weight: torch.Tensor, bias: Optional[torch.Tensor], eps: float,
                 slope: float = 0.01, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """norm_act(a, stats_a, r, instnorm_stats(r, eps)) with r = conv1x1(x; weight, bias) for
    x with few channels (Cin <= 7), r never materialised: x's fp64 moments (wf_moments_cl) give
    InstanceNorm(r)'s per-sample mean and variance, folded into per-sample weights that
    wf_norm_act_lin_cl applies on the fly (exact in real arithmetic)."""
    lda = cl_ld(a)
    x = to_cl(x)
    ldx = cl_ld(x)
    if lda is None or ldx is None:
        raise ValueError("norm_act_lin: channel-last inputs expected")
    B, C = a.shape[:2]
    K = x.shape[1]
    if not 1 <= K <= 7 or tuple(x.shape[2:]) != tuple(a.shape[2:]) or x.shape[0] != B:
        raise ValueError(f"norm_act_lin: x {tuple(x.shape)} does not fit a {tuple(a.shape)}")
    P = a.shape[2] * a.shape[3] * a.shape[4]
    acc = torch.empty((B, K + K * K), dtype=torch.float64, device=a.device)
    _lib.call("wf_moments_cl", x.data_ptr(), ldx, B, K, P, acc.data_ptr(), _stream())
    mu = acc[:, :K] / P
    cov = acc[:, K:].view(B, K, K) / P - mu[:, :, None] * mu[:, None, :]
    W = weight.detach().reshape(C, K).double()
    bv = bias.detach().double() if bias is not None else torch.zeros(C, dtype=torch.float64,
                                                                     device=a.device)
    mean_r = mu @ W.t() + bv                                      # (B, C)
    var_r = torch.einsum("ck,bkl,cl->bc", W, cov, W).clamp_min(0)  # biased, as InstanceNorm
    rstd_r = torch.rsqrt(var_r + eps)
    wfold = (W[None] * rstd_r[..., None]).float().contiguous()     # (B, C, K)
    bfold = ((bv[None] - mean_r) * rstd_r).float().contiguous()    # (B, C)
    if out is None:
        out = empty_cl(*a.shape, device=a.device)
    ldo = cl_ld(out)
    if ldo is None or tuple(out.shape) != tuple(a.shape):
        raise ValueError("norm_act_lin: out must be channel-last and shaped like a")
    _lib.call("wf_norm_act_lin_cl", a.data_ptr(), lda, stats_a.data_ptr(), x.data_ptr(), ldx, K,
              wfold.data_ptr(), bfold.data_ptr(), out.data_ptr(), ldo, B, C, P, float(slope),
              _stream())
    return out


# ------------------------------------------------------------------------------------------
# a2/a3: attention
# ------------------------------------------------------------------------------------------
def rel_pos_bias(table: torch.Tensor, index: torch.Tensor) -> torch.Tensor:
    """Dense (heads, N, N) relative-position bias: table[index.view(-1)] (attention.py:94-97)."""
    _check(table, "relative_position_bias_table")
    _check(index, "relative_position_index", dtype=torch.int64)
    T, heads = table.shape
    N = index.shape[0]
    out = torch.empty((heads, N, N), dtype=torch.float32, device=table.device)
    _lib.call("wf_rel_pos_bias", table.data_ptr(), index.data_ptr(), out.data_ptr(), N, heads, T,
              _stream())
    return out


def index_is_formula(index: torch.Tensor, ws: int) -> bool:
    """relative_position_index == the reference's formula for window ws (attention.py:40-56)?
    A host-synchronising check: Attention runs it at init and on load_state_dict, never in a
    forward."""
    r = torch.arange(ws)
    s, h, w = torch.meshgrid(r, r, r, indexing="ij")
    pos = torch.stack([s.reshape(-1), h.reshape(-1), w.reshape(-1)], dim=-1)
    d = pos[:, None, :] - pos[None, :, :] + (ws - 1)
    ref = d[..., 0] * (3 * ws - 1) + d[..., 1] * (2 * ws - 1) + d[..., 2]
    return tuple(index.shape) == tuple(ref.shape) and bool(torch.equal(index.detach().cpu(), ref))


def attention_bias(table: torch.Tensor, index: torch.Tensor, ws: int, heads: int,
                   head_dim: int, formula: bool = False) -> torch.Tensor:
    """What the window-attention kernels read as the bias: the ((2ws-1)^3, heads) table itself
    when the table-bias kernel applies (ws 8, head_dim 16, and the caller vouches that the
    index is the reference's formula), else the dense (heads, N, N) expansion, made once per
    weight_scope."""
    if ws == 8 and head_dim == 16 and formula:
        return table.detach()
    return per_forward(("relbias", table.data_ptr(), index.data_ptr()),
                       lambda: rel_pos_bias(table.detach(), index))


def window_attention(x_cl: torch.Tensor, wqkv: torch.Tensor, bqkv: Optional[torch.Tensor],
                     bias: torch.Tensor, wproj: torch.Tensor, bproj: Optional[torch.Tensor],
                     ws: int, heads: int, scale: float,
                     ln: Optional[Tuple[torch.Tensor, torch.Tensor, float]] = None,
                     prec: Optional[int] = None) -> torch.Tensor:
    """window_partition + Attention.forward + reshape-reverse (Q1) over a channel-last raster.
    Returns (B, D1, H1, W1, C) whose rows are the window-major attention outputs.  `bias` is
    the dense (heads, N, N) bias, or the ((2ws-1)^3, heads) table itself when the index is the
    reference's formula (wf_window_attention_fwd_table, ws 8 / head_dim 16)."""
    _check(x_cl, "x")
    B, D1, H1, W1, C = x_cl.shape
    prec = _prec() if prec is None else prec
    wq = split_weight(wqkv, prec=prec)
    wp = split_weight(wproj, prec=prec)
    if bqkv is not None:
        _check(bqkv, "qkv.bias")
    if bproj is not None:
        _check(bproj, "proj.bias")
    _check(bias, "bias")
    N = ws ** 3
    table = tuple(bias.shape) == ((2 * ws - 1) ** 3, heads)
    if not table and tuple(bias.shape) != (heads, N, N):
        raise ValueError(f"window_attention: bias {tuple(bias.shape)} is neither ({heads},{N},{N}) "
                         f"nor the ({(2 * ws - 1) ** 3},{heads}) table")
    lw = lb = None
    eps = 0.0
    if ln is not None:
        lw, lb, eps = ln
    out = torch.empty_like(x_cl)
    prec = _prec() if prec is None else prec
    wsb = _lib.query("wf_window_attention_workspace_bytes", B, C, D1, H1, W1, prec)
    work = torch.empty(wsb, dtype=torch.uint8, device=x_cl.device)
    _lib.call("wf_window_attention_fwd_table" if table else "wf_window_attention_fwd",
              x_cl.data_ptr(), _ptr(lw), _ptr(lb), float(eps),
              wq.data_ptr(), _ptr(bqkv), bias.data_ptr(), wp.data_ptr(), _ptr(bproj),
              out.data_ptr(), work.data_ptr(), B, C, D1, H1, W1, ws, heads, float(scale),
              prec, _stream())
    return out


# ------------------------------------------------------------------------------------------
# a6: multi-scale fuse
# ------------------------------------------------------------------------------------------
def msfuse(srcs: Sequence[torch.Tensor], shortcut: torch.Tensor, ln_eps: Optional[float],
           branch_scale: Optional[torch.Tensor] = None
           ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """shortcut + sum_s trilinear(src_s) (align_corners=False), channel-last; optional stats."""
    _check(shortcut, "shortcut")
    B, D, H, W, C = shortcut.shape
    if len(srcs) > 4:
        raise ValueError("msfuse: at most 4 sources")
    dhw: List[int] = []
    for s in srcs:
        _check(s, "src")
        if s.shape[0] != B or s.shape[4] != C:
            raise ValueError("msfuse: source batch/channels mismatch")
        dhw.extend(s.shape[1:4])
    out = torch.empty_like(shortcut)
    stats = None
    if ln_eps is not None:
        stats = torch.empty((B * D * H * W, 2), dtype=torch.float32, device=shortcut.device)
    arr = (ctypes.c_void_p * max(1, len(srcs)))(*[s.data_ptr() for s in srcs])
    darr = (ctypes.c_int64 * max(1, len(dhw)))(*dhw)
    if branch_scale is not None:
        _check(branch_scale, "branch_scale")
    _lib.call("wf_msfuse_fwd", arr, darr, len(srcs), shortcut.data_ptr(), _ptr(branch_scale),
              out.data_ptr(),
              _ptr(stats), float(ln_eps or 0.0), B, C, D, H, W, _stream())
    return out, stats


# ------------------------------------------------------------------------------------------
# a7/a8: CCF_FFN (+ norm2 / double residual)
# ------------------------------------------------------------------------------------------
def ccf_ffn(xh: torch.Tensor, stats: Optional[torch.Tensor], norm2: Optional[torch.nn.Module],
            mlp: torch.nn.Module, branch_scale: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Block path (stats given): xh + n2 + ffn(n2), n2 = norm2(xh).  Bare (stats None): xh + ffn(xh)."""
    n2w = n2b = None
    if stats is not None:
        n2w, n2b = norm2.weight, norm2.bias
    return ccf_ffn_raw(xh, stats, n2w, n2b, mlp.pwconv.weight, mlp.pwconv.bias,
                       mlp.norm1.weight, mlp.norm1.bias, float(mlp.norm1.eps),
                       mlp.dwconv.weight, mlp.dwconv.bias, mlp.norm2.weight, mlp.norm2.bias,
                       float(mlp.norm2.eps), mlp.fc.weight, mlp.fc.bias, branch_scale)


def ccf_ffn_raw(xh, stats, n2w, n2b, pww, pwb, l1w, l1b, eps1, dww, dwb, l2w, l2b, eps2, fcw, fcb,
                branch_scale=None, prec: Optional[int] = None) -> torch.Tensor:
    """ccf_ffn on the parameter tensors themselves (the waveformer::ccf_ffn op's kernel)."""
    _check(xh, "x")
    B, D, H, W, C = xh.shape
    hid = pww.shape[0]
    prec = _prec() if prec is None else prec
    pw = split_weight(pww, (hid, C), prec)
    fc = split_weight(fcw, prec=prec)
    out = torch.empty_like(xh)
    wsb = _lib.query("wf_ccf_ffn_workspace_bytes", B, C, hid, D, H, W, prec)
    work = torch.empty(wsb, dtype=torch.uint8, device=xh.device)
    args = (xh.data_ptr(), _ptr(stats), _ptr(n2w), _ptr(n2b),
            pw.data_ptr(), _ptr(pwb), l1w.data_ptr(), l1b.data_ptr(), float(eps1),
            dww.data_ptr(), dwb.data_ptr(), l2w.data_ptr(), l2b.data_ptr(), float(eps2),
            fc.data_ptr(), _ptr(fcb), _ptr(branch_scale),
            out.data_ptr(), work.data_ptr(), B, C, hid, D, H, W, prec, _stream())
    # the three launches are issued separately so they can be timed one by one (bench.py)
    ccf_ffn_pwconv(args)
    ccf_ffn_dwconv(args, B * D * H * W, hid)
    ccf_ffn_fc(args)
    return out


def ccf_ffn_pwconv(args):
    _lib.call("wf_ccf_ffn_stage", 1, *args)


def ccf_ffn_dwconv(args, positions: int, hidden: int):
    """Depthwise 3^3 conv over the (positions, hidden) h1 of the workspace -> h2 + LN partials
    (positions/hidden are only used by the bench's byte count)."""
    _lib.call("wf_ccf_ffn_stage", 2, *args)


def ccf_ffn_fc(args):
    _lib.call("wf_ccf_ffn_stage", 3, *args)


# ------------------------------------------------------------------------------------------
# a9: PatchMerging
# ------------------------------------------------------------------------------------------
def patch_merging(x_cl: torch.Tensor, norm: torch.nn.LayerNorm, reduction: torch.nn.Linear,
                  v2: bool = False) -> torch.Tensor:
    return _patch_merging_raw(x_cl, norm.weight, norm.bias, float(norm.eps), reduction.weight,
                              v2, _prec())


def _patch_merging_raw(x_cl, ln_w, ln_b, eps, red_w, v2, prec) -> torch.Tensor:
    _check(x_cl, "x")
    B, D, H, W, C = x_cl.shape
    red = split_weight(red_w, prec=prec)
    out = torch.empty((B, D // 2, H // 2, W // 2, 2 * C), dtype=torch.float32, device=x_cl.device)
    _lib.call("wf_patch_merging_fwd", x_cl.data_ptr(), ln_w.data_ptr(), ln_b.data_ptr(),
              float(eps), red.data_ptr(), int(bool(v2)), out.data_ptr(), B, C, D, H, W, prec,
              _stream())
    return out


# ------------------------------------------------------------------------------------------
# config 3: sliding-window inference (importance map + stitch)
# ------------------------------------------------------------------------------------------
BLEND_MODES = {"constant": 0, "gaussian": 1}


def importance_map(roi: Sequence[int], mode: str = "constant",
                   sigma_scale: Sequence[float] = (0.125, 0.125, 0.125),
                   device: Optional[torch.device] = None) -> torch.Tensor:
    """compute_importance_map (monai/data/utils.py:1088-1138) for a 3-D window, on the GPU."""
    if mode not in BLEND_MODES:
        raise ValueError(f"Unsupported mode: {mode}, available options are {sorted(BLEND_MODES)}.")
    rd, rh, rw = (int(v) for v in roi)
    device = torch.device(device) if device is not None else torch.device(
        "cuda", torch.cuda.current_device())
    if device.type != "cuda":
        raise RuntimeError("importance_map: GPU only")
    out = torch.empty((rd, rh, rw), dtype=torch.float32, device=device)
    sig = (ctypes.c_float * 3)(*[float(s) for s in sigma_scale])
    _lib.call("wf_importance_map", BLEND_MODES[mode], sig, out.data_ptr(), rd, rh, rw, _stream())
    return out


def sliding_window_stitch(patches: torch.Tensor, weight_map: torch.Tensor,
                          starts: Sequence[Sequence[int]], image_size: Sequence[int],
                          batch: int, world: int = 1, slots_per_round: int = 1) -> torch.Tensor:
    """sum_w pred_w * map / sum_w map over the windows covering each voxel (the accumulation of
    monai/inferers/utils.py:216-299) -> (batch, C, *image_size).  `patches` is
    (rows, C, *roi); see wf_sliding_window_stitch for the row layout of sharded gathers."""
    _check(patches, "patches")
    _check(weight_map, "importance_map")
    rows, C = patches.shape[:2]
    roi = tuple(patches.shape[2:])
    if tuple(weight_map.shape) != roi:
        raise ValueError(f"sliding_window_stitch: map {tuple(weight_map.shape)} != roi {roi}")
    nwin = [len(s) for s in starts]
    total = batch * nwin[0] * nwin[1] * nwin[2]
    slots = -(-total // world)
    slots = -(-slots // slots_per_round) * slots_per_round
    if rows < slots * world:
        raise ValueError(f"sliding_window_stitch: {rows} patch rows < {slots * world} needed")
    D, H, W = (int(v) for v in image_size)
    out = torch.empty((batch, C, D, H, W), dtype=torch.float32, device=patches.device)
    flat = [int(s) for ax in starts for s in ax]
    sarr = (ctypes.c_int64 * len(flat))(*flat)
    narr = (ctypes.c_int64 * 3)(*nwin)
    _lib.call("wf_sliding_window_stitch", patches.data_ptr(), int(world), int(slots_per_round),
              weight_map.data_ptr(), sarr, narr, out.data_ptr(), batch, C, D, H, W, *roi,
              _stream())
    return out


def sliding_window_stitch_partial(patches: torch.Tensor, weight_map: torch.Tensor,
                                  starts: Sequence[Sequence[int]], image_size: Sequence[int],
                                  batch: int, world: int, rank: int) -> torch.Tensor:
    """This rank's share of the stitch for the all-reduce exchange: (batch, C + 1, *image)
    with the weighted sums of the windows g % world == rank (local rows g // world of
    `patches`) and, in channel C, their summed weights (wf_sliding_window_stitch_partial)."""
    _check(patches, "patches")
    _check(weight_map, "importance_map")
    rows, C = patches.shape[:2]
    roi = tuple(patches.shape[2:])
    if tuple(weight_map.shape) != roi:
        raise ValueError(f"sliding_window_stitch_partial: map {tuple(weight_map.shape)} != roi {roi}")
    nwin = [len(s) for s in starts]
    total = batch * nwin[0] * nwin[1] * nwin[2]
    if rows < -(-total // world):
        raise ValueError(f"sliding_window_stitch_partial: {rows} rows < {-(-total // world)}")
    D, H, W = (int(v) for v in image_size)
    out = torch.empty((batch, C + 1, D, H, W), dtype=torch.float32, device=patches.device)
    flat = [int(s) for ax in starts for s in ax]
    _lib.call("wf_sliding_window_stitch_partial", patches.data_ptr(), int(world), int(rank),
              weight_map.data_ptr(), (ctypes.c_int64 * len(flat))(*flat),
              (ctypes.c_int64 * 3)(*nwin), out.data_ptr(), batch, C, D, H, W, *roi, _stream())
    return out


def sliding_window_normalize(num: torch.Tensor) -> torch.Tensor:
    """(B, C + 1, D, H, W) summed partials -> (B, C, D, H, W) = num[:, :C] / num[:, C]."""
    _check(num, "num")
    B, C1, D, H, W = num.shape
    out = torch.empty((B, C1 - 1, D, H, W), dtype=torch.float32, device=num.device)
    _lib.call("wf_sliding_window_normalize", num.data_ptr(), out.data_ptr(), B, C1 - 1, D, H, W,
              _stream())
    return out


def tta_merge(pred: torch.Tensor, passes: Sequence[Sequence[int]]) -> torch.Tensor:
    """(P, C, D, H, W) per-pass predictions on flipped inputs -> (1, C, D, H, W) average of the
    flipped-back passes (light_training/prediction.py:123-155).  passes[p] lists the flipped
    tensor dims (2, 3, 4) of pass p."""
    _check(pred, "pred")
    P, C, D, H, W = pred.shape
    if len(passes) != P:
        raise ValueError(f"tta_merge: {len(passes)} passes for {P} predictions")
    masks = [sum(1 << (d - 2) for d in f) for f in passes]
    out = torch.empty((1, C, D, H, W), dtype=torch.float32, device=pred.device)
    _lib.call("wf_tta_merge", pred.data_ptr(), (ctypes.c_int * P)(*masks), P, out.data_ptr(),
              C, D, H, W, _stream())
    return out


# ------------------------------------------------------------------------------------------
# a10: proj_out
# ------------------------------------------------------------------------------------------
def proj_out(x_cl: torch.Tensor, normalize: bool, eps: float = 1e-5) -> torch.Tensor:
    """(B,D,H,W,C) -> NCDHW (B,C,D,H,W), non-affine LayerNorm over C when normalize."""
    _check(x_cl, "x")
    B, D, H, W, C = x_cl.shape
    out = torch.empty((B, C, D, H, W), dtype=torch.float32, device=x_cl.device)
    _lib.call("wf_proj_out_fwd", x_cl.data_ptr(), out.data_ptr(), int(bool(normalize)),
              float(eps), B, C, D * H * W, _stream())
    return out


def proj_out_cl(x_cl: torch.Tensor, normalize: bool, eps: float = 1e-5) -> torch.Tensor:
    """proj_out's values as an NCDHW-shaped channels_last_3d tensor (the layout the decoder's
    UnetResBlocks read): no NCDHW write and no transpose back.  Bitwise equal to proj_out."""
    _check(x_cl, "x")
    B, D, H, W, C = x_cl.shape
    out = torch.empty_like(x_cl)
    if normalize:
        _lib.call("wf_proj_out_cl_fwd", x_cl.data_ptr(), out.data_ptr(), float(eps),
                  B * D * H * W, C, _stream())
    else:
        out.copy_(x_cl)
    return out.permute(0, 4, 1, 2, 3)
