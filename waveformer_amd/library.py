"""torch.library registration of the hot-path ops (SURVEY 8b "Registration").

The network_models modules call these ops -- `torch.ops.waveformer.*` -- for the §8 rows, so
FX tracing, torch.compile (the ops are opaque graph nodes with fake-tensor shape functions)
and meta-device shape inference see the same drop-in the reference's plain-torch modules give
them (attention.py:83-104, wave_helper.py:349 / :470-512, idwt_upsample.py:160).

  waveformer::dwt3d          ptwt.wavedec3(level=1, 'db1') of a channel-last volume (+ norm1)
  waveformer::idwt3d         ptwt.waverec3(..., 'db1'), 1..4 levels
  waveformer::window_attn    window_partition + Attention.forward + the Q1 reshape-reverse
  waveformer::msfuse         the multi-scale trilinear fuse + shortcut (+ norm2 statistics)
  waveformer::ccf_ffn        norm2 + CCF_FFN + the Q4 double residual
  waveformer::patch_merging  PatchMerging(V2) (Q3 sub-lattices)

Each op's CUDA kernel is the HIP path of waveformer_amd.ops; `register_fake` gives output
shapes from input shapes alone; `register_autograd` wires the HIP backward kernels
(csrc/train.hip) and the fp32 platform-BLAS GEMM gradients.  Ops whose backward needs forward
intermediates (window_attn, ccf_ffn) take a `train` flag and then also return their workspace
(and the attention's log-sum-exp) as extra, non-differentiable outputs; with train=False those
outputs are empty and the backward raises.  Arithmetic precision is an explicit argument
(WF_PREC_*), not the global setting, so a traced graph does not depend on it.
"""
from __future__ import annotations

import ctypes
import os
import weakref
from typing import List, Optional, Sequence, Tuple

import torch
from torch import Tensor

from . import _lib, ops
from .autograd import _f32, _p, _s, _scale_rows, colsum, ln_bwd, ln_fwd

DETAIL_KEYS = ops.DETAIL_KEYS
SPLIT = ops.PRECISIONS["bf16x3"]
_FFN_KEEP = 16  # wf_ccf_ffn_stage flag: staged path, h1 / h2 kept in the workspace


def _empty(x: Tensor, dtype=torch.uint8) -> Tensor:
    return x.new_empty((0,), dtype=dtype)


def _round256(n):
    return (n + 255) // 256 * 256


def attn_workspace_bytes(B, C, D1, H1, W1):
    """wf_window_attention_workspace_bytes(..., WF_PREC_BF16X3) in plain (Sym)int arithmetic
    (fake tensors and dynamic shapes cannot call into the library): qkv + core output, fp32."""
    rows = B * D1 * H1 * W1
    return _round256(rows * 3 * C * 4) + _round256(rows * C * 4)


def ffn_workspace_bytes(B, C, hidden, D, H, W):
    """wf_ccf_ffn_workspace_bytes(..., WF_PREC_BF16X3): h1 and h2 fp32 + the dwconv's
    (mean, M2) per 32 channels of every position + the same-size area of the pwconv's LN1
    partials + their per-row (mean, rstd) (ffn.hip, WF_FFN_LN1_FUSE)."""
    M = B * D * H * W
    return (2 * _round256(M * hidden * 4) + 2 * _round256(M * (hidden // 32) * 2 * 4)
            + _round256(M * 2 * 4))


# ------------------------------------------------------------------------------------------
# a1: Haar analysis (+ norm1)
# ------------------------------------------------------------------------------------------
@torch.library.custom_op("waveformer::dwt3d", mutates_args=(), device_types="cuda")
def dwt3d(x: Tensor, ln_w: Optional[Tensor], ln_b: Optional[Tensor], eps: float) -> Tensor:
    """x (B, D, H, W, C) -> bands (8, B, D/2, H/2, W/2, C): band 0 = LL, 1..7 = DETAIL_KEYS."""
    return ops.dwt3d_haar(x, (ln_w, ln_b, eps) if ln_w is not None else None)


@dwt3d.register_fake
def _(x, ln_w, ln_b, eps):
    B, D, H, W, C = x.shape
    return x.new_empty((8, B, D // 2, H // 2, W // 2, C))


def _dwt3d_setup(ctx, inputs, output):
    x, ln_w, ln_b, eps = inputs
    ctx.save_for_backward(x, ln_w, ln_b)
    ctx.eps = eps


@torch.library.custom_op("waveformer::dwt3d_backward", mutates_args=(), device_types="cuda")
def dwt3d_backward(gbands: Tensor, x: Tensor, ln_w: Optional[Tensor], ln_b: Optional[Tensor],
                   eps: float) -> Tuple[Tensor, Tensor, Tensor]:
    """(dx, d ln_w, d ln_b) of dwt3d: the Haar adjoint (wf_dwt3d_haar_bwd), then the norm1
    LayerNorm backward; the LN gradients are empty without norm1."""
    B, D, H, W, C = x.shape
    g = gbands.contiguous()
    ptrs = [g[k].data_ptr() for k in range(8)]
    strides = []
    for k in range(8):
        strides.extend(g[k].stride())  # (b, d, h, w, c)
    dx = torch.empty_like(x)
    _lib.call("wf_dwt3d_haar_bwd", (ctypes.c_void_p * 8)(*ptrs), (ctypes.c_int64 * 40)(*strides),
              dx.data_ptr(), B, C, D, H, W, _s())
    if ln_w is None:
        return dx, _empty(x, torch.float32), _empty(x, torch.float32)
    dx2, dw, db = ln_bwd(x.view(-1, C), ln_w, ln_b, eps, False, dx.view(-1, C))
    return dx2.view(B, D, H, W, C), dw, db


@dwt3d_backward.register_fake
def _(gbands, x, ln_w, ln_b, eps):
    if ln_w is None:
        return torch.empty_like(x), _empty(x, torch.float32), _empty(x, torch.float32)
    return torch.empty_like(x), torch.empty_like(ln_w), torch.empty_like(ln_b)


def _dwt3d_bwd(ctx, gbands):
    x, ln_w, ln_b = ctx.saved_tensors
    dx, dw, db = torch.ops.waveformer.dwt3d_backward(gbands, x, ln_w, ln_b, ctx.eps)
    return dx, (dw if ln_w is not None else None), (db if ln_w is not None else None), None


dwt3d.register_autograd(_dwt3d_bwd, setup_context=_dwt3d_setup)


# ------------------------------------------------------------------------------------------
# a11: Haar synthesis
# ------------------------------------------------------------------------------------------
@torch.library.custom_op("waveformer::idwt3d", mutates_args=(), device_types="cuda")
def idwt3d(ll: Tensor, details: List[Tensor]) -> Tensor:
    """ptwt.waverec3((ll,) + details, 'db1'): ll (B, C, d, h, w) NCDHW-shaped, details the
    7 tensors of each level (DETAIL_KEYS order), coarse -> fine, flattened level-major."""
    L = len(details) // 7
    dets = [dict(zip(DETAIL_KEYS, details[7 * l:7 * l + 7])) for l in range(L)]
    return ops.idwt3d_haar(ll, dets)


@idwt3d.register_fake
def _(ll, details):
    L = len(details) // 7
    B, C, d, h, w = ll.shape
    s = 2 ** L
    return ll.new_empty((B, C, d * s, h * s, w * s))


def _idwt3d_setup(ctx, inputs, output):
    ll, details = inputs
    ctx.L = len(details) // 7
    ctx.save_for_backward(ll)


@torch.library.custom_op("waveformer::idwt3d_backward", mutates_args=(), device_types="cuda")
def idwt3d_backward(gout: Tensor, ll: Tensor, levels: int) -> List[Tensor]:
    """[d ll] + the 7 detail gradients of each level (coarse -> fine) of idwt3d: the Haar
    analysis of the output gradient (wf_haar_analysis_ncdhw), finest level first."""
    B, C, d, h, w = ll.shape
    L = levels
    cur = _f32(gout)
    per_level: List[List[Tensor]] = [None] * L
    for l in range(L - 1, -1, -1):  # finest level first
        s = 2 ** l
        dl, hl, wl = d * s, h * s, w * s
        lo = torch.empty((B, C, dl, hl, wl), dtype=torch.float32, device=cur.device)
        # 7 separate channel-last tensors (op outputs may not alias), identical strides
        dets = [torch.empty((B, dl, hl, wl, C), dtype=torch.float32,
                            device=cur.device).permute(0, 4, 1, 2, 3) for _ in range(7)]
        parr = (ctypes.c_void_p * 7)(*[t.data_ptr() for t in dets])
        sarr = (ctypes.c_int64 * 5)(*dets[0].stride())
        _lib.call("wf_haar_analysis_ncdhw", cur.data_ptr(), cur.stride(0), cur.stride(1),
                  lo.data_ptr(), parr, sarr, B, C, dl, hl, wl, _s())
        per_level[l] = dets
        cur = lo
    return [cur] + [t for lv in per_level for t in lv]


@idwt3d_backward.register_fake
def _(gout, ll, levels):
    B, C, d, h, w = ll.shape
    out = [ll.new_empty((B, C, d, h, w))]
    for l in range(levels):
        s = 2 ** l
        out += [ll.new_empty((B, d * s, h * s, w * s, C)).permute(0, 4, 1, 2, 3)
                for _ in range(7)]
    return out


def _idwt3d_bwd(ctx, gout):
    (ll,) = ctx.saved_tensors
    g = torch.ops.waveformer.idwt3d_backward(gout, ll, ctx.L)
    return g[0], list(g[1:])


idwt3d.register_autograd(_idwt3d_bwd, setup_context=_idwt3d_setup)


# ------------------------------------------------------------------------------------------
# a2-a5: window attention
# ------------------------------------------------------------------------------------------
@torch.library.custom_op("waveformer::window_attn", mutates_args=(), device_types="cuda")
def window_attn(x: Tensor, ln_w: Optional[Tensor], ln_b: Optional[Tensor], eps: float,
                wqkv: Tensor, bqkv: Optional[Tensor], table: Tensor, index: Tensor,
                wproj: Tensor, bproj: Optional[Tensor], ws: int, heads: int, scale: float,
                prec: int, train: bool, index_formula: bool = False
                ) -> Tuple[Tensor, Tensor, Tensor]:
    """Attention over the ws^3 windows of a channel-last raster x (B, D1, H1, W1, C) ->
    (out (B, D1, H1, W1, C), workspace, lse); workspace / lse are empty unless train.
    index_formula: the caller vouches that `index` equals the reference's formula
    (attention.py:40-56) -- Attention checks it at init and on load_state_dict -- so the
    table-bias kernel may evaluate the formula itself instead of reading `index`."""
    C = x.shape[-1]
    ln = (ln_w, ln_b, eps) if ln_w is not None else None
    if not train:
        bias = ops.attention_bias(table, index, ws, heads, C // heads, index_formula)
        out = ops.window_attention(x, wqkv, bqkv, bias, wproj, bproj, ws, heads, scale, ln,
                                   prec=prec)
        return out, _empty(x), _empty(x, torch.float32)
    # training: fp32-faithful forward keeping qkv, the core output and the row log-sum-exp
    B, D1, H1, W1, _ = x.shape
    N = ws ** 3
    bias = ops.rel_pos_bias(table.detach(), index)
    wq, wp = ops.split_weight(wqkv, prec=SPLIT), ops.split_weight(wproj, prec=SPLIT)
    out = torch.empty_like(x)
    wsb = _lib.query("wf_window_attention_workspace_bytes", B, C, D1, H1, W1, SPLIT)
    work = torch.empty(wsb, dtype=torch.uint8, device=x.device)
    lse = torch.empty(B * D1 * H1 * W1 * heads, dtype=torch.float32, device=x.device)
    _lib.call("wf_window_attention_fwd_train", x.data_ptr(), _p(ln_w), _p(ln_b), float(eps),
              wq.data_ptr(), _p(bqkv), bias.data_ptr(), wp.data_ptr(), _p(bproj),
              out.data_ptr(), work.data_ptr(), lse.data_ptr(), B, C, D1, H1, W1, ws, heads,
              float(scale), SPLIT, _s())
    return out, work, lse


@window_attn.register_fake
def _(x, ln_w, ln_b, eps, wqkv, bqkv, table, index, wproj, bproj, ws, heads, scale, prec,
      train, index_formula=False):
    if not train:
        return torch.empty_like(x), _empty(x), _empty(x, torch.float32)
    B, D1, H1, W1, C = x.shape
    wsb = attn_workspace_bytes(B, C, D1, H1, W1)
    return (torch.empty_like(x), x.new_empty((wsb,), dtype=torch.uint8),
            x.new_empty((B * D1 * H1 * W1 * heads,), dtype=torch.float32))


def _attn_setup(ctx, inputs, output):
    (x, ln_w, ln_b, eps, wqkv, bqkv, table, index, wproj, bproj, ws, heads, scale, prec,
     train, _formula) = inputs
    _, work, lse = output
    ctx.meta = (ws, heads, float(scale), float(eps), bool(train))
    ctx.save_for_backward(x, ln_w, ln_b, wqkv, bqkv, table, index, wproj, bproj, work, lse)
    ctx.set_materialize_grads(False)  # no zero gradients for the workspace / lse outputs


_BLAS_WGRAD = os.environ.get("WF_TRAIN_BLAS_WGRAD") == "1"


def _wgrad(dy: Tensor, x: Tensor) -> Tensor:
    """dW = dy^T x over the position rows: wf_gemm_tn (bf16x3 MFMAs, deterministic split over
    the rows); WF_TRAIN_BLAS_WGRAD=1 keeps the platform BLAS's fp32 GEMM (A/B only)."""
    if _BLAS_WGRAD:
        return dy.t().mm(x)
    return ops.gemm_tn(dy, x)


_INDEX_GROUPS: dict = {}


def _index_groups(index: Tensor, rows: int) -> Tuple[Tensor, Tensor]:
    """The relative-position index (attention.py:40-56) grouped by table row for the
    deterministic bias-table gather (wf_rel_pos_bias_bwd): `perm` = the flat positions in a
    stable sort by row, `offsets` (rows + 1) the group boundaries.  The index is a constant
    buffer: the grouping is kept per (tensor, version) instead of a device sort per backward
    (a weak reference checks that the cached entry is still that tensor)."""
    key = (index.data_ptr(), index._version, tuple(index.shape), rows, str(index.device))
    hit = _INDEX_GROUPS.get(key)
    if hit is not None and hit[0]() is index:
        return hit[1], hit[2]
    flat = index.reshape(-1)
    vals, perm = torch.sort(flat, stable=True)
    offsets = torch.searchsorted(vals, torch.arange(rows + 1, device=index.device,
                                                    dtype=vals.dtype))
    perm, offsets = perm.contiguous(), offsets.to(torch.int64).contiguous()
    if len(_INDEX_GROUPS) >= 64:
        _INDEX_GROUPS.clear()
    _INDEX_GROUPS[key] = (weakref.ref(index), perm, offsets)
    return perm, offsets


@torch.library.custom_op("waveformer::window_attn_backward", mutates_args=(),
                         device_types="cuda")
def window_attn_backward(gout: Tensor, x: Tensor, ln_w: Optional[Tensor],
                         ln_b: Optional[Tensor], wqkv: Tensor, bqkv: Optional[Tensor],
                         table: Tensor, index: Tensor, wproj: Tensor, bproj: Optional[Tensor],
                         work: Tensor, lse: Tensor, eps: float, ws: int, heads: int,
                         scale: float) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor,
                                                Tensor, Tensor]:
    """(dx, d ln_w, d ln_b, d wqkv, d bqkv, d table, d wproj, d bproj) of a train=True
    window_attn: the proj / qkv data gradients on the streaming MFMA GEMM (bf16x3), the weight
    gradients on wf_gemm_tn, the core backward
    with the softmax recomputed from the saved log-sum-exp (wf_window_attention_bwd_core),
    the bias-table scatter (wf_rel_pos_bias_bwd) and the norm1 backward.  Absent inputs get
    empty gradients."""
    if work.numel() == 0:
        raise RuntimeError("waveformer::window_attn: backward of a train=False call")
    B, D1, H1, W1, C = x.shape
    N = ws ** 3
    rows = B * D1 * H1 * W1
    E = lambda: _empty(x, torch.float32)  # noqa: E731  (outputs may not alias)
    bias = ops.rel_pos_bias(table.detach(), index)
    qkv_bytes = (rows * 3 * C * 4 + 255) & ~255
    qkv = work[:rows * 3 * C * 4].view(torch.float32).view(rows, 3 * C)
    o = work[qkv_bytes:qkv_bytes + rows * C * 4].view(torch.float32).view(rows, C)
    g = _f32(gout).view(rows, C)
    # proj: out = o Wp^T + bp (rows in window-major order == the Q1 raster order)
    dwproj = _wgrad(g, o)
    dbproj = colsum(g) if bproj is not None else E()
    do = ops.mm_rows(g, wproj)
    dqkv = torch.empty((rows, 3 * C), dtype=torch.float32, device=x.device)
    dbias = torch.empty((heads, N, N), dtype=torch.float32, device=x.device)
    bws = torch.empty(_lib.query("wf_window_attention_bwd_workspace_bytes", B, C, D1, H1, W1, ws,
                                 heads), dtype=torch.uint8, device=x.device)
    _lib.call("wf_window_attention_bwd_core", qkv.data_ptr(), o.data_ptr(), do.data_ptr(),
              bias.data_ptr(), lse.data_ptr(), dqkv.data_ptr(), dbias.data_ptr(),
              bws.data_ptr(), B, C, D1, H1, W1, ws, heads, float(scale), _s())
    dtable = torch.empty(tuple(table.shape), dtype=torch.float32, device=x.device)
    perm, offsets = _index_groups(index, table.shape[0])
    _lib.call("wf_rel_pos_bias_bwd", dbias.data_ptr(), perm.data_ptr(), offsets.data_ptr(),
              dtable.data_ptr(), N, heads, table.shape[0], _s())
    # qkv = xin Wqkv^T + bqkv with xin = norm1?(x) in raster order (dqkv is raster-ordered)
    x2 = x.view(rows, C)
    xin = ln_fwd(x2, ln_w, ln_b, eps, False) if ln_w is not None else x2
    dwqkv = _wgrad(dqkv, xin)
    dbqkv = colsum(dqkv) if bqkv is not None else E()
    dxin = ops.mm_rows(dqkv, wqkv)
    dlnw, dlnb = E(), E()
    if ln_w is not None:
        dx, dlnw, dlnb = ln_bwd(x2, ln_w, ln_b, eps, False, dxin)
    else:
        dx = dxin
    return dx.view_as(x), dlnw, dlnb, dwqkv, dbqkv, dtable, dwproj, dbproj


@window_attn_backward.register_fake
def _(gout, x, ln_w, ln_b, wqkv, bqkv, table, index, wproj, bproj, work, lse, eps, ws, heads,
      scale):
    like = lambda t: torch.empty_like(t) if t is not None else _empty(x, torch.float32)  # noqa
    return (torch.empty_like(x), like(ln_w), like(ln_b), torch.empty_like(wqkv), like(bqkv),
            torch.empty_like(table), torch.empty_like(wproj), like(bproj))


def _attn_bwd(ctx, gout, _gwork, _glse):
    x, ln_w, ln_b, wqkv, bqkv, table, index, wproj, bproj, work, lse = ctx.saved_tensors
    if gout is None:  # grads are not materialized (see _attn_setup)
        gout = torch.zeros_like(x)
    ws, heads, scale, eps, train = ctx.meta
    if not train:
        raise RuntimeError("waveformer::window_attn: backward of a train=False call")
    dx, dlnw, dlnb, dwqkv, dbqkv, dtable, dwproj, dbproj = \
        torch.ops.waveformer.window_attn_backward(gout, x, ln_w, ln_b, wqkv, bqkv, table, index,
                                                  wproj, bproj, work, lse, eps, ws, heads,
                                                  scale)
    opt = lambda g, t: g if t is not None else None  # noqa: E731
    return (dx, opt(dlnw, ln_w), opt(dlnb, ln_b), None, dwqkv, opt(dbqkv, bqkv), dtable, None,
            dwproj, opt(dbproj, bproj), None, None, None, None, None, None)


window_attn.register_autograd(_attn_bwd, setup_context=_attn_setup)


# ------------------------------------------------------------------------------------------
# a6: multi-scale fuse
# ------------------------------------------------------------------------------------------
@torch.library.custom_op("waveformer::msfuse", mutates_args=(), device_types="cuda")
def msfuse(srcs: List[Tensor], shortcut: Tensor, branch_scale: Optional[Tensor], ln_eps: float,
           want_stats: bool) -> Tuple[Tensor, Tensor]:
    """shortcut + branch_scale * sum_s trilinear(src_s) (align_corners=False), channel-last;
    stats (M, 2) {mean, rstd} of each output row over C for norm2 when want_stats."""
    out, st = ops.msfuse(list(srcs), shortcut, ln_eps if want_stats else None, branch_scale)
    return out, (st if st is not None else _empty(shortcut, torch.float32))


@msfuse.register_fake
def _(srcs, shortcut, branch_scale, ln_eps, want_stats):
    B, D, H, W, C = shortcut.shape
    st = shortcut.new_empty((B * D * H * W, 2)) if want_stats else _empty(shortcut, torch.float32)
    return torch.empty_like(shortcut), st


def _msfuse_setup(ctx, inputs, output):
    srcs, shortcut, branch_scale, ln_eps, want_stats = inputs
    ctx.save_for_backward(branch_scale, *srcs)
    ctx.shortcut_like = (shortcut.shape, shortcut.dtype, shortcut.device)
    ctx.set_materialize_grads(False)  # no zero gradient for the statistics output


@torch.library.custom_op("waveformer::msfuse_backward", mutates_args=(), device_types="cuda")
def msfuse_backward(gxh: Tensor, branch_scale: Optional[Tensor],
                    srcs: List[Tensor]) -> List[Tensor]:
    """The source gradients of msfuse (only the sources' shapes are read): the exact adjoint
    of the trilinear interpolation as three separable gather passes, z / y / x, the DropPath
    factor folded into the first (wf_interp_adjoint_axis)."""
    s_attn = branch_scale
    g = _f32(gxh)
    B, D, H, W, C = g.shape
    dsrcs = []
    for src in srcs:
        sb, sd, sh, sw, sc = src.shape
        if (sd, sh, sw) == (D, H, W):
            dsrcs.append(g.clone() if s_attn is None else _scale_rows(g, s_attn))
            continue
        t1 = torch.empty((B, sd, H, W, C), dtype=torch.float32, device=g.device)
        _lib.call("wf_interp_adjoint_axis", g.data_ptr(), t1.data_ptr(), B, D, sd, H * W * C,
                  _p(s_attn), 1, _s())
        t2 = torch.empty((B, sd, sh, W, C), dtype=torch.float32, device=g.device)
        _lib.call("wf_interp_adjoint_axis", t1.data_ptr(), t2.data_ptr(), B * sd, H, sh, W * C,
                  None, 0, _s())
        t3 = torch.empty((B, sd, sh, sw, C), dtype=torch.float32, device=g.device)
        _lib.call("wf_interp_adjoint_axis", t2.data_ptr(), t3.data_ptr(), B * sd * sh, W, sw, C,
                  None, 0, _s())
        dsrcs.append(t3)
    return dsrcs


@msfuse_backward.register_fake
def _(gxh, branch_scale, srcs):
    return [torch.empty_like(s) for s in srcs]


def _msfuse_bwd(ctx, gxh, _gstats):
    s_attn, *srcs = ctx.saved_tensors
    if gxh is None:  # grads are not materialized (see _msfuse_setup)
        shape, dtype, device = ctx.shortcut_like
        gxh = torch.zeros(shape, dtype=dtype, device=device)
    return torch.ops.waveformer.msfuse_backward(gxh, s_attn, srcs), gxh, None, None, None


msfuse.register_autograd(_msfuse_bwd, setup_context=_msfuse_setup)


# ------------------------------------------------------------------------------------------
# a7/a8: norm2 + CCF_FFN + the double residual (Q4)
# ------------------------------------------------------------------------------------------
@torch.library.custom_op("waveformer::ccf_ffn", mutates_args=(), device_types="cuda")
def ccf_ffn(xh: Tensor, stats: Optional[Tensor], n2w: Optional[Tensor], n2b: Optional[Tensor],
            pww: Tensor, pwb: Optional[Tensor], l1w: Tensor, l1b: Tensor, dww: Tensor,
            dwb: Tensor, l2w: Tensor, l2b: Tensor, fcw: Tensor, fcb: Optional[Tensor],
            s_mlp: Optional[Tensor], n2eps: float, eps1: float, eps2: float, prec: int,
            train: bool) -> Tuple[Tensor, Tensor]:
    """Block form (stats = norm2's row statistics of xh): xh + s_mlp * (n2 + ffn(n2)),
    n2 = norm2(xh) (wave_helper.py:509, CCF_FFN.forward :260-294).  Bare (stats None):
    xh + ffn(xh).  Returns (out, workspace); the workspace (h1, h2 kept for the backward) is
    empty unless train."""
    if not train:
        out = ops.ccf_ffn_raw(xh, stats, n2w, n2b, pww, pwb, l1w, l1b, eps1, dww, dwb, l2w, l2b,
                              eps2, fcw, fcb, s_mlp, prec=prec)
        return out, _empty(xh)
    B, D, H, W, C = xh.shape
    hid = pww.shape[0]
    pw = ops.split_weight(pww, (hid, C), SPLIT)
    fc = ops.split_weight(fcw, prec=SPLIT)
    out = torch.empty_like(xh)
    wsb = _lib.query("wf_ccf_ffn_workspace_bytes", B, C, hid, D, H, W, SPLIT)
    work = torch.empty(wsb, dtype=torch.uint8, device=xh.device)
    # the training path writes h1, h2 and the LN2 partials; the inference-only LN1 areas after
    # them are zeroed so the returned workspace is a deterministic function of the inputs
    M = B * D * H * W
    used = 2 * _round256(M * hid * 4) + _round256(M * (hid // 32) * 2 * 4)
    work[used:].zero_()
    _lib.call("wf_ccf_ffn_stage", _FFN_KEEP, xh.data_ptr(), _p(stats), _p(n2w), _p(n2b),
              pw.data_ptr(), _p(pwb), l1w.data_ptr(), l1b.data_ptr(), float(eps1),
              dww.data_ptr(), dwb.data_ptr(), l2w.data_ptr(), l2b.data_ptr(), float(eps2),
              fc.data_ptr(), _p(fcb), _p(s_mlp), out.data_ptr(), work.data_ptr(), B, C, hid,
              D, H, W, SPLIT, _s())
    return out, work


@ccf_ffn.register_fake
def _(xh, stats, n2w, n2b, pww, pwb, l1w, l1b, dww, dwb, l2w, l2b, fcw, fcb, s_mlp, n2eps, eps1,
      eps2, prec, train):
    if not train:
        return torch.empty_like(xh), _empty(xh)
    B, D, H, W, C = xh.shape
    wsb = ffn_workspace_bytes(B, C, pww.shape[0], D, H, W)
    return torch.empty_like(xh), xh.new_empty((wsb,), dtype=torch.uint8)


def _ffn_setup(ctx, inputs, output):
    (xh, stats, n2w, n2b, pww, pwb, l1w, l1b, dww, dwb, l2w, l2b, fcw, fcb, s_mlp, n2eps, eps1,
     eps2, prec, train) = inputs
    ctx.block = stats is not None
    ctx.meta = (n2eps, eps1, eps2, bool(train))
    # the workspace output never receives a gradient: without this, autograd fills a zero
    # gradient of its full size (hundreds of MB per block) before calling the backward
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(xh, n2w, n2b, pww, pwb, l1w, l1b, dww, l2w, l2b, fcw, fcb, s_mlp,
                          output[1])


@torch.library.custom_op("waveformer::ccf_ffn_backward", mutates_args=(), device_types="cuda")
def ccf_ffn_backward(gout: Tensor, xh: Tensor, n2w: Optional[Tensor], n2b: Optional[Tensor],
                     pww: Tensor, pwb: Optional[Tensor], l1w: Tensor, l1b: Tensor, dww: Tensor,
                     l2w: Tensor, l2b: Tensor, fcw: Tensor, fcb: Optional[Tensor],
                     s_mlp: Optional[Tensor], work: Tensor, n2eps: float, eps1: float,
                     eps2: float, block: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor,
                                                        Tensor, Tensor, Tensor, Tensor, Tensor,
                                                        Tensor, Tensor, Tensor]:
    """(dx, d n2w, d n2b, d pww, d pwb, d l1w, d l1b, d dww, d dwb, d l2w, d l2b, d fcw, d fcb)
    of a train=True ccf_ffn from the kept h1 / h2: LN / GELU backward (wf_ln_act_bwd), the
    depthwise data / weight gradients (wf_dwconv3d_cl flipped, wf_dwconv3d_wgrad), the GEMM
    gradients on the library's MFMA GEMMs (data: streaming GEMM, weights: wf_gemm_tn; bf16x3);
    absent inputs get empty gradients."""
    if work.numel() == 0:
        raise RuntimeError("waveformer::ccf_ffn: backward of a train=False call")
    B, D, H, W, C = xh.shape
    hid = pww.shape[0]
    M = B * D * H * W
    E = lambda: _empty(xh, torch.float32)  # noqa: E731  (outputs may not alias)
    one = (M * hid * 4 + 255) & ~255
    u1 = work[:M * hid * 4].view(torch.float32).view(M, hid)           # GELU(LN1(pw))
    h2 = work[one:one + M * hid * 4].view(torch.float32).view(M, hid)  # dwconv + bias
    g = _f32(gout).view(M, C)
    x2 = xh.view(M, C)
    df = _scale_rows(g.view(B, -1), s_mlp).view(M, C) if block else g
    # fc: f = u2 Wfc^T + bfc, u2 = GELU(LN2(h2))
    u2 = ln_fwd(h2, l2w, l2b, eps2, True)
    dfcw = _wgrad(df, u2)
    dfcb = colsum(df) if fcb is not None else E()
    du2 = ops.mm_rows(df, fcw)
    del u2
    dh2, dl2w, dl2b = ln_bwd(h2, l2w, l2b, eps2, True, du2)
    del du2
    # depthwise conv: h2 = dw(u1) + bdw
    ddwb = colsum(dh2)
    part = torch.empty(_lib.query("wf_dwconv_wgrad_ws_floats", B, hid, D, H, W),
                       dtype=torch.float32,
                       device=xh.device)
    ddww = torch.empty(hid * 27, dtype=torch.float32, device=xh.device)
    _lib.call("wf_dwconv3d_wgrad", dh2.data_ptr(), u1.data_ptr(), part.data_ptr(),
              ddww.data_ptr(), B, hid, D, H, W, _s())
    du1 = torch.empty_like(dh2)
    dw2 = _f32(dww.detach()).view(hid, 27)
    _lib.call("wf_dwconv3d_cl", dh2.data_ptr(), dw2.data_ptr(), None, 1, du1.data_ptr(), B, hid,
              D, H, W, _s())
    del dh2
    # pw: h1 = n2 Wpw^T + bpw, u1 = GELU(LN1(h1))
    n2 = ln_fwd(x2, n2w, n2b, n2eps, False) if block else x2
    wpw = pww.view(hid, C)
    h1 = ops.linear_rows_any(n2, wpw, pwb)
    dh1, dl1w, dl1b = ln_bwd(h1, l1w, l1b, eps1, True, du1)
    del h1, du1
    dpww = _wgrad(dh1, n2).view_as(pww)
    dpwb = colsum(dh1) if pwb is not None else E()
    dn2 = ops.mm_rows(dh1, wpw)
    dn2w, dn2b = E(), E()
    if block:
        dn2 += df
        dx, dn2w, dn2b = ln_bwd(x2, n2w, n2b, n2eps, False, dn2, dadd=g)
    else:
        dx = dn2 + g
    return (dx.view_as(xh), dn2w, dn2b, dpww, dpwb, dl1w, dl1b, ddww.view_as(dww), ddwb, dl2w,
            dl2b, dfcw, dfcb)


@ccf_ffn_backward.register_fake
def _(gout, xh, n2w, n2b, pww, pwb, l1w, l1b, dww, l2w, l2b, fcw, fcb, s_mlp, work, n2eps, eps1,
      eps2, block):
    E = lambda: _empty(xh, torch.float32)  # noqa: E731
    like = lambda t: torch.empty_like(t) if t is not None else E()  # noqa: E731
    return (torch.empty_like(xh), like(n2w) if block else E(), like(n2b) if block else E(),
            torch.empty_like(pww), like(pwb), torch.empty_like(l1w), torch.empty_like(l1b),
            torch.empty_like(dww), xh.new_empty((pww.shape[0],)), torch.empty_like(l2w),
            torch.empty_like(l2b), torch.empty_like(fcw), like(fcb))


def _ffn_bwd(ctx, gout, _gwork):
    xh, n2w, n2b, pww, pwb, l1w, l1b, dww, l2w, l2b, fcw, fcb, s_mlp, work = ctx.saved_tensors
    if gout is None:  # grads are not materialized (see _ffn_setup)
        gout = torch.zeros_like(xh)
    n2eps, eps1, eps2, train = ctx.meta
    if not train:
        raise RuntimeError("waveformer::ccf_ffn: backward of a train=False call")
    (dx, dn2w, dn2b, dpww, dpwb, dl1w, dl1b, ddww, ddwb, dl2w, dl2b, dfcw, dfcb) = \
        torch.ops.waveformer.ccf_ffn_backward(gout, xh, n2w, n2b, pww, pwb, l1w, l1b, dww, l2w,
                                              l2b, fcw, fcb, s_mlp, work, n2eps, eps1, eps2,
                                              ctx.block)
    opt = lambda g, t: g if t is not None else None  # noqa: E731
    return (dx, None, opt(dn2w, n2w) if ctx.block else None, opt(dn2b, n2b) if ctx.block else None,
            dpww, opt(dpwb, pwb), dl1w, dl1b, ddww, ddwb, dl2w, dl2b, dfcw, opt(dfcb, fcb), None,
            None, None, None, None, None)


ccf_ffn.register_autograd(_ffn_bwd, setup_context=_ffn_setup)


# ------------------------------------------------------------------------------------------
# a9: PatchMerging
# ------------------------------------------------------------------------------------------
@torch.library.custom_op("waveformer::patch_merging", mutates_args=(), device_types="cuda")
def patch_merging(x: Tensor, ln_w: Tensor, ln_b: Tensor, eps: float, red_w: Tensor, v2: bool,
                  prec: int) -> Tensor:
    """PatchMerging(V2).forward (wave_helper.py:147-194) of a channel-last (B, D, H, W, C)."""
    return ops._patch_merging_raw(x, ln_w, ln_b, eps, red_w, v2, prec)


@patch_merging.register_fake
def _(x, ln_w, ln_b, eps, red_w, v2, prec):
    B, D, H, W, C = x.shape
    return x.new_empty((B, D // 2, H // 2, W // 2, 2 * C))


def _merge_setup(ctx, inputs, output):
    x, ln_w, ln_b, eps, red_w, v2, prec = inputs
    ctx.meta = (float(eps), bool(v2))
    ctx.save_for_backward(x, ln_w, ln_b, red_w)


@torch.library.custom_op("waveformer::patch_merging_backward", mutates_args=(),
                         device_types="cuda")
def patch_merging_backward(gout: Tensor, x: Tensor, nw: Tensor, nb: Tensor, red: Tensor,
                           eps: float, v2: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """(dx, d norm.weight, d norm.bias, d reduction.weight) of patch_merging: gather of the 8
    sub-lattices (wf_patch_merging_gather), LayerNorm backward, GEMM gradients, scatter
    back (wf_patch_merging_scatter, the duplicated Q3 lattices accumulate); the GEMMs on
    the library's MFMA kernels (bf16x3)."""
    B, D, H, W, C = x.shape
    M = B * (D // 2) * (H // 2) * (W // 2)
    merged = torch.empty((M, 8 * C), dtype=torch.float32, device=x.device)
    _lib.call("wf_patch_merging_gather", x.data_ptr(), int(v2), merged.data_ptr(), B, C, D, H, W,
              _s())
    z = ln_fwd(merged, nw, nb, eps, False)
    g = _f32(gout).view(M, 2 * C)
    dred = _wgrad(g, z)
    del z
    dz = ops.mm_rows(g, red)
    dm, dnw, dnb = ln_bwd(merged, nw, nb, eps, False, dz)
    dx = torch.empty_like(x)
    _lib.call("wf_patch_merging_scatter", dm.data_ptr(), int(v2), dx.data_ptr(), B, C, D, H, W,
              _s())
    return dx, dnw, dnb, dred


@patch_merging_backward.register_fake
def _(gout, x, nw, nb, red, eps, v2):
    return torch.empty_like(x), torch.empty_like(nw), torch.empty_like(nb), torch.empty_like(red)


def _merge_bwd(ctx, gout):
    x, nw, nb, red = ctx.saved_tensors
    eps, v2 = ctx.meta
    dx, dnw, dnb, dred = torch.ops.waveformer.patch_merging_backward(gout, x, nw, nb, red, eps,
                                                                     v2)
    return dx, dnw, dnb, None, dred, None, None


patch_merging.register_autograd(_merge_bwd, setup_context=_merge_setup)


OPS = {"dwt3d": dwt3d, "idwt3d": idwt3d, "window_attn": window_attn, "msfuse": msfuse,
       "ccf_ffn": ccf_ffn, "patch_merging": patch_merging}
# the backward kernels are ops too, so AOT autograd can trace a backward graph through them
BACKWARD_OPS = {"dwt3d_backward": dwt3d_backward, "idwt3d_backward": idwt3d_backward,
                "window_attn_backward": window_attn_backward, "msfuse_backward": msfuse_backward,
                "ccf_ffn_backward": ccf_ffn_backward,
                "patch_merging_backward": patch_merging_backward}


# CPU: no kernel -- the product path has no CPU or eager-PyTorch fallback; a CPU tensor fails
# loudly with the same message as the ops wrappers (the CPU restatement of the reference is
# test infrastructure, oracle/, never a dispatch target)
def _cpu_kernel(name):
    def fail(*args, **kwargs):
        raise RuntimeError(f"waveformer::{name}: waveformer_amd kernels run on the GPU only "
                           "(got CPU tensors); move the module and inputs to cuda")
    return fail


for _name, _op in {**OPS, **BACKWARD_OPS}.items():
    _op.register_kernel("cpu", _cpu_kernel(_name))
