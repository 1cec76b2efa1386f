"""Training path (config 4): torch.autograd.Functions over the HIP forward and backward kernels.

The reference trains with PyTorch autograd through the same modules (3_train.py:99-135, fp32,
trainer.py:454).  Here each hot-path op is one autograd.Function whose forward is the HIP
forward kernel (saving what its backward needs) and whose backward is the HIP backward kernels
of csrc/train.hip, with the dense GEMM gradients (dX = dY W, dW = dY^T X) on the platform
BLAS (torch.mm -> hipBLASLt, fp32).  The modules in network_models switch to these Functions
when autograd is recording (`needs_grad`); inference keeps the fused kernels.

Training always computes in fp32-faithful mode (bf16x3 forward, fp32 backward): the forward
workspaces the backward consumes are fp32 in that mode.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib
from . import ops

DETAIL_KEYS = ops.DETAIL_KEYS
_SPLIT = ops.PRECISIONS["bf16x3"]


def needs_grad(*tensors) -> bool:
    """True when autograd records an op on any of `tensors` (inputs or parameters)."""
    if not torch.is_grad_enabled():
        return False
    return any(t is not None and isinstance(t, torch.Tensor) and t.requires_grad
               for t in tensors)


def _s() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _f32(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


# ------------------------------------------------------------------------------------------
# primitives
# ------------------------------------------------------------------------------------------
def colsum(x2d: torch.Tensor, row_scale: Optional[torch.Tensor] = None,
           rows_per_scale: int = 0) -> torch.Tensor:
    """sum over rows of an (R, N) fp32 matrix (bias gradients), optionally row-scaled."""
    x2d = _f32(x2d)
    R, N = x2d.shape
    part = torch.empty(max(1, _lib.query("wf_colsum_parts", R)) * N, dtype=torch.float32,
                       device=x2d.device)
    out = torch.empty(N, dtype=torch.float32, device=x2d.device)
    _lib.call("wf_colsum", x2d.data_ptr(), R, N, _p(row_scale), int(rows_per_scale),
              part.data_ptr(), out.data_ptr(), _s())
    return out


def ln_fwd(x2d: torch.Tensor, w: Optional[torch.Tensor], b: Optional[torch.Tensor], eps: float,
           gelu: bool) -> torch.Tensor:
    x2d = _f32(x2d)
    M, N = x2d.shape
    y = torch.empty_like(x2d)
    _lib.call("wf_ln_act_fwd", x2d.data_ptr(), _p(w), _p(b), float(eps), int(gelu),
              y.data_ptr(), M, N, _s())
    return y


def ln_bwd(x2d: torch.Tensor, w: Optional[torch.Tensor], b: Optional[torch.Tensor], eps: float,
           gelu: bool, dy: torch.Tensor, dadd: Optional[torch.Tensor] = None
           ) -> Tuple[torch.Tensor, Optional[torch.Tensor], Optional[torch.Tensor]]:
    """(dx, dw, db) of y = GELU?(LN(x)); dx += dadd when given."""
    x2d, dy = _f32(x2d), _f32(dy)
    if dadd is not None:
        dadd = _f32(dadd)
    M, N = x2d.shape
    dx = torch.empty_like(x2d)
    dw = db = part = None
    if w is not None:
        dw = torch.empty(N, dtype=torch.float32, device=x2d.device)
        db = torch.empty(N, dtype=torch.float32, device=x2d.device)
        part = torch.empty(_lib.query("wf_ln_bwd_workspace_floats", M, N), dtype=torch.float32,
                           device=x2d.device)
    _lib.call("wf_ln_act_bwd", x2d.data_ptr(), _p(w), _p(b), float(eps), int(gelu),
              dy.data_ptr(), _p(dadd), dx.data_ptr(), _p(part), _p(dw), _p(db), M, N, _s())
    return dx, dw, db


def _scale_rows(t: torch.Tensor, s: Optional[torch.Tensor]) -> torch.Tensor:
    """t (B, ...) times the per-sample DropPath factor s (B) (None: t itself)."""
    if s is None:
        return t
    return t * s.view((-1,) + (1,) * (t.dim() - 1))


# ------------------------------------------------------------------------------------------
# a1: Haar analysis (+ norm1)
# ------------------------------------------------------------------------------------------
class DWTHaar(torch.autograd.Function):
    """x (B,D,H,W,C) -> (LL (B,d,h,w,C), 7 detail tensors NCDHW-shaped) with optional LN first
    (wave_helper.py:477 + :484-486 + ptwt.wavedec3 at :350)."""

    @staticmethod
    def forward(ctx, x, ln_w, ln_b, eps):
        ctx.set_materialize_grads(False)
        ln = (ln_w, ln_b, eps) if ln_w is not None else None
        bands = ops.dwt3d_haar(x, ln)
        ctx.save_for_backward(x, ln_w, ln_b)
        ctx.eps = eps
        ll = bands[0]
        dets = tuple(bands[k].permute(0, 4, 1, 2, 3) for k in range(1, 8))
        return (ll,) + dets

    @staticmethod
    def backward(ctx, *grads):
        x, ln_w, ln_b = ctx.saved_tensors
        B, D, H, W, C = x.shape
        ptrs, strides, keep = [], [], []
        for k, g in enumerate(grads):
            if g is None:
                ptrs.append(None)
                strides.extend([0] * 5)
                continue
            keep.append(g)
            st = g.stride()
            ptrs.append(g.data_ptr())
            if k == 0:  # (B, d, h, w, C)
                strides.extend([st[0], st[1], st[2], st[3], st[4]])
            else:       # (B, C, d, h, w)
                strides.extend([st[0], st[2], st[3], st[4], st[1]])
        dx = torch.empty_like(x)
        parr = (ctypes.c_void_p * 8)(*ptrs)
        sarr = (ctypes.c_int64 * 40)(*strides)
        _lib.call("wf_dwt3d_haar_bwd", parr, sarr, dx.data_ptr(), B, C, D, H, W, _s())
        del keep
        dw = db = None
        if ln_w is not None:
            dx2, dw, db = ln_bwd(x.view(-1, C), ln_w, ln_b, ctx.eps, False, dx.view(-1, C))
            dx = dx2.view(B, D, H, W, C)
        return dx, dw, db, None


def dwt3d_haar(x: torch.Tensor, ln=None):
    """Differentiable 1-level Haar analysis: (LL channel-last, {key: detail NCDHW view})."""
    if ln is None:
        outs = DWTHaar.apply(x, None, None, 0.0)
    else:
        outs = DWTHaar.apply(x, ln[0], ln[1], float(ln[2]))
    return outs[0], dict(zip(DETAIL_KEYS, outs[1:]))


# ------------------------------------------------------------------------------------------
# a11: Haar synthesis (decoder)
# ------------------------------------------------------------------------------------------
class IDWTHaar(torch.autograd.Function):
    """ptwt.waverec3((ll,) + details, 'db1') (idwt_upsample.py:160); details coarse -> fine,
    flattened level-major in DETAIL_KEYS order."""

    @staticmethod
    def forward(ctx, ll, *flat):
        ctx.set_materialize_grads(False)
        L = len(flat) // 7
        details = [dict(zip(DETAIL_KEYS, flat[7 * l:7 * l + 7])) for l in range(L)]
        out = ops.idwt3d_haar(ll, details)
        ctx.shape = tuple(ll.shape)
        ctx.L = L
        return out

    @staticmethod
    def backward(ctx, gout):
        B, C, d, h, w = ctx.shape
        L = ctx.L
        if gout is None:
            return (None,) * (1 + 7 * L)
        cur = _f32(gout)
        per_level: List[List[torch.Tensor]] = [None] * L
        for l in range(L - 1, -1, -1):  # finest level first
            s = 2 ** l
            dl, hl, wl = d * s, h * s, w * s
            ll = torch.empty((B, C, dl, hl, wl), dtype=torch.float32, device=cur.device)
            base = torch.empty((7, B, dl, hl, wl, C), dtype=torch.float32, device=cur.device)
            dets = [base[k].permute(0, 4, 1, 2, 3) for k in range(7)]
            st = dets[0].stride()
            parr = (ctypes.c_void_p * 7)(*[t.data_ptr() for t in dets])
            sarr = (ctypes.c_int64 * 5)(*st)
            _lib.call("wf_haar_analysis_ncdhw", cur.data_ptr(), cur.stride(0), cur.stride(1),
                      ll.data_ptr(), parr, sarr, B, C, dl, hl, wl, _s())
            per_level[l] = dets
            cur = ll
        grads = [cur]
        for l in range(L):
            grads.extend(per_level[l])
        return tuple(grads)


def idwt3d_haar(ll: torch.Tensor, details: Sequence[Dict[str, torch.Tensor]]) -> torch.Tensor:
    flat = [dct[k] for dct in details for k in DETAIL_KEYS]
    return IDWTHaar.apply(ll, *flat)


# ------------------------------------------------------------------------------------------
# a2-a5: window attention
# ------------------------------------------------------------------------------------------
class WindowAttention(torch.autograd.Function):
    """window_partition + Attention.forward + the Q1 reshape-reverse over a channel-last raster
    (attention.py:83-104, wave_helper.py:491-499), optional norm1 on the tokens."""

    @staticmethod
    def forward(ctx, x, ln_w, ln_b, wqkv, bqkv, table, wproj, bproj, meta):
        ws, heads, scale, eps, index = meta
        B, D1, H1, W1, C = x.shape
        N = ws ** 3
        bias = ops.rel_pos_bias(table.detach(), index)
        wq = ops.split_weight(wqkv)
        wp = ops.split_weight(wproj)
        rows = B * D1 * H1 * W1
        out = torch.empty_like(x)
        wsb = _lib.query("wf_window_attention_workspace_bytes", B, C, D1, H1, W1, _SPLIT)
        work = torch.empty(wsb, dtype=torch.uint8, device=x.device)
        lse = torch.empty((rows // N) * heads * N, dtype=torch.float32, device=x.device)
        _lib.call("wf_window_attention_fwd_train", x.data_ptr(), _p(ln_w), _p(ln_b),
                  float(eps), wq.data_ptr(), _p(bqkv), bias.data_ptr(), wp.data_ptr(),
                  _p(bproj), out.data_ptr(), work.data_ptr(), lse.data_ptr(), B, C, D1, H1, W1,
                  ws, heads, float(scale), _SPLIT, _s())
        ctx.save_for_backward(x, ln_w, ln_b, wqkv, bqkv, wproj, bproj, bias, work, lse)
        ctx.meta = meta
        ctx.has_table = table.requires_grad
        ctx.table_rows = table.shape[0]
        return out

    @staticmethod
    def backward(ctx, gout):
        x, ln_w, ln_b, wqkv, bqkv, wproj, bproj, bias, work, lse = ctx.saved_tensors
        ws, heads, scale, eps, index = ctx.meta
        B, D1, H1, W1, C = x.shape
        N = ws ** 3
        rows = B * D1 * H1 * W1
        qkv_bytes = (rows * 3 * C * 4 + 255) & ~255
        qkv = work[:rows * 3 * C * 4].view(torch.float32).view(rows, 3 * C)
        o = work[qkv_bytes:qkv_bytes + rows * C * 4].view(torch.float32).view(rows, C)
        g = _f32(gout).view(rows, C)
        # proj: out = o Wp^T + bp (rows in window-major order == the Q1 raster order)
        dwproj = g.t().mm(o)
        dbproj = colsum(g) if bproj is not None else None
        do = g.mm(wproj)
        dqkv = torch.empty((rows, 3 * C), dtype=torch.float32, device=x.device)
        dbias = torch.empty((heads, N, N), dtype=torch.float32, device=x.device)
        _lib.call("wf_window_attention_bwd_core", qkv.data_ptr(), o.data_ptr(), do.data_ptr(),
                  bias.data_ptr(), lse.data_ptr(), dqkv.data_ptr(), dbias.data_ptr(), B, C, D1,
                  H1, W1, ws, heads, float(scale), _s())
        dtable = None
        if ctx.has_table:
            dtable = torch.empty((ctx.table_rows, heads), dtype=torch.float32, device=x.device)
            _lib.call("wf_rel_pos_bias_bwd", dbias.data_ptr(), index.data_ptr(),
                      dtable.data_ptr(), N, heads, ctx.table_rows, _s())
        # qkv = xin Wqkv^T + bqkv with xin = norm1?(x) in raster order (dqkv is raster-ordered)
        x2 = x.view(rows, C)
        xin = ln_fwd(x2, ln_w, ln_b, eps, False) if ln_w is not None else x2
        dwqkv = dqkv.t().mm(xin)
        dbqkv = colsum(dqkv) if bqkv is not None else None
        dxin = dqkv.mm(wqkv)
        dlnw = dlnb = None
        if ln_w is not None:
            dx, dlnw, dlnb = ln_bwd(x2, ln_w, ln_b, eps, False, dxin)
        else:
            dx = dxin
        return (dx.view_as(x), dlnw, dlnb, dwqkv, dbqkv, dtable, dwproj, dbproj, None)


def window_attention(attn, x_cl: torch.Tensor, ln=None) -> torch.Tensor:
    lw, lb, eps = (ln if ln is not None else (None, None, 0.0))
    meta = (attn.window_size, attn.num_heads, float(attn.scale), float(eps),
            attn.relative_position_index)
    return WindowAttention.apply(x_cl, lw, lb, attn.qkv.weight, attn.qkv.bias,
                                 attn.relative_position_bias_table, attn.proj.weight,
                                 attn.proj.bias, meta)


# ------------------------------------------------------------------------------------------
# a6: multi-scale fuse
# ------------------------------------------------------------------------------------------
class MsFuse(torch.autograd.Function):
    """xh = shortcut + s_attn * sum_s trilinear(src_s) (wave_helper.py:500-508); also returns
    norm2's row statistics of xh (non-differentiable, consumed by CCFFFN's forward)."""

    @staticmethod
    def forward(ctx, shortcut, s_attn, ln_eps, *srcs):
        xh, stats = ops.msfuse(list(srcs), shortcut, ln_eps, s_attn)
        ctx.shapes = [tuple(s.shape) for s in srcs]
        ctx.save_for_backward(s_attn)
        if stats is not None:
            ctx.mark_non_differentiable(stats)
        return xh, stats

    @staticmethod
    def backward(ctx, gxh, _gstats):
        (s_attn,) = ctx.saved_tensors
        g = _f32(gxh)
        B, D, H, W, C = g.shape
        dsrcs = []
        for (sb, sd, sh, sw, sc) in ctx.shapes:
            if (sd, sh, sw) == (D, H, W):
                dsrcs.append(g.clone() if s_attn is None else _scale_rows(g, s_attn))
                continue
            # separable adjoint: z, then y, then x (DropPath factor in the first pass)
            t1 = torch.empty((B, sd, H, W, C), dtype=torch.float32, device=g.device)
            _lib.call("wf_interp_adjoint_axis", g.data_ptr(), t1.data_ptr(), B, D, sd,
                      H * W * C, _p(s_attn), 1, _s())
            t2 = torch.empty((B, sd, sh, W, C), dtype=torch.float32, device=g.device)
            _lib.call("wf_interp_adjoint_axis", t1.data_ptr(), t2.data_ptr(), B * sd, H, sh,
                      W * C, None, 0, _s())
            t3 = torch.empty((B, sd, sh, sw, C), dtype=torch.float32, device=g.device)
            _lib.call("wf_interp_adjoint_axis", t2.data_ptr(), t3.data_ptr(), B * sd * sh, W,
                      sw, C, None, 0, _s())
            dsrcs.append(t3)
        return (g, None, None) + tuple(dsrcs)


# ------------------------------------------------------------------------------------------
# a7/a8: CCF_FFN + norm2 + the double residual (Q4)
# ------------------------------------------------------------------------------------------
_FFN_KEEP = 16  # wf_ccf_ffn_stage flag: staged path, h1 / h2 kept in the workspace


class CCFFFN(torch.autograd.Function):
    """Block mode (stats given): out = xh + s * (n2 + ffn(n2)), n2 = norm2(xh)
    (wave_helper.py:509 with CCF_FFN.forward :260-294 returning n2 + ffn).
    Bare mode (stats None): out = xh + ffn(xh)."""

    @staticmethod
    def forward(ctx, xh, stats, n2w, n2b, pww, pwb, l1w, l1b, dww, dwb, l2w, l2b, fcw, fcb,
                s_mlp, meta):
        n2eps, eps1, eps2 = meta
        B, D, H, W, C = xh.shape
        hid = pww.shape[0]
        pw = ops.split_weight(pww, (hid, C))
        fc = ops.split_weight(fcw)
        out = torch.empty_like(xh)
        wsb = _lib.query("wf_ccf_ffn_workspace_bytes", B, C, hid, D, H, W, _SPLIT)
        work = torch.empty(wsb, dtype=torch.uint8, device=xh.device)
        _lib.call("wf_ccf_ffn_stage", _FFN_KEEP, xh.data_ptr(), _p(stats), _p(n2w), _p(n2b),
                  pw.data_ptr(), _p(pwb), l1w.data_ptr(), l1b.data_ptr(), float(eps1),
                  dww.data_ptr(), dwb.data_ptr(), l2w.data_ptr(), l2b.data_ptr(), float(eps2),
                  fc.data_ptr(), _p(fcb), _p(s_mlp), out.data_ptr(), work.data_ptr(), B, C, hid,
                  D, H, W, _SPLIT, _s())
        ctx.block = stats is not None
        ctx.meta = meta
        ctx.save_for_backward(xh, n2w, n2b, pww, pwb, l1w, l1b, dww, l2w, l2b, fcw, fcb, s_mlp,
                              work)
        return out

    @staticmethod
    def backward(ctx, gout):
        xh, n2w, n2b, pww, pwb, l1w, l1b, dww, l2w, l2b, fcw, fcb, s_mlp, work = \
            ctx.saved_tensors
        n2eps, eps1, eps2 = ctx.meta
        B, D, H, W, C = xh.shape
        hid = pww.shape[0]
        M = B * D * H * W
        one = (M * hid * 4 + 255) & ~255
        u1 = work[:M * hid * 4].view(torch.float32).view(M, hid)           # GELU(LN1(pw))
        h2 = work[one:one + M * hid * 4].view(torch.float32).view(M, hid)  # dwconv + bias
        g = _f32(gout).view(M, C)
        x2 = xh.view(M, C)
        df = _scale_rows(g.view(B, -1), s_mlp).view(M, C) if ctx.block else g
        # fc: f = u2 Wfc^T + bfc, u2 = GELU(LN2(h2))
        u2 = ln_fwd(h2, l2w, l2b, eps2, True)
        dfcw = df.t().mm(u2)
        dfcb = colsum(df) if fcb is not None else None
        du2 = df.mm(fcw)
        del u2
        dh2, dl2w, dl2b = ln_bwd(h2, l2w, l2b, eps2, True, du2)
        del du2
        # depthwise conv: h2 = dw(u1) + bdw
        ddwb = colsum(dh2)
        part = torch.empty(_lib.query("wf_dwconv_wgrad_ws_floats", M, hid), dtype=torch.float32,
                           device=xh.device)
        ddww = torch.empty(hid * 27, dtype=torch.float32, device=xh.device)
        _lib.call("wf_dwconv3d_wgrad", dh2.data_ptr(), u1.data_ptr(), part.data_ptr(),
                  ddww.data_ptr(), B, hid, D, H, W, _s())
        du1 = torch.empty_like(dh2)
        dw2 = _f32(dww.detach()).view(hid, 27)
        _lib.call("wf_dwconv3d_cl", dh2.data_ptr(), dw2.data_ptr(), None, 1, du1.data_ptr(), B,
                  hid, D, H, W, _s())
        del dh2
        # pw: h1 = n2 Wpw^T + bpw, u1 = GELU(LN1(h1))
        n2 = ln_fwd(x2, n2w, n2b, n2eps, False) if ctx.block else x2
        wpw = pww.view(hid, C)
        h1 = torch.addmm(pwb, n2, wpw.t()) if pwb is not None else n2.mm(wpw.t())
        dh1, dl1w, dl1b = ln_bwd(h1, l1w, l1b, eps1, True, du1)
        del h1, du1
        dpww = dh1.t().mm(n2).view_as(pww)
        dpwb = colsum(dh1) if pwb is not None else None
        dn2 = dh1.mm(wpw)
        dn2w = dn2b = None
        if ctx.block:
            dn2 += df
            dx, dn2w, dn2b = ln_bwd(x2, n2w, n2b, n2eps, False, dn2, dadd=g)
        else:
            dx = dn2 + g
        return (dx.view_as(xh), None, dn2w, dn2b, dpww, dpwb, dl1w, dl1b,
                ddww.view_as(dww), ddwb, dl2w, dl2b, dfcw, dfcb, None, None)


def ccf_ffn(xh, stats, norm2, mlp, s_mlp=None):
    n2w = n2b = None
    n2eps = 0.0
    if stats is not None:
        n2w, n2b, n2eps = norm2.weight, norm2.bias, float(norm2.eps)
    meta = (n2eps, float(mlp.norm1.eps), float(mlp.norm2.eps))
    return CCFFFN.apply(xh, stats, n2w, n2b, mlp.pwconv.weight, mlp.pwconv.bias,
                        mlp.norm1.weight, mlp.norm1.bias, mlp.dwconv.weight, mlp.dwconv.bias,
                        mlp.norm2.weight, mlp.norm2.bias, mlp.fc.weight, mlp.fc.bias, s_mlp,
                        meta)


# ------------------------------------------------------------------------------------------
# a9: PatchMerging
# ------------------------------------------------------------------------------------------
class PatchMergingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, nw, nb, red, meta):
        eps, v2 = meta
        out = ops._patch_merging_raw(x, nw, nb, eps, red, v2, _SPLIT)
        ctx.save_for_backward(x, nw, nb, red)
        ctx.meta = meta
        return out

    @staticmethod
    def backward(ctx, gout):
        x, nw, nb, red = ctx.saved_tensors
        eps, v2 = ctx.meta
        B, D, H, W, C = x.shape
        M = B * (D // 2) * (H // 2) * (W // 2)
        merged = torch.empty((M, 8 * C), dtype=torch.float32, device=x.device)
        _lib.call("wf_patch_merging_gather", x.data_ptr(), int(v2), merged.data_ptr(), B, C, D,
                  H, W, _s())
        z = ln_fwd(merged, nw, nb, eps, False)
        g = _f32(gout).view(M, 2 * C)
        dred = g.t().mm(z)
        del z
        dz = g.mm(red)
        dm, dnw, dnb = ln_bwd(merged, nw, nb, eps, False, dz)
        dx = torch.empty_like(x)
        _lib.call("wf_patch_merging_scatter", dm.data_ptr(), int(v2), dx.data_ptr(), B, C, D, H,
                  W, _s())
        return dx, dnw, dnb, dred, None


def patch_merging(x, norm, reduction, v2):
    return PatchMergingFn.apply(x, norm.weight, norm.bias, reduction.weight,
                                (float(norm.eps), bool(v2)))


# ------------------------------------------------------------------------------------------
# a10: PatchEmbed and proj_out
# ------------------------------------------------------------------------------------------
class PatchEmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        out = ops.patch_embed(x, w, b)
        ctx.save_for_backward(x, w, b)
        return out

    @staticmethod
    def backward(ctx, gout):
        x, w, b = ctx.saved_tensors
        B, Cin, D2, H2, W2 = x.shape
        D, H, W = D2 // 2, H2 // 2, W2 // 2
        Cout = w.shape[0]
        M = B * D * H * W
        g = _f32(gout).view(M, Cout)
        dx = dw = db = None
        if ctx.needs_input_grad[1]:
            rows = torch.empty((M, Cin * 8), dtype=torch.float32, device=x.device)
            _lib.call("wf_patchify", x.data_ptr(), rows.data_ptr(), 0, B, Cin, D, H, W, _s())
            dw = g.t().mm(rows).view_as(w)
        if b is not None and ctx.needs_input_grad[2]:
            db = colsum(g)
        if ctx.needs_input_grad[0]:
            drows = g.mm(w.reshape(Cout, Cin * 8))
            dx = torch.empty_like(x)
            _lib.call("wf_patchify", dx.data_ptr(), drows.data_ptr(), 1, B, Cin, D, H, W, _s())
        return dx, dw, db


class ProjOutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, normalize, eps):
        out = ops.proj_out(x, normalize, eps)
        ctx.save_for_backward(x)
        ctx.normalize, ctx.eps = normalize, eps
        return out

    @staticmethod
    def backward(ctx, gout):
        (x,) = ctx.saved_tensors
        B, D, H, W, C = x.shape
        S = D * H * W
        g = _f32(gout)
        dcl = torch.empty_like(x)
        _lib.call("wf_transpose_cs", g.data_ptr(), dcl.data_ptr(), B, C, S, _s())
        if ctx.normalize:
            dx, _, _ = ln_bwd(x.view(-1, C), None, None, ctx.eps, False, dcl.view(-1, C))
            dcl = dx.view_as(x)
        return dcl, None, None


# ------------------------------------------------------------------------------------------
# trilinear up-sampling (align_corners=True) of ProjectionUpsample, channel-last
# ------------------------------------------------------------------------------------------
class UpsampleCL(torch.autograd.Function):
    """nn.Upsample(size, 'trilinear', align_corners=True) (wave_helper.py:33-81): forward =
    wf_upsample_trilinear_cl, backward = its exact adjoint as three separable gather passes
    (x, then y, then z; wf_interp_adjoint_axis_ac) -- no atomics, unlike the framework's
    scatter-add backward (measured 13.7 ms per call at 64^3 x 192)."""

    @staticmethod
    def forward(ctx, x, size):
        ctx.src = tuple(x.shape[2:])
        return ops.upsample_cl(x, size, True)

    @staticmethod
    def backward(ctx, g):
        B, C, D, H, W = g.shape
        d, h, w = ctx.src
        g = g.contiguous(memory_format=torch.channels_last_3d)   # (B, D, H, W, C) storage
        t1 = torch.empty((B, D, H, w, C), dtype=torch.float32, device=g.device)
        _lib.call("wf_interp_adjoint_axis_ac", g.data_ptr(), t1.data_ptr(), B * D * H, W, w, C,
                  _s())
        t2 = torch.empty((B, D, h, w, C), dtype=torch.float32, device=g.device)
        _lib.call("wf_interp_adjoint_axis_ac", t1.data_ptr(), t2.data_ptr(), B * D, H, h, w * C,
                  _s())
        t3 = torch.empty((B, d, h, w, C), dtype=torch.float32, device=g.device)
        _lib.call("wf_interp_adjoint_axis_ac", t2.data_ptr(), t3.data_ptr(), B, D, d, h * w * C,
                  _s())
        return t3.permute(0, 4, 1, 2, 3), None


def upsample_cl(x: torch.Tensor, size) -> torch.Tensor:
    return UpsampleCL.apply(x, tuple(size))


# ------------------------------------------------------------------------------------------
# decoder 3x3x3 convolution (MONAI Convolution / UnetResBlock conv1, conv2) for training
# ------------------------------------------------------------------------------------------
class Conv3dK3(torch.autograd.Function):
    """Conv3d(k=3, stride 1, padding 1) on the implicit-GEMM MFMA kernel (bf16x3) with its
    input gradient on the same kernel: dx = conv(dy, W~), W~[ci, co, k] = W[co, ci, 26 - k]
    (flipped taps, swapped channels).  The weight gradient is the framework's conv3d_weight
    (MIOpen), as in the reference's training."""

    @staticmethod
    def forward(ctx, x, w, b):
        xc = ops.to_cl(x)
        ctx.save_for_backward(xc, w)
        ctx.has_bias = b is not None
        with ops.precision("bf16x3"):  # training is fp32-faithful whatever the global mode
            return ops.conv3d_k3(xc, w, b)

    @staticmethod
    def backward(ctx, g):
        xc, w = ctx.saved_tensors
        g = ops.to_cl(g)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if w.shape[1] % 16 == 0 and w.shape[0] % 4 == 0:
                wt = w.detach().flip(2, 3, 4).transpose(0, 1).contiguous()
                with ops.precision("bf16x3"):
                    dx = ops.conv3d_k3(g, wt)
            else:
                dx = torch.nn.grad.conv3d_input(xc.shape, w, g, padding=1)
        if ctx.needs_input_grad[1]:
            dw = torch.nn.grad.conv3d_weight(xc, w.shape, g, padding=1)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = g.sum(dim=(0, 2, 3, 4))
        return dx, dw, db


def conv3d_k3(x, w, b=None):
    return Conv3dK3.apply(x, w, b)
