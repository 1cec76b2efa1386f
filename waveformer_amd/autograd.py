"""Training path (config 4): torch.autograd.Functions over the HIP forward and backward kernels.

The reference trains with PyTorch autograd through the same modules (3_train.py:99-135, fp32,
trainer.py:454).  Here each hot-path op is one autograd.Function whose forward is the HIP
forward kernel (saving what its backward needs) and whose backward is the HIP backward kernels
of csrc/train.hip.  The dense GEMMs of the step run on the library's own MFMA GEMMs at bf16x3
(fp32-faithful operands, fp32 accumulation): the data gradients dX = dY W and the 1x1 /
transposed-conv forwards on the streaming GEMM (ops.mm_rows / linear_rows_any /
convtranspose2_cl), the weight gradients dW = dY^T X on wf_gemm_tn -- no hipBLASLt on the
step, except the shapes those kernels do not take (a channel count not a multiple of 8 / 4:
the 4-channel input and output convolutions), which fall back to torch.mm.  The modules in
network_models switch to these Functions when autograd is recording (`needs_grad`);
inference keeps the fused kernels.

Training always computes in fp32-faithful mode (bf16x3 forward, fp32 backward): the forward
workspaces the backward consumes are fp32 in that mode.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib
from . import ops

DETAIL_KEYS = ops.DETAIL_KEYS
SPLIT = _SPLIT = ops.PRECISIONS["bf16x3"]


def needs_grad(*tensors) -> bool:
    """True when autograd records an op on any of `tensors` (inputs or parameters)."""
    if not torch.is_grad_enabled():
        return False
    return any(t is not None and isinstance(t, torch.Tensor) and t.requires_grad
               for t in tensors)


def prec_for(*tensors) -> int:
    """Operand precision of an op over `tensors`: fp32-faithful bf16x3 whenever autograd
    records it (training), else the global setting (ops.set_precision)."""
    return SPLIT if needs_grad(*tensors) else ops.prec_id()


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
# the hot-path ops (DWT, IDWT, window attention, multi-scale fuse, CCF_FFN, PatchMerging) are
# torch.library custom ops with registered autograd: waveformer_amd/library.py
# ------------------------------------------------------------------------------------------
def idwt3d_haar(ll: torch.Tensor, details: Sequence[Dict[str, torch.Tensor]]) -> torch.Tensor:
    """Differentiable ptwt.waverec3((ll,) + details, 'db1') (waveformer::idwt3d)."""
    from . import library  # noqa: F401
    return torch.ops.waveformer.idwt3d(ll, [dct[k] for dct in details for k in DETAIL_KEYS])


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
            dw = ops.gemm_tn(g, rows).view_as(w)
        if b is not None and ctx.needs_input_grad[2]:
            db = colsum(g)
        if ctx.needs_input_grad[0]:
            drows = ops.mm_rows(g, w.reshape(Cout, Cin * 8))
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
    (flipped taps, swapped channels), and its weight gradient on wf_conv3d_k3_wgrad (implicit
    GEMM over the positions, bf16x3, deterministic) -- no MIOpen find for any shape."""

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
            if w.shape[0] % 16 == 0 and w.shape[1] % 4 == 0:
                dw = ops.conv3d_k3_wgrad(xc, g, w.shape)   # HIP, no MIOpen find
            else:
                dw = torch.nn.grad.conv3d_weight(xc, w.shape, g, padding=1)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = g.sum(dim=(0, 2, 3, 4))
        return dx, dw, db


def conv3d_k3(x, w, b=None):
    return Conv3dK3.apply(x, w, b)


# ------------------------------------------------------------------------------------------
# the decoder's other convolutions in training: depthwise 3^3 on HIP, 1x1 and the 2^3
# transposed conv as channel-last MFMA GEMMs -- no MIOpen convolution anywhere, so a
# training step needs no MIOpen find / kernel compilation (minutes at B = 4 on a fresh box)
# ------------------------------------------------------------------------------------------
class DWConv3dK3(torch.autograd.Function):
    """Depthwise Conv3d(C, C, 3, padding=1, groups=C) channel-last: forward wf_dwconv3d_cl,
    input gradient the same kernel with flipped taps, weight gradient wf_dwconv3d_wgrad."""

    @staticmethod
    def forward(ctx, x, w, b):
        xc = ops.to_cl(x)
        ctx.save_for_backward(xc, w)
        ctx.has_bias = b is not None
        return ops.dwconv3d_cl(xc, w, b)

    @staticmethod
    def backward(ctx, g):
        xc, w = ctx.saved_tensors
        g = ops.to_cl(g)
        B, C, D, H, W = xc.shape
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = ops.empty_cl(B, C, D, H, W, g.device)
            _lib.call("wf_dwconv3d_cl", g.data_ptr(), _f32(w.detach()).data_ptr(), None, 1,
                      dx.data_ptr(), B, C, D, H, W, _s())
        if ctx.needs_input_grad[1]:
            part = torch.empty(_lib.query("wf_dwconv_wgrad_ws_floats", B, C, D, H, W),
                               dtype=torch.float32, device=g.device)
            dw = torch.empty(C * 27, dtype=torch.float32, device=g.device)
            _lib.call("wf_dwconv3d_wgrad", g.data_ptr(), xc.data_ptr(), part.data_ptr(),
                      dw.data_ptr(), B, C, D, H, W, _s())
            dw = dw.view_as(w)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = colsum(g.permute(0, 2, 3, 4, 1).reshape(-1, C))
        return dx, dw, db


def _rows(x: torch.Tensor) -> torch.Tensor:
    """(B, C, D, H, W) -> the (B, D, H, W, C) channel-last view (a copy if x is not)."""
    return ops.to_cl(x).permute(0, 2, 3, 4, 1)


_TORCH_CONV = os.environ.get("WF_TRAIN_TORCH_CONV") == "1"


def conv_train(conv: torch.nn.Module, x: torch.Tensor) -> torch.Tensor:
    """A decoder Conv3d / ConvTranspose3d on the waveformer_amd paths (autograd-aware):
    3^3 dense (Conv3dK3), 3^3 depthwise (DWConv3dK3), 1^3 (F.linear over channel-last rows),
    2^3 stride-2 transposed (one GEMM into the 8 sub-voxels).  Other shapes: the module."""
    F = torch.nn.functional
    nn = torch.nn
    ok = x.is_cuda and x.dtype == torch.float32 and x.dim() == 5
    if _TORCH_CONV and type(conv) is nn.Conv3d and conv.kernel_size == (3, 3, 3):
        # diagnostics only (tools/grad128_diag.py): the 3^3 convs on the framework's fp32
        # convolution, to attribute the gradient error of the bf16x3 kernels
        return conv(x.contiguous())
    if ok and type(conv) is nn.Conv3d and conv.padding_mode == "zeros" \
            and conv.dilation == (1, 1, 1) and conv.stride == (1, 1, 1):
        Cin, Cout = conv.in_channels, conv.out_channels
        if conv.kernel_size == (3, 3, 3) and conv.padding == (1, 1, 1):
            if conv.groups == 1 and Cin % 4 == 0 and Cout % 16 == 0:
                return conv3d_k3(x, conv.weight, conv.bias)
            if conv.groups == Cin == Cout and Cin % 4 == 0:
                return DWConv3dK3.apply(x, conv.weight, conv.bias)
        if conv.kernel_size == (1, 1, 1) and conv.padding == (0, 0, 0) and conv.groups == 1:
            return Conv1x1Fn.apply(x, conv.weight, conv.bias)
    if ok and type(conv) is nn.ConvTranspose3d and conv.kernel_size == (2, 2, 2) \
            and conv.stride == (2, 2, 2) and conv.padding == (0, 0, 0) \
            and conv.output_padding == (0, 0, 0) and conv.groups == 1 \
            and conv.dilation == (1, 1, 1):
        return ConvT2Fn.apply(x, conv.weight, conv.bias)
    return conv(x)


class Conv1x1Fn(torch.autograd.Function):
    """Conv3d(k=1) over channel-last position rows: y = x W^T + b and dx = dy W on the
    streaming MFMA GEMM (bf16x3; torch.mm for channel counts it does not take), dW = dy^T x on
    wf_gemm_tn (the platform BLAS put this long-K shape on a handful of workgroups: 1.8-8 ms per
    call at 128^3), db = column sums (deterministic)."""

    @staticmethod
    def forward(ctx, x, w, b):
        B, Cin, D, H, W = x.shape
        Cout = w.shape[0]
        rows = _rows(x).reshape(-1, Cin)
        y = ops.linear_rows_any(rows, w.view(Cout, Cin), b)
        ctx.save_for_backward(rows, w)
        ctx.has_bias, ctx.shape = b is not None, (B, D, H, W)
        return y.view(B, D, H, W, Cout).permute(0, 4, 1, 2, 3)

    @staticmethod
    def backward(ctx, g):
        rows, w = ctx.saved_tensors
        B, D, H, W = ctx.shape
        Cout, Cin = w.shape[0], w.shape[1]
        gr = _rows(g).reshape(-1, Cout)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = ops.mm_rows(gr, w.view(Cout, Cin)).view(B, D, H, W, Cin).permute(0, 4, 1, 2, 3)
        if ctx.needs_input_grad[1]:
            dw = ops.gemm_tn(gr, rows).view_as(w)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = colsum(gr)
        return dx, dw, db


class LinearFn(torch.autograd.Function):
    """nn.Linear over (M, K) rows (ChannelCalibration's squeeze-excitation fc1 / fc2,
    network_backbone.py:66-128): y = x W^T + b and dx = dy W on the streaming MFMA GEMM
    (bf16x3), dW = dy^T x on wf_gemm_tn, db = column sums -- the step's last platform-BLAS
    GEMMs (M = batch)."""

    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.contiguous()
        ctx.save_for_backward(x2, w)
        ctx.has_bias = b is not None
        return ops.linear_rows_any(x2, w, b)

    @staticmethod
    def backward(ctx, g):
        x2, w = ctx.saved_tensors
        g = _f32(g).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = ops.mm_rows(g, w)
        if ctx.needs_input_grad[1]:
            dw = ops.gemm_tn(g, x2)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = colsum(g)
        return dx, dw, db


def linear(lin: torch.nn.Linear, x: torch.Tensor) -> torch.Tensor:
    """lin(x) for 2-D fp32 GPU rows on the library's GEMMs (autograd-aware); else the module."""
    if x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and type(lin) is torch.nn.Linear:
        if needs_grad(x, lin.weight, lin.bias):
            return LinearFn.apply(x, lin.weight, lin.bias)
        return ops.linear_rows_any(x.contiguous(), lin.weight, lin.bias)
    return lin(x)


class ConvT2Fn(torch.autograd.Function):
    """ConvTranspose3d(k=2, s=2) (unetr_block.py:73-80) as one GEMM into the 8 sub-voxels:
    y[2z+dz, 2y+dy, 2x+dx] = x W[:, :, dz, dy, dx] + b -- the MFMA GEMM whose epilogue stores
    each sub-voxel + bias (wf_convtranspose2_cl, bf16x3).  Backward: the sub-voxel gradient
    rows (M, 8 Cout), dx = rows . Wr^T on the streaming MFMA GEMM, dW = x^T rows on wf_gemm_tn,
    db = column sums.  Channel counts the kernels do not take use torch.mm."""

    @staticmethod
    def forward(ctx, x, w, b):
        B, Cin, d, h, ww = x.shape
        Cout = w.shape[1]
        rows = _rows(x).reshape(-1, Cin)
        ctx.save_for_backward(rows, w)
        ctx.has_bias, ctx.shape = b is not None, (B, d, h, ww)
        if Cin % 8 == 0 and Cout % 4 == 0:
            y = ops.empty_cl(B, Cout, 2 * d, 2 * h, 2 * ww, x.device)
            return ops.convtranspose2_cl(x, w.detach(), None if b is None else b.detach(), y)
        wr = w.permute(0, 2, 3, 4, 1).reshape(Cin, 8 * Cout)
        y = (rows @ wr).view(B, d, h, ww, 2, 2, 2, Cout)
        y = y.permute(0, 1, 4, 2, 5, 3, 6, 7).reshape(B, 2 * d, 2 * h, 2 * ww, Cout)
        if b is not None:
            y = y + b
        return y.permute(0, 4, 1, 2, 3)

    @staticmethod
    def backward(ctx, g):
        rows, w = ctx.saved_tensors
        B, d, h, ww = ctx.shape
        Cin, Cout = w.shape[0], w.shape[1]
        gcl = _rows(g)                                            # (B, 2d, 2h, 2w, Cout)
        gsub = gcl.reshape(B, d, 2, h, 2, ww, 2, Cout).permute(0, 1, 3, 5, 2, 4, 6, 7)
        gsub = gsub.reshape(-1, 8 * Cout)                         # rows (b, z, y, x) x (s, c)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wr = w.permute(0, 2, 3, 4, 1).reshape(Cin, 8 * Cout)
            dx = ops.mm_rows(gsub, wr.t()).view(B, d, h, ww, Cin).permute(0, 4, 1, 2, 3)
        if ctx.needs_input_grad[1]:
            dw = ops.gemm_tn(rows, gsub).view(Cin, 2, 2, 2, Cout).permute(0, 4, 1, 2, 3)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = colsum(gcl.reshape(-1, Cout))
        return dx, dw, db


# ------------------------------------------------------------------------------------------
# InstanceNorm3d(affine=False) + residual + LeakyReLU of UnetResBlock / UnetBasicBlock in
# training: the forward's HIP statistics + fused pass, the backward's two HIP passes
# (wf_norm_act_bwd_cl) -- instead of the framework's layout copies, batch-norm kernels,
# LeakyReLU and add, each a full-resolution pass of its own
# ------------------------------------------------------------------------------------------
class NormActFn(torch.autograd.Function):
    """y = LeakyReLU(slope)(IN_eps(a) + r'), r' = IN_eps_r(r) (mode 2), r (mode 1) or 0."""

    @staticmethod
    def forward(ctx, a, r, slope, eps, eps_r, mode):
        a = ops.to_cl(a)
        sa = ops.instnorm_stats(a, eps)
        sr = None
        if mode == 2:
            r = ops.to_cl(r)
            sr = ops.instnorm_stats(r, eps_r)
        y = ops.norm_act(a, sa, r if mode else None, sr, slope)
        ctx.save_for_backward(a, r if mode == 2 else None, y, sa, sr)
        ctx.slope, ctx.mode = slope, mode
        return y

    @staticmethod
    def backward(ctx, g):
        a, r, y, sa, sr = ctx.saved_tensors
        g = ops.to_cl(g)
        B, C, D, H, W = a.shape
        P = D * H * W
        da = ops.empty_cl(B, C, D, H, W, a.device)
        want_r = ctx.mode and ctx.needs_input_grad[1]
        dr = ops.empty_cl(B, C, D, H, W, a.device) if want_r else None
        ws = torch.empty(_lib.query("wf_norm_act_bwd_workspace_bytes", B, C), dtype=torch.uint8,
                         device=a.device)
        _lib.call("wf_norm_act_bwd_cl", g.data_ptr(), ops.cl_ld(g), y.data_ptr(), ops.cl_ld(y),
                  a.data_ptr(), ops.cl_ld(a), sa.data_ptr(), _p(r), ops.cl_ld(r) if r is not None
                  else 0, _p(sr), da.data_ptr(), C, _p(dr), C if dr is not None else 0, B, C, P,
                  float(ctx.slope), ws.data_ptr(), _s())
        return da, dr, None, None, None, None


class GroupNormCLFn(torch.autograd.Function):
    """GroupNorm(C, C) with affine (ProjectionUpsample.norm, wave_helper.py:65) on a
    channel-last tensor in training: per-(sample, channel) statistics on wf_instnorm_stats_cl
    (fp64 sums), y = x * (rstd gamma) + (beta - mean rstd gamma) in one pass that keeps the
    layout; backward = wf_norm_act_bwd_cl of the non-affine normalisation (slope 1: no
    activation) times gamma, whose per-(sample, channel) sums of dy and dy * xhat are the beta /
    gamma gradients.  The framework's GroupNorm needs NCDHW: a layout copy before and after
    each call and its two backward kernels (~12 ms per config-4 step at B = 4)."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        x = ops.to_cl(x)
        B, C = x.shape[:2]
        st = ops.instnorm_stats(x, eps)                        # (B, 2, C) {mean, rstd}
        scale = st[:, 1] * w                                   # (B, C)
        shift = b - st[:, 0] * scale
        y = ops.empty_cl(*x.shape, x.device)
        torch.addcmul(shift.view(B, C, 1, 1, 1), x, scale.view(B, C, 1, 1, 1), out=y)
        ctx.save_for_backward(x, w, st)
        return y

    @staticmethod
    def backward(ctx, g):
        x, w, st = ctx.saved_tensors
        g = ops.to_cl(g)
        B, C, D, H, W = x.shape
        da = ops.empty_cl(B, C, D, H, W, x.device)
        ws = torch.empty(_lib.query("wf_norm_act_bwd_workspace_bytes", B, C), dtype=torch.uint8,
                         device=x.device)
        _lib.call("wf_norm_act_bwd_cl", g.data_ptr(), ops.cl_ld(g), g.data_ptr(), ops.cl_ld(g),
                  x.data_ptr(), ops.cl_ld(x), st.data_ptr(), None, 0, None, da.data_ptr(), C,
                  None, 0, B, C, D * H * W, 1.0, ws.data_ptr(), _s())
        sums = ws.view(torch.float64).view(B, C, 3).sum(0)     # {sum dy, sum dy*xhat, -}
        da.mul_(w.view(1, C, 1, 1, 1))
        dw = sums[:, 1].float() if ctx.needs_input_grad[1] else None
        db = sums[:, 0].float() if ctx.needs_input_grad[2] else None
        return da, dw, db, None


def group_norm_cl(norm: torch.nn.GroupNorm, x: torch.Tensor) -> torch.Tensor:
    """norm(x) for a per-channel affine GroupNorm on the channel-last path (training)."""
    if (norm.num_groups == norm.num_channels and norm.affine and x.is_cuda
            and x.dtype == torch.float32 and x.dim() == 5 and x.shape[1] % 4 == 0
            and x.shape[1] <= 1024):
        return GroupNormCLFn.apply(x, norm.weight, norm.bias, float(norm.eps))
    return norm(x)


def norm_act(a, r=None, slope=0.01, eps=1e-5, eps_r=1e-5, normed_residual=False):
    mode = 0 if r is None else (2 if normed_residual else 1)
    return NormActFn.apply(a, r, float(slope), float(eps), float(eps_r), mode)
