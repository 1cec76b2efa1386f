"""Decoder building blocks with the module names / state_dict keys of the MONAI blocks the
reference uses (vendored MONAI, monai/networks/blocks/{dynunet_block,unetr_block}.py).

These are the decoder's full-resolution 3^3 convolutions.  Inference
(no autograd recording) on the GPU runs UnetResBlock / UnetBasicBlock / Convolution(3^3, stride
1) on the waveformer_amd kernels, channel-last end to end: the implicit-GEMM MFMA convolution
(ops.conv3d_k3), InstanceNorm statistics and one fused norm + residual + LeakyReLU pass
(ops.instnorm_stats / ops.norm_act), the 1x1 residual conv as one GEMM.  Training (autograd)
runs every convolution through wfa.conv_train: the 3^3 convs on the HIP forward / input- /
weight-gradient kernels, 1x1 and 2^3 transposed convs on the library's MFMA GEMMs -- no MIOpen
convolution, hence no MIOpen find, and no hipBLASLt but for the 4-channel shapes.  norm_name is always "instance" (InstanceNorm3d, affine=False) and the
activation LeakyReLU(0.01), as Waveformer builds them.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple, Union

import torch
import torch.nn as nn

from . import autograd as wfa
from . import ops


def _records_grad(x: torch.Tensor, *mods: nn.Module) -> bool:
    if not torch.is_grad_enabled():
        return False
    return x.requires_grad or any(p.requires_grad for m in mods for p in m.parameters())


def _k3_ok(conv: nn.Module, cin: int) -> bool:
    """A Conv3d the channel-last MFMA kernel implements: 3^3, stride 1, padding 1, dense."""
    return (type(conv) is nn.Conv3d and conv.kernel_size == (3, 3, 3) and conv.stride == (1, 1, 1)
            and conv.padding == (1, 1, 1) and conv.dilation == (1, 1, 1) and conv.groups == 1
            and conv.padding_mode == "zeros" and cin % 4 == 0 and conv.out_channels % 16 == 0)


def _in_ok(norm: nn.Module) -> bool:
    return (type(norm) is nn.InstanceNorm3d and not norm.affine
            and not norm.track_running_stats)


def _fast_ok(x: torch.Tensor, *mods: nn.Module) -> bool:
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 5
            and not _records_grad(x, *mods))


def _norm(norm_name, channels: int) -> nn.Module:
    name = norm_name[0] if isinstance(norm_name, tuple) else norm_name
    kw = dict(norm_name[1]) if isinstance(norm_name, tuple) and len(norm_name) > 1 else {}
    name = str(name).lower()
    if name == "instance":
        return nn.InstanceNorm3d(channels, **kw)
    if name == "batch":
        return nn.BatchNorm3d(channels, **kw)
    if name == "group":
        return nn.GroupNorm(num_channels=channels, **kw)
    raise ValueError(f"unsupported norm_name {norm_name!r}")


class Convolution(nn.Sequential):
    """monai Convolution with conv_only / act=None / norm=None: a container whose single child
    is named `conv` (state_dict key `<name>.conv.weight`)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, bias,
                 is_transposed=False, output_padding=0):
        super().__init__()
        if is_transposed:
            conv = nn.ConvTranspose3d(in_channels, out_channels, kernel_size, stride, padding,
                                      output_padding=output_padding, bias=bias)
        else:
            conv = nn.Conv3d(in_channels, out_channels, kernel_size, stride, padding, bias=bias)
        self.add_module("conv", conv)

    def forward(self, x):
        conv = self.conv
        if _fast_ok(x, self) and _k3_ok(conv, x.shape[1]):
            return ops.conv3d_k3(x, conv.weight, conv.bias)
        # training (autograd recording): the MFMA conv forward / input / weight gradients
        # (wfa.Conv3dK3), 1x1 and transposed convs as channel-last GEMMs (wfa.conv_train)
        return wfa.conv_train(conv, x)


def get_conv_layer(spatial_dims: int, in_channels: int, out_channels: int,
                   kernel_size: Union[Sequence[int], int] = 3, stride: Union[Sequence[int], int] = 1,
                   bias: bool = False, conv_only: bool = True, is_transposed: bool = False,
                   **_unused) -> Convolution:
    """monai.networks.blocks.dynunet_block.get_conv_layer (dynunet_block.py:270-301) for 3D,
    act/norm/dropout None: padding (k - s + 1) // 2, output_padding 2p + s - k."""
    if spatial_dims != 3:
        raise ValueError("only 3D is supported")
    k = kernel_size if isinstance(kernel_size, int) else kernel_size[0]
    s = stride if isinstance(stride, int) else stride[0]
    pad = (k - s + 1) // 2
    if pad < 0:
        raise AssertionError("padding value should not be negative")
    op = 2 * pad + s - k if is_transposed else 0
    return Convolution(in_channels, out_channels, kernel_size, stride, pad, bias, is_transposed, op)


def _act_for_conv2(h: torch.Tensor, s1: torch.Tensor, slope: float) -> torch.Tensor:
    """norm1 + lrelu of conv1's output, the input of conv2: stored fp16 when conv2 runs at the
    fp16 precision (the operands it would round to anyway, half the bytes), else in place."""
    if ops.prec_id() == ops.FP16 and h.shape[1] % 4 == 0:
        return ops.norm_act_h(h, s1, slope=slope)
    return ops.norm_act(h, s1, slope=slope, out=h)


def _into(y: torch.Tensor, out: Optional[torch.Tensor]) -> torch.Tensor:
    return y if out is None else out.copy_(y)


class UnetResBlock(nn.Module):
    """conv3-norm-lrelu-conv3-norm (+ 1x1 conv + norm residual when channels change) -> lrelu
    (monai dynunet_block.py:25-111)."""

    _split_conv1 = False  # fp16 policy: conv1 keeps bf16x3 (ops.FP16_SPLIT_OPS "skip_conv")

    def __init__(self, spatial_dims: int, in_channels: int, out_channels: int,
                 kernel_size=3, stride=1, norm_name: Union[Tuple, str] = "instance",
                 act_name=("leakyrelu", {"inplace": True, "negative_slope": 0.01}), dropout=None):
        super().__init__()
        self.conv1 = get_conv_layer(spatial_dims, in_channels, out_channels, kernel_size, stride)
        self.conv2 = get_conv_layer(spatial_dims, out_channels, out_channels, kernel_size, 1)
        self.lrelu = nn.LeakyReLU(negative_slope=0.01, inplace=True)
        self.norm1 = _norm(norm_name, out_channels)
        self.norm2 = _norm(norm_name, out_channels)
        s = stride if isinstance(stride, int) else max(stride)
        self.downsample = in_channels != out_channels or s != 1
        if self.downsample:
            self.conv3 = get_conv_layer(spatial_dims, in_channels, out_channels, 1, stride)
            self.norm3 = _norm(norm_name, out_channels)

    def _fast(self, inp) -> bool:
        c3 = self.conv3.conv if self.downsample else None
        return (_fast_ok(inp, self) and _k3_ok(self.conv1.conv, inp.shape[1])
                and _k3_ok(self.conv2.conv, self.conv2.conv.in_channels)
                and _in_ok(self.norm1) and _in_ok(self.norm2)
                and (c3 is None or (type(c3) is nn.Conv3d and c3.kernel_size == (1, 1, 1)
                                    and c3.stride == (1, 1, 1) and _in_ok(self.norm3))))

    def forward(self, inp, out=None):
        """out: optional channel-last destination (e.g. a channel slice of a decoder's concat
        buffer) the result is written into and returned as."""
        if self._fast(inp):
            slope = self.lrelu.negative_slope
            x = ops.to_cl(inp)
            with ops.op_precision("skip_conv" if self._split_conv1 else "conv"):
                h, s1 = ops.conv3d_k3(x, self.conv1.conv.weight, self.conv1.conv.bias,
                                      norm_eps=self.norm1.eps)
            y, s2 = ops.conv3d_k3(_act_for_conv2(h, s1, slope), self.conv2.conv.weight,
                                  self.conv2.conv.bias, norm_eps=self.norm2.eps)
            dst = y if out is None else out
            if self.downsample:
                c3 = self.conv3.conv
                if x.shape[1] <= 7:  # few input channels (encoder1): residual on the fly
                    return ops.norm_act_lin(y, s2, x, c3.weight, c3.bias, self.norm3.eps,
                                            slope=slope, out=dst)
                res = ops.conv1x1_cl(x, c3.weight, c3.bias)
                return ops.norm_act(y, s2, res, ops.instnorm_stats(res, self.norm3.eps),
                                    slope=slope, out=dst)
            return ops.norm_act(y, s2, x, slope=slope, out=dst)
        return _into(self._forward_slow(inp), out)

    def _forward_slow(self, inp):
        if self._train_ok(inp):
            # training on the GPU: convolutions through wfa.conv_train, each InstanceNorm +
            # residual + LeakyReLU as one fused HIP op with a HIP backward (wfa.NormActFn)
            slope = self.lrelu.negative_slope
            h = wfa.norm_act(self.conv1(inp), slope=slope, eps=self.norm1.eps)
            out = self.conv2(h)
            if self.downsample:
                return wfa.norm_act(out, self.conv3(inp), slope, self.norm2.eps, self.norm3.eps,
                                    normed_residual=True)
            return wfa.norm_act(out, inp, slope, self.norm2.eps)
        out = self.lrelu(self.norm1(self.conv1(inp)))
        out = self.norm2(self.conv2(out))
        res = self.norm3(self.conv3(inp)) if self.downsample else inp
        return self.lrelu(out + res)

    def _train_ok(self, inp) -> bool:
        return (inp.is_cuda and inp.dtype == torch.float32 and inp.dim() == 5
                and inp.shape[1] % 4 == 0 and self.conv1.conv.out_channels % 4 == 0
                and _in_ok(self.norm1) and _in_ok(self.norm2)
                and (not self.downsample or _in_ok(self.norm3))
                and type(self.lrelu) is nn.LeakyReLU and self.lrelu.negative_slope > 0)


class UnetBasicBlock(nn.Module):
    """conv3-norm-lrelu-conv3-norm-lrelu (monai dynunet_block.py:114-185)."""

    _split_conv1 = False  # fp16 policy, as UnetResBlock

    def __init__(self, spatial_dims: int, in_channels: int, out_channels: int, kernel_size=3,
                 stride=1, norm_name: Union[Tuple, str] = "instance", act_name=None, dropout=None):
        super().__init__()
        self.conv1 = get_conv_layer(spatial_dims, in_channels, out_channels, kernel_size, stride)
        self.conv2 = get_conv_layer(spatial_dims, out_channels, out_channels, kernel_size, 1)
        self.lrelu = nn.LeakyReLU(negative_slope=0.01, inplace=True)
        self.norm1 = _norm(norm_name, out_channels)
        self.norm2 = _norm(norm_name, out_channels)

    def forward(self, inp, out=None):
        if (_fast_ok(inp, self) and _k3_ok(self.conv1.conv, inp.shape[1])
                and _k3_ok(self.conv2.conv, self.conv2.conv.in_channels)
                and _in_ok(self.norm1) and _in_ok(self.norm2)):
            slope = self.lrelu.negative_slope
            with ops.op_precision("skip_conv" if self._split_conv1 else "conv"):
                h, s1 = ops.conv3d_k3(inp, self.conv1.conv.weight, self.conv1.conv.bias,
                                      norm_eps=self.norm1.eps)
            y, s2 = ops.conv3d_k3(_act_for_conv2(h, s1, slope), self.conv2.conv.weight,
                                  self.conv2.conv.bias, norm_eps=self.norm2.eps)
            return ops.norm_act(y, s2, slope=slope, out=y if out is None else out)
        return _into(self._forward_slow(inp), out)

    def _forward_slow(self, inp):
        if (inp.is_cuda and inp.dtype == torch.float32 and inp.dim() == 5
                and self.conv1.conv.out_channels % 4 == 0 and _in_ok(self.norm1)
                and _in_ok(self.norm2) and self.lrelu.negative_slope > 0):
            slope = self.lrelu.negative_slope  # training: fused HIP norm + LeakyReLU
            h = wfa.norm_act(self.conv1(inp), slope=slope, eps=self.norm1.eps)
            return wfa.norm_act(self.conv2(h), slope=slope, eps=self.norm2.eps)
        out = self.lrelu(self.norm1(self.conv1(inp)))
        return self.lrelu(self.norm2(self.conv2(out)))


class UnetOutBlock(nn.Module):
    """1x1x1 conv with bias (monai dynunet_block.py:188-210)."""

    def __init__(self, spatial_dims: int, in_channels: int, out_channels: int, dropout=None):
        super().__init__()
        self.conv = get_conv_layer(spatial_dims, in_channels, out_channels, 1, 1, bias=True)

    def forward(self, inp):
        c = self.conv.conv if hasattr(self.conv, "conv") else self.conv
        if (_fast_ok(inp, self) and type(c) is nn.Conv3d and c.kernel_size == (1, 1, 1)
                and c.stride == (1, 1, 1) and c.padding == (0, 0, 0) and c.dilation == (1, 1, 1)
                and c.groups == 1 and inp.shape[1] % 4 == 0
                and inp.shape[1] <= 120 and c.out_channels <= 16
                and ops.cl_ld(inp) is not None):
            # channel-last decoder output -> NCDHW logits in one pass (wf_conv1x1_head_cl)
            return ops.conv1x1_head(inp, c.weight, c.bias)
        return self.conv(inp)


class UnetrBasicBlock(nn.Module):
    """monai unetr_block.py:209-259: `layer` = UnetResBlock or UnetBasicBlock."""

    def __init__(self, spatial_dims: int, in_channels: int, out_channels: int, kernel_size,
                 stride, norm_name, res_block: bool = False):
        super().__init__()
        cls = UnetResBlock if res_block else UnetBasicBlock
        self.layer = cls(spatial_dims, in_channels, out_channels, kernel_size, stride, norm_name)

    def forward(self, inp, out=None):
        return self.layer(inp, out=out)


class UnetrUpBlock(nn.Module):
    """monai unetr_block.py:22-86: transposed conv (no bias), concat skip, conv block."""

    def __init__(self, spatial_dims: int, in_channels: int, out_channels: int, kernel_size,
                 upsample_kernel_size, norm_name, res_block: bool = False):
        super().__init__()
        self.transp_conv = get_conv_layer(spatial_dims, in_channels, out_channels,
                                          upsample_kernel_size, upsample_kernel_size,
                                          is_transposed=True)
        cls = UnetResBlock if res_block else UnetBasicBlock
        self.conv_block = cls(spatial_dims, 2 * out_channels, out_channels, kernel_size, 1,
                              norm_name)

    def forward(self, inp, skip, skip_in_place: bool = False):
        """`skip_in_place=True` (the backbone's decoder1 only): `skip` is channels [Cout, ...)
        of a channel-last buffer the caller allocated for this block's concatenation, so the
        transposed conv writes channels [0, Cout) of that same buffer.  Without the flag the
        skip is never written through, whatever storage it views."""
        tc = self.transp_conv.conv
        if (_fast_ok(inp, self) and type(tc) is nn.ConvTranspose3d and tc.kernel_size == (2, 2, 2)
                and tc.stride == (2, 2, 2) and tc.padding == (0, 0, 0)
                and tc.output_padding == (0, 0, 0) and tc.groups == 1 and tc.dilation == (1, 1, 1)):
            return self.conv_block(self._upsample_cat(inp, skip, tc, skip_in_place))
        out = self.transp_conv(inp)
        return self.conv_block(torch.cat((out, skip), dim=1))

    @staticmethod
    def _upsample_cat(inp, skip, tc, skip_in_place=False):
        """ConvTranspose3d(k=2, s=2) + torch.cat((out, skip), 1) into one channel-last buffer:
        the transposed conv is one GEMM (positions x Cin) . (Cin x 8 Cout) whose columns are the
        8 sub-voxels, stored straight into the buffer's first Cout channels (the MFMA GEMM's
        sub-voxel epilogue; an fp32 torch GEMM + scatter for channel counts it does not take)."""
        B, Cin, d, h, w = inp.shape
        Cout = tc.out_channels
        if tuple(skip.shape) != (B, skip.shape[1], 2 * d, 2 * h, 2 * w):
            raise ValueError(f"skip {tuple(skip.shape)} does not match the up-sampled input")
        # a skip the caller produced into channels [Cout, ...) of the concat buffer it
        # allocated for this block (the backbone's encoder1, flagged skip_in_place) needs no copy
        parent = ops.cl_parent(skip, Cout) if skip_in_place else None
        in_place = parent is not None and parent.shape[1] == Cout + skip.shape[1]
        buf = parent if in_place else ops.empty_cl(B, Cout + skip.shape[1], 2 * d, 2 * h, 2 * w,
                                                   inp.device)
        if Cin % 8 == 0 and Cout % 4 == 0:
            # one MFMA GEMM whose epilogue stores the sub-voxels + bias (wf_convtranspose2_cl)
            ops.convtranspose2_cl(inp, tc.weight, tc.bias, buf)
            if not in_place:
                ops.copy_cl(skip, buf[:, Cout:])
            return buf
        rows = ops.to_cl(inp).permute(0, 2, 3, 4, 1).reshape(-1, Cin)
        wr = tc.weight.permute(0, 2, 3, 4, 1).reshape(Cin, 8 * Cout)
        g = rows @ wr
        if Cout % 4 == 0:
            # sub-voxel scatter + bias in one HIP pass (layout.hip), skip copied channel-last
            bias = tc.bias.detach().contiguous() if tc.bias is not None else None
            ops.subvoxel_scatter_cl(g, bias, buf)
            if not in_place:
                ops.copy_cl(skip, buf[:, Cout:])
            return buf
        if tc.bias is not None:
            g = g + tc.bias.repeat(8)
        dst = buf.permute(0, 2, 3, 4, 1)[..., :Cout]
        dst = dst.unflatten(3, (w, 2)).unflatten(2, (h, 2)).unflatten(1, (d, 2))
        dst.permute(0, 1, 3, 5, 2, 4, 6, 7).copy_(g.view(B, d, h, w, 2, 2, 2, Cout))
        if not in_place:
            buf[:, Cout:].copy_(skip)
        return buf


class PatchEmbed(nn.Module):
    """monai.networks.blocks.PatchEmbed (patchembedding.py:147-225) as MultiscaleTransformer
    builds it: `proj` = Conv3d(k = s = patch_size), optional `norm`.  The forward used by the
    encoder is ops.patch_embed (HIP); this module only owns the parameters."""

    def __init__(self, patch_size=2, in_chans: int = 1, embed_dim: int = 48, norm_layer=None,
                 spatial_dims: int = 3):
        super().__init__()
        if spatial_dims != 3:
            raise ValueError("only 3D is supported")
        ps = patch_size if isinstance(patch_size, int) else patch_size[0]
        self.patch_size = (ps, ps, ps)
        self.embed_dim = embed_dim
        self.proj = nn.Conv3d(in_chans, embed_dim, kernel_size=ps, stride=ps)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None
