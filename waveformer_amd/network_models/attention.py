"""Window multi-head self-attention with a 3D relative-position bias.

Mirrors network_models/attention.py (class Attention, :15-129): same constructor, parameters,
buffers and state_dict keys.  The forward is the waveformer::window_attn op (library.py) on the HIP kernels:
qkv GEMM -> flash-style QK^T + bias / softmax / PV core -> proj.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn as nn

from .. import autograd as wfa
from .. import library  # noqa: F401  (registers the torch.ops.waveformer ops)
from .. import ops

_OPS = torch.ops.waveformer


def relative_position_index(ws: int) -> torch.Tensor:
    """Pairwise index into the (2ws-1)^3-row bias table for the ws^3 tokens of a window
    (row-major (s, h, w) token order).  Reproduces the reference's depth stride of 3*ws-1
    (attention.py:51-52; quirk Q2) -- not the collision-free (2ws-1)^2."""
    ar = torch.arange(ws)
    s, h, w = torch.meshgrid(ar, ar, ar, indexing="ij")
    pos = torch.stack([s.reshape(-1), h.reshape(-1), w.reshape(-1)], dim=-1)  # (N, 3)
    d = pos[:, None, :] - pos[None, :, :] + (ws - 1)                           # (N, N, 3)
    return d[..., 0] * (3 * ws - 1) + d[..., 1] * (2 * ws - 1) + d[..., 2]


class Attention(nn.Module):
    def __init__(self, dim, num_heads=8, qkv_bias=False, qk_scale=None, attn_drop=0.,
                 proj_drop=0., window_size=6, img_size=(48, 48, 48)):
        super().__init__()
        assert dim % num_heads == 0, f"dim {dim} should be divided by num_heads {num_heads}."
        self.dim = dim
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = qk_scale or self.head_dim ** -0.5
        self.window_size = window_size
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * window_size - 1) ** 3, num_heads))
        self.register_buffer("relative_position_index", relative_position_index(window_size))
        # the index equals the reference's formula (re-checked when a state_dict is loaded):
        # the table-bias kernel then evaluates the formula in-kernel instead of reading it.
        # Valid for the buffer version it was checked at: an in-place write afterwards
        # (copy_ / fill_) bumps the version and the forward falls back to the dense bias built
        # from the buffer's contents (no host sync in the forward).  A device move keeps the
        # contents and starts the new tensor at a fresh version counter: _apply re-records it.
        self._index_formula = True
        self._index_version = self.relative_position_index._version
        nn.init.trunc_normal_(self.relative_position_bias_table, std=.02)
        self.softmax = nn.Softmax(dim=-1)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)
        self._index_formula = ops.index_is_formula(self.relative_position_index,
                                                   self.window_size)
        self._index_version = self.relative_position_index._version

    def _apply(self, fn, *args, **kwargs):
        # .to() / .cuda() / .half() replace the buffer by a copy of the same contents (at a
        # fresh version counter): the formula check still holds for the new tensor -- unless
        # the buffer was written in place since that check (its version moved on), in which
        # case the moved contents are checked again (a host sync, outside any forward)
        stale = self._index_formula and \
            self.relative_position_index._version != self._index_version
        ret = super()._apply(fn, *args, **kwargs)
        if stale:
            self._index_formula = ops.index_is_formula(self.relative_position_index,
                                                       self.window_size)
        self._index_version = self.relative_position_index._version
        return ret

    def _formula_valid(self) -> bool:
        if not self._index_formula:
            return False
        if torch.compiler.is_compiling():
            # a traced graph sees tensor versions as data-dependent symbols: the check stays
            # with eager mode (a compiled forward does not write the buffer in place)
            return True
        return self.relative_position_index._version == self._index_version

    def _check_train(self):
        if self.training and (self.attn_drop.p > 0 or self.proj_drop.p > 0):
            raise NotImplementedError("waveformer_amd: attention dropout > 0 is not supported")

    def _wf_split_params(self):
        return [self.qkv.weight, self.proj.weight]

    def forward_raster(self, x_cl: torch.Tensor,
                       ln: Optional[Tuple[torch.Tensor, torch.Tensor, float]] = None) -> torch.Tensor:
        """Attention over the ws^3 windows of a channel-last raster (B, D, H, W, C): the
        window_partition + forward + plain-reshape "reverse" of Block (wave_helper.py:491-499,
        quirk Q1).  Row r of the result (as a (B*D*H*W, C) matrix) is token r % N of window
        r // N; viewed as (B, D, H, W, C) it is exactly the reference's attn_windows.  One
        waveformer::window_attn op: it reads the bias table itself (ws 8, head_dim 16, the
        index buffer equal to the reference's formula) or its dense expansion."""
        self._check_train()
        lw, lb, eps = ln if ln is not None else (None, None, 0.0)
        train = wfa.needs_grad(x_cl, *self.parameters(), lw, lb)
        prec = wfa.SPLIT if train else ops.op_prec("attn")
        out, _, _ = _OPS.window_attn(x_cl, lw, lb, float(eps), self.qkv.weight, self.qkv.bias,
                                     self.relative_position_bias_table,
                                     self.relative_position_index, self.proj.weight,
                                     self.proj.bias, self.window_size, self.num_heads,
                                     float(self.scale), prec, train, self._formula_valid())
        return out

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: (B_, N, C) token batches, N = window_size^3 (attention.py:83-104)."""
        B_, N, C = x.shape
        ws = self.window_size
        if N != ws ** 3:
            raise ValueError(f"expected N = window_size^3 = {ws ** 3}, got {N}")
        x = x.contiguous()
        return self.forward_raster(x.view(B_, ws, ws, ws, C)).view(B_, N, C)

    def flops(self):
        N = self.window_size ** 3
        return 2 * N * self.dim * 3 * self.dim + 4 * N * N * self.dim + 2 * N * self.dim * self.dim
