"""MultiscaleTransformer -- the 4-stage WaveFormer encoder.

Mirrors network_models/waveformer.py (class MultiscaleTransformer, :36-340): same constructor,
submodules and state_dict keys.  forward_features keeps every activation channel-last and runs
PatchEmbed, the Blocks, PatchMerging and proj_out on the HIP kernels; the only layout change
is proj_out's transposed write of each stage output to NCDHW (the tensors the decoder uses).
"""
from __future__ import annotations

import math
import os
import time
from typing import List, Tuple

import torch
import torch.nn as nn
import torch.nn.init as init

from .. import autograd as wfa
from .. import ops
from ..blocks import PatchEmbed as _MonaiPatchEmbed
from . import wave_helper as WH
from .wave_helper import Block, PatchMerging


# WF_HF_SKIP=0 (A/B): every Block computes its detail bands, as the reference does
_HF_SKIP = os.environ.get("WF_HF_SKIP", "1") != "0"


class MultiscaleTransformer(nn.Module):
    def __init__(self, img_size=(128, 128, 128), patch_size=2, in_chans=4, num_classes=4,
                 embed_dims=[48, 96, 192, 384], num_heads=[3, 6, 12, 24], mlp_ratios=[4, 4, 4, 4],
                 decom_levels=[3, 2, 1, 0], multi_scale_attention=True, qkv_bias=False,
                 qk_scale=None, drop_rate=0., attn_drop_rate=0., drop_path_rate=0.,
                 norm_layer=nn.LayerNorm, patch_norm=False, depths=[2, 2, 2, 2],
                 network_config=None):
        super().__init__()
        self.network_config = network_config or {}
        self.num_classes = num_classes
        self.depths = depths
        self.patch_norm = patch_norm
        self.patch_size = patch_size
        self.img_size = img_size
        self.levels = decom_levels
        self.multi_scale_attention = multi_scale_attention
        self.patch_embed = _MonaiPatchEmbed(patch_size=patch_size, in_chans=in_chans,
                                            embed_dim=embed_dims[0],
                                            norm_layer=norm_layer if patch_norm else None,
                                            spatial_dims=len(img_size))
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [v.item() for v in torch.linspace(0, drop_path_rate, sum(depths))]
        cur = 0
        for s in range(4):
            div = 2 ** (s + 1)
            blocks = nn.ModuleList([
                Block(dim=embed_dims[s], num_heads=num_heads[s], mlp_ratio=mlp_ratios[s],
                      qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop_rate,
                      attn_drop=attn_drop_rate, drop_path=dpr[cur + i], norm_layer=norm_layer,
                      level=self.levels[s], ms_attention=self.multi_scale_attention,
                      img_size=tuple(d // div for d in img_size),
                      network_config=self.network_config)
                for i in range(depths[s])])
            setattr(self, f"block{s + 1}", blocks)
            cur += depths[s]
            if s < 3:
                setattr(self, f"downsample_{s + 1}",
                        PatchMerging(dim=embed_dims[s], norm_layer=norm_layer,
                                     spatial_dims=len(img_size)))
        self.apply(self._init_weights)

    def _init_weights(self, m: nn.Module):
        cfg = self.network_config.get('initialization', {})
        if isinstance(m, nn.Linear):
            nn.init.trunc_normal_(m.weight, std=cfg.get('weight_std', 0.02))
            if m.bias is not None:
                init.constant_(m.bias, cfg.get('bias_constant', 0.0))
        elif isinstance(m, nn.LayerNorm):
            init.constant_(m.bias, cfg.get('layer_norm_bias', 0.0))
            init.constant_(m.weight, cfg.get('layer_norm_weight', 1.0))
        elif isinstance(m, (nn.Conv2d, nn.Conv3d)):
            fan_out = math.prod(m.kernel_size) * m.out_channels // m.groups
            m.weight.data.normal_(0, math.sqrt(2.0 / fan_out))
            if m.bias is not None:
                m.bias.data.zero_()

    def proj_out(self, x: torch.Tensor, normalize: bool = False) -> torch.Tensor:
        """waveformer.py:182-204 on an NCDHW tensor (API form).  forward_features calls the
        fused channel-last -> NCDHW kernel directly."""
        if x.dim() != 5:
            raise NotImplementedError("waveformer_amd: 3D (5-D tensor) proj_out only")
        return ops.proj_out(x.permute(0, 2, 3, 4, 1).contiguous(), normalize)

    def init_weights(self, pretrained: str):
        if isinstance(pretrained, str):
            self.load_dualpath_model(self, pretrained)
        else:
            raise TypeError('pretrained must be a str or None')

    def load_dualpath_model(self, model: nn.Module, model_file):
        t0 = time.time()
        if isinstance(model_file, str):
            sd = torch.load(model_file, map_location=torch.device('cpu'), weights_only=True)
            if 'model' in sd.keys():
                sd = sd['model']
        else:
            sd = model_file
        model.load_state_dict(sd, strict=False)
        if hasattr(self, 'logger'):
            self.logger.info(f"Load model, Time usage: {time.time() - t0}")

    def forward_features(self, x_rgb: torch.Tensor, normalize: bool = True, *,
                         channel_last: bool = False) -> Tuple[List[torch.Tensor], List]:
        """waveformer.py:260-322: PatchEmbed -> 4 stages (Blocks, PatchMerging) -> proj_out.
        Returns (outs: 4 NCDHW tensors, outs_hf: the last block's detail dicts of stages 1-3).
        channel_last (inference only): the outs are NCDHW-shaped channels_last_3d tensors of the
        same values -- the layout the full model's UnetResBlocks read (network_backbone.py)."""
        if self.patch_norm:
            raise NotImplementedError("waveformer_amd: patch_norm=True is not implemented")
        if x_rgb.dtype != torch.float32:
            raise TypeError("waveformer_amd: float32 input expected")
        pe = self.patch_embed.proj
        train = wfa.needs_grad(x_rgb, *self.parameters())
        ll0 = None  # the first Block's level-1 LL, formed by the fused PatchEmbed kernel
        b0 = self.block1[0]
        if train:
            x = wfa.PatchEmbedFn.apply(x_rgb.contiguous(), pe.weight.contiguous(), pe.bias)
        elif (_HF_SKIP and len(self.block1) > 1 and b0.ms_attention and b0.level > 0
              and x_rgb.is_cuda and not torch.compiler.is_compiling()):
            r = ops.patch_embed_ll(x_rgb.contiguous(), pe.weight.contiguous(), pe.bias,
                                   (b0.norm1.weight, b0.norm1.bias, b0.norm1.eps))
            x, ll0 = r if r is not None else (
                ops.patch_embed(x_rgb.contiguous(), pe.weight.contiguous(), pe.bias), None)
        else:
            x = ops.patch_embed(x_rgb.contiguous(), pe.weight.contiguous(), pe.bias)
        outs, outs_hf = [], []
        for s in range(4):
            if s > 0:
                x = getattr(self, f"downsample_{s}")(x)
            x_h = None
            blocks = getattr(self, f"block{s + 1}")
            for i, blk in enumerate(blocks):
                # only the stage's last Block's hf is kept (waveformer.py:288-292): the others
                # run the LL-only DWT in inference
                skip = _HF_SKIP and not train and i < len(blocks) - 1
                WH.HF_SKIP.blocks = {id(blk): ll0 if s == 0 and i == 0 else None} if skip else {}
                try:
                    r = blk(x)
                finally:
                    WH.HF_SKIP.blocks = {}
                if isinstance(r, tuple):
                    x, x_h = r
                else:
                    x = r
            B, D, H, W, C = x.shape
            if train:
                outs.append(wfa.ProjOutFn.apply(x, bool(normalize), 1e-5))
            elif channel_last:
                outs.append(ops.proj_out_cl(x, normalize))
            else:
                outs.append(ops.proj_out(x, normalize))
            if s < 3:
                outs_hf.append(x_h if x_h is not None else ())
        return outs, outs_hf

    def forward(self, x_rgb: torch.Tensor, *, channel_last: bool = False):
        with ops.weight_scope(self):  # split weights rebuilt once per forward (one launch)
            return self.forward_features(x_rgb, channel_last=channel_last)

    def flops(self) -> int:
        return 0
