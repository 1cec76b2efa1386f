"""Waveformer -- the full U-shaped network and its factory.

Mirrors network_models/network_backbone.py (ProjectionHead :35-63, ChannelCalibration :66-128,
Waveformer :131-407, create_waveformer :410-431): same constructor signatures and the same 232
state_dict keys at the default configuration, so reference checkpoints load with strict=True.
The encoder and the IDWT synthesis run on the waveformer_amd HIP kernels; so do the MONAI-style
decoder blocks, ChannelCalibration and ProjectionUpsample (3^3 convolutions on conv3d_k3,
InstanceNorm + LeakyReLU fused, 1x1 / transposed convolutions on the in-house MFMA GEMMs;
blocks.py) -- no MIOpen convolution on any path.
"""
from __future__ import annotations

import os
from typing import Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F
from functools import partial

from .. import autograd as wfa
from .. import ops

from ..blocks import UnetOutBlock, UnetrBasicBlock, UnetrUpBlock
from .idwt_upsample import UnetrIDWTBlock
from .wave_helper import ProjectionUpsample
from .waveformer import MultiscaleTransformer

# WF_CL_OUTS=0 (A/B): the encoder hands NCDHW stage outputs over, as the reference's proj_out
_CL_OUTS = os.environ.get("WF_CL_OUTS", "1") != "0"


class ProjectionHead(nn.Module):
    """Contrastive projection head (never instantiated by Waveformer).  'convmlp' uses
    Conv3d -> BatchNorm3d + ReLU -> Conv3d (lib ModuleHelper.BNReLU with 'torchbn')."""

    def __init__(self, dim_in: int, proj_dim: int = 256, proj: str = 'convmlp',
                 bn_type: str = 'torchbn'):
        super().__init__()
        if proj == 'linear':
            self.proj = nn.Conv2d(dim_in, proj_dim, kernel_size=1)
        elif proj == 'convmlp':
            self.proj = nn.Sequential(nn.Conv3d(dim_in, dim_in, kernel_size=1),
                                      nn.Sequential(nn.BatchNorm3d(dim_in), nn.ReLU()),
                                      nn.Conv3d(dim_in, proj_dim, kernel_size=1))
        else:
            raise ValueError(f"Unknown projection type: {proj}")

    def forward(self, x):
        return F.normalize(self.proj(x), p=2, dim=1)


class ChannelCalibration(nn.Module):
    """SE-style calibration of the deepest encoder output (network_backbone.py:66-128)."""

    def __init__(self, in_channels: int = 384, reduction_ratio: int = 4,
                 norm_layer: type = nn.BatchNorm3d):
        super().__init__()
        r = in_channels // reduction_ratio
        self.reduce = nn.Conv3d(in_channels, r, kernel_size=1)
        self.norm_reduce = norm_layer(r)
        self.conv = nn.Conv3d(r, r, kernel_size=3, padding=1)
        self.norm_conv = norm_layer(r)
        self.expand = nn.Conv3d(r, in_channels, kernel_size=1)
        self.norm_expand = norm_layer(in_channels)
        self.global_pool = nn.AdaptiveAvgPool3d(1)
        self.fc1 = nn.Linear(in_channels, r)
        self.fc2 = nn.Linear(r, in_channels)
        self.residual = nn.Conv3d(in_channels, in_channels, kernel_size=1)
        self.sigmoid = nn.Sigmoid()
        self.relu = nn.ReLU()

    def forward(self, x):
        # the convs through wfa.conv_train (GEMM 1x1s, HIP 3^3; the modules for CPU tensors):
        # MIOpen picks its naive direct kernels for these NCDHW 6^3 shapes (2 ms a launch)
        cv = wfa.conv_train
        identity = cv(self.residual, x)
        x = self.relu(self.norm_reduce(cv(self.reduce, x)))
        x = self.relu(self.norm_conv(cv(self.conv, x)))
        x = self.norm_expand(cv(self.expand, x))
        b, c = x.shape[:2]
        # fc1 / fc2 (M = batch rows) on the library's GEMMs too: no platform-BLAS call remains
        se = self.sigmoid(wfa.linear(self.fc2, F.relu(wfa.linear(self.fc1,
                                                                 self.global_pool(x).view(b, c)))))
        return self.relu(x * se.view(b, c, 1, 1, 1) + identity)


class Waveformer(nn.Module):
    def __init__(self, img_size: Tuple[int, int, int] = (96, 96, 96), patch_size: int = 2,
                 in_chans: int = 1, out_chans: int = 13, depths: list = None,
                 feat_size: list = None, num_heads: list = None, drop_path_rate: float = 0.1,
                 layer_scale_init_value: float = 1e-6, hidden_size: int = 768,
                 norm_name: Union[Tuple, str] = "instance", conv_block: bool = True,
                 res_block: bool = True, spatial_dims: int = 3, use_checkpoint: bool = False,
                 network_config: dict = None) -> None:
        super().__init__()
        depths = depths or [2, 2, 2, 2]
        feat_size = feat_size or [48, 96, 192, 384]
        num_heads = num_heads or [3, 6, 12, 24]
        self.img_size = img_size
        self.hidden_size = hidden_size
        self.patch_size = patch_size
        self.num_heads = num_heads
        self.in_chans = in_chans
        self.out_chans = out_chans
        self.depths = depths
        self.drop_path_rate = drop_path_rate
        self.feat_size = feat_size
        self.layer_scale_init_value = layer_scale_init_value
        self.spatial_dims = spatial_dims
        self.network_config = network_config or {}
        self.transformer_config = self.network_config.get('transformer', {})
        self.hf_refinement = self.transformer_config.get('hf_refinement', False)
        self.out_indice = list(range(len(self.depths)))
        tc = self.transformer_config
        self.waveformer_encoder = MultiscaleTransformer(
            img_size=self.img_size, in_chans=self.in_chans, patch_size=self.patch_size,
            num_classes=self.out_chans, embed_dims=tc.get('embed_dims', self.feat_size),
            depths=tc.get('depths', self.depths), num_heads=tc.get('num_heads', self.num_heads),
            drop_path_rate=tc.get('drop_path_rate', self.drop_path_rate),
            mlp_ratios=tc.get('mlp_ratios', [4, 4, 4, 4]),
            decom_levels=tc.get('decom_levels', [3, 2, 1, 0]),
            multi_scale_attention=tc.get('multi_scale_attention', True), qkv_bias=True,
            norm_layer=partial(nn.LayerNorm, eps=1e-6), attn_drop_rate=0, drop_rate=0,
            network_config=self.network_config)
        fs = self.feat_size
        blk = partial(UnetrBasicBlock, spatial_dims=spatial_dims, kernel_size=3, stride=1,
                      norm_name=norm_name, res_block=res_block)
        self.encoder1 = blk(in_channels=in_chans, out_channels=fs[0])
        self.encoder2 = blk(in_channels=fs[0], out_channels=fs[0])
        self.encoder3 = blk(in_channels=fs[1], out_channels=fs[1])
        self.encoder4 = blk(in_channels=fs[2], out_channels=fs[2])
        # config 5's fp16 policy (ops.FP16_SPLIT_OPS): the first convolution of each block
        # reading the transformer's skip features keeps the fp32-faithful split
        for e in (self.encoder2, self.encoder3, self.encoder4):
            e.layer._split_conv1 = True
        self.encoder10 = ChannelCalibration(in_channels=fs[3], reduction_ratio=4,
                                            norm_layer=nn.InstanceNorm3d)
        idwt = partial(UnetrIDWTBlock, spatial_dims=spatial_dims, in_channels=fs[3],
                       hf_refinement=self.hf_refinement, wavelet='db1', kernel_size=3,
                       norm_name=norm_name, res_block=res_block)
        self.decoder4 = idwt(out_channels=fs[2], stage=1)
        self.decoder3 = idwt(out_channels=fs[1], stage=2)
        self.decoder2 = idwt(out_channels=fs[0], stage=3)
        self.learnable_up4 = ProjectionUpsample(fs[2], fs[0], stride=4, residual=True,
                                                use_double_conv=True)
        self.learnable_up3 = ProjectionUpsample(fs[1], fs[0], stride=2, residual=True)
        self.decoder1 = UnetrUpBlock(spatial_dims=spatial_dims, in_channels=fs[0] * 3,
                                     out_channels=fs[0], kernel_size=3, upsample_kernel_size=2,
                                     norm_name=norm_name, res_block=res_block)
        self.out = UnetOutBlock(spatial_dims=spatial_dims, in_channels=fs[0],
                                out_channels=self.out_chans)

    def _get_norm_layer(self, norm_name: str) -> type:
        layers = {'LayerNorm': nn.LayerNorm, 'BatchNorm3d': nn.BatchNorm3d,
                  'InstanceNorm3d': nn.InstanceNorm3d, 'GroupNorm': nn.GroupNorm}
        if norm_name not in layers:
            raise ValueError(f"Unknown normalization layer: {norm_name}")
        return layers[norm_name]

    def forward(self, x_in: torch.Tensor) -> torch.Tensor:
        """network_backbone.py:380-407.  One weight_scope per forward: the split / packed
        forms of the weights are rebuilt once at its start (ops.weight_scope)."""
        with ops.weight_scope(self):
            return self._forward(x_in)

    def _forward(self, x_in: torch.Tensor) -> torch.Tensor:
        infer = x_in.is_cuda and not torch.is_grad_enabled()
        # inference: the stage outputs come channel-last, the layout encoder2-4 / encoder10 read
        # (proj_out's NCDHW write and ops.to_cl's transpose back are skipped; same values)
        outs, outs_hf = self.waveformer_encoder(x_in, channel_last=infer and _CL_OUTS)
        fs0 = self.decoder1.transp_conv.conv.out_channels
        if infer:
            # inference: encoder1 writes straight into channels [fs0, 2 fs0) of decoder1's
            # channel-last concat buffer (blocks.UnetrUpBlock finds it there, no skip copy)
            B, _, D, H, W = x_in.shape
            buf1 = ops.empty_cl(B, fs0 + self.encoder1.layer.conv1.conv.out_channels, D, H, W,
                                x_in.device)
            enc0 = self.encoder1(x_in, out=buf1[:, fs0:])
            enc0_in_place = True
        else:
            enc0 = self.encoder1(x_in)
            enc0_in_place = False
        enc1 = self.encoder2(outs[0])
        enc2 = self.encoder3(outs[1])
        enc3 = self.encoder4(outs[2])
        dec5 = self.encoder10(outs[3])
        dec4 = self.decoder4(dec5, enc3, outs_hf[-1])
        dec3 = self.decoder3(dec5, enc2, outs_hf[-2])
        dec2 = self.decoder2(dec5, enc1, outs_hf[-3])
        up4 = self.learnable_up4(dec4)
        up3 = self.learnable_up3(dec3)
        if torch.is_grad_enabled() and any(t.requires_grad for t in (up4, up3, dec2)):
            cat = torch.cat([up4, up3, dec2], dim=1)
        else:  # inference: one channel-last buffer, the layout decoder1's kernels read
            cat = ops.cat_cl([up4, up3, dec2])
        dec1 = self.decoder1(cat, enc0, skip_in_place=enc0_in_place)
        # the HIP decoder path is channel-last; hand the caller the reference's NCDHW layout
        return self.out(dec1).contiguous()


def create_waveformer(network_config: dict) -> Waveformer:
    """network_backbone.py:410-431."""
    return Waveformer(img_size=network_config['img_size'],
                      patch_size=network_config['patch_size'],
                      in_chans=network_config['in_chans'],
                      out_chans=network_config['out_chans'],
                      depths=network_config['depths'],
                      feat_size=network_config['embed_dims'],
                      num_heads=network_config['num_heads'],
                      drop_path_rate=network_config['drop_path_rate'],
                      use_checkpoint=network_config.get('use_checkpoint', False),
                      network_config=network_config)
