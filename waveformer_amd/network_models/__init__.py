"""Drop-in replacement for the reference's `network_models` package
(network_models/__init__.py:11-62): the same exported names, backed by the MI355X kernels.

Use it in place of the reference package with e.g.
    import sys, waveformer_amd.network_models as nm; sys.modules["network_models"] = nm
before `from network_models import Waveformer, create_waveformer`.
"""
from .network_backbone import Waveformer, create_waveformer, ProjectionHead, ChannelCalibration
from .waveformer import MultiscaleTransformer
from .wave_helper import (
    Block, PatchMerging, PatchMergingV2, CCF_FFN, Mlp,
    WaveletTransform3D, DWConv, OverlapPatchEmbed, PatchEmbed,
    PosCNN, ProjectionUpsample,
)
from .idwt_upsample import UnetrIDWTBlock as IDWTBlock, HFRefinementRes
from .attention import Attention

__version__ = "1.0.0"

__all__ = [
    "Waveformer", "create_waveformer", "ProjectionHead", "ChannelCalibration",
    "MultiscaleTransformer",
    "Block", "PatchMerging", "PatchMergingV2", "CCF_FFN", "Mlp", "WaveletTransform3D", "DWConv",
    "OverlapPatchEmbed", "PatchEmbed", "PosCNN", "ProjectionUpsample",
    "IDWTBlock", "HFRefinementRes",
    "Attention",
]
