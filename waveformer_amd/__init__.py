"""waveformer_amd -- MI355X (gfx950) implementation of the WaveFormer encoder/decoder hot path.

`waveformer_amd.network_models` mirrors the reference `network_models` package (same class
names, constructor arguments and state_dict keys); its hot-path ops run on the HIP kernels of
`libwaveformer_hip.so` through the C-ABI in include/waveformer_hip.h.
"""
__version__ = "0.1.0"
