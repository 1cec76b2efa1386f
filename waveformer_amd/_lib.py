"""ctypes binding of libwaveformer_hip.so (the C-ABI declared in include/waveformer_hip.h).

This is the reference-side FFI a Python caller uses: every entry point takes raw device
pointers, int64 sizes and a hipStream_t, and returns an int status.  `call()` turns a non-zero
status into RuntimeError carrying `wf_last_error()`.

There is deliberately no fallback: if the library cannot be loaded every op raises, so a GPU
run can never silently take another path.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WAVEFORMER_HIP_LIB", os.path.join(_HERE, "libwaveformer_hip.so"))

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_F = ctypes.c_float

# name -> (restype, argtypes); must match include/waveformer_hip.h
SIGNATURES = {
    "wf_abi_version": (_I, []),
    "wf_last_error": (ctypes.c_char_p, []),
    "wf_cast_f32_to_bf16": (_I, [_P, _P, _I64, _P]),
    "wf_split_f32_to_bf16x2": (_I, [_P, _P, _I64, _P]),
    "wf_split_f32_to_bf16x2_multi": (_I, [_P, _I64, _I64, _P]),
    "wf_cast_f32_to_f16x2": (_I, [_P, _P, _I64, _P]),
    "wf_cast_f32_to_f16x2_multi": (_I, [_P, _I64, _I64, _P]),
    "wf_debug_poison_lds": (_I, [_I64, _I, _P]),
    "wf_patch_embed_ll_fwd": (_I, [_P, _P, _P, _P, _P, _P, _F, _P, _I64, _I64, _I64, _I64, _I64,
                                   _I64, _P]),
    "wf_patch_embed_fwd": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_dwt3d_haar_fwd": (_I, [_P, _P, _P, _F, _P, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_dwt3d_haar_fwd_ll": (_I, [_P, _P, _P, _F, _P, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_idwt3d_haar": (_I, [_P, _I64, _P, _P, _I, _P, _I64, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_idwt3d_haar_cl": (_I, [_P, _I64, _I64, _I64, _P, _P, _I, _P, _I64, _I64, _I64, _I64,
                               _I64, _I64, _I64, _P]),
    "wf_idwt3d_haar_cl_cat": (_I, [_P, _I64, _I64, _I64, _P, _P, _I, _P, _I64, _I64, _P, _I64,
                                   _I64, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_copy_cl": (_I, [_P, _I64, _P, _I64, _I64, _I64, _P]),
    "wf_subvoxel_scatter_cl": (_I, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_convtranspose2_cl": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _I, _P]),
    "wf_moments_cl": (_I, [_P, _I64, _I64, _I64, _I64, _P, _P]),
    "wf_conv3d_k3_fwd_xh": (_I, [_P, _I64, _P, _P, _P, _I64, _P, _P, _I64, _I64, _I64, _I64, _I64,
                                 _I64, _P]),
    "wf_conv3d_k3_workspace_bytes": (_I64, [_I64, _I64, _I64, _I64, _I64, _I64, _I, _I]),
    "wf_norm_act_h_cl": (_I, [_P, _I64, _P, _P, _I64, _I64, _I64, _I64, _F, _P]),
    "wf_upsample_trilinear_add_cl": (_I, [_P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _I, _P]),
    "wf_conv1x1_head_cl": (_I, [_P, _I64, _P, _P, _P, _I64, _I64, _I64, _I64, _P]),
    "wf_linear_smallk_fwd": (_I, [_P, _I64, _P, _P, _P, _I64, _I64, _I64, _I64, _P]),
    "wf_dwconv3d_stats_cl": (_I, [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_norm_act_lin_cl": (_I, [_P, _I64, _P, _P, _I64, _I64, _P, _P, _P, _I64, _I64, _I64, _I64, _F, _P]),
    "wf_dwt3d_fwd": (_I, [_P, _P, _I64, _I64, _I64, _I64, _P, _P, _I, _P]),
    "wf_idwt3d_level": (_I, [_P, _P, _I64, _I64, _I64, _I64, _I64, _P, _P, _I, _P, _I64, _I64,
                             _P]),
    "wf_conv3d_k3_packed_elems": (_I64, [_I64, _I64]),
    "wf_conv3d_k3_pack": (_I, [_P, _P, _I64, _I64, _P]),
    "wf_conv3d_k3_pack_f16": (_I, [_P, _P, _I64, _I64, _P]),
    "wf_conv3d_k3_fwd": (_I, [_P, _I64, _P, _P, _P, _I64, _P, _P, _I64, _I64, _I64, _I64,
                              _I64, _I64, _I, _P]),
    "wf_instnorm_finalize": (_I, [_P, _P, _I64, _I64, _I64, _F, _P]),
    "wf_instnorm_workspace_bytes": (_I64, [_I64, _I64]),
    "wf_instnorm_stats_cl": (_I, [_P, _I64, _I64, _I64, _I64, _F, _P, _P, _P]),
    "wf_resample_trilinear_cf": (_I, [_P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _I,
                                      _P, _I, _P]),
    "wf_conv3d_k3_wgrad_workspace_bytes": (_I64, [_I64] * 6),
    "wf_conv3d_k3_wgrad": (_I, [_P, _I64, _P, _I64, _P, _I, _P, _I64, _I64, _I64, _I64, _I64,
                                _I64, _P]),
    "wf_norm_act_bwd_workspace_bytes": (_I64, [_I64, _I64]),
    "wf_norm_act_bwd_cl": (_I, [_P, _I64, _P, _I64, _P, _I64, _P, _P, _I64, _P, _P, _I64, _P, _I64,
                                _I64, _I64, _I64, _F, _P, _P]),
    "wf_hf_refine_workspace_bytes": (_I64, [_I64, _I64]),
    "wf_hf_refine_fwd": (_I, [_P, _I64, _P, _P, _P, _P, _F, _P, _P, _I, _P, _P, _I64, _I64,
                              _I64, _I64, _I64, _P]),
    "wf_norm_act_cl": (_I, [_P, _I64, _P, _P, _I64, _P, _P, _I64, _I64, _I64, _I64, _F, _P]),
    "wf_upsample_trilinear_cl": (_I, [_P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _I64,
                                      _I, _P]),
    "wf_linear_fwd": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I, _I, _P]),
    "wf_window_attention_fwd_table": (_I, [_P, _P, _P, _F, _P, _P, _P, _P, _P, _P, _P,
                                           _I64, _I64, _I64, _I64, _I64, _I64, _I64, _F, _I,
                                           _P]),
    "wf_rel_pos_bias": (_I, [_P, _P, _P, _I64, _I64, _I64, _P]),
    "wf_window_attention_workspace_bytes": (_I64, [_I64, _I64, _I64, _I64, _I64, _I]),
    "wf_window_attention_fwd": (_I, [_P, _P, _P, _F, _P, _P, _P, _P, _P, _P, _P,
                                     _I64, _I64, _I64, _I64, _I64, _I64, _I64, _F, _I, _P]),
    "wf_msfuse_fwd": (_I, [_P, _P, _I, _P, _P, _P, _P, _F, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_ccf_ffn_workspace_bytes": (_I64, [_I64, _I64, _I64, _I64, _I64, _I64, _I]),
    "wf_ccf_ffn_fwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _F, _P, _P,
                            _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I, _P]),
    "wf_ccf_ffn_stage": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _F, _P,
                              _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I, _P]),
    "wf_patch_merging_fwd": (_I, [_P, _P, _P, _F, _P, _I, _P, _I64, _I64, _I64, _I64, _I64,
                                  _I, _P]),
    "wf_proj_out_fwd": (_I, [_P, _P, _I, _F, _I64, _I64, _I64, _P]),
    "wf_proj_out_cl_fwd": (_I, [_P, _P, _F, _I64, _I64, _P]),
    "wf_upsample_dwconv3d_stats_cl": (_I, [_P, _P, _P, _P, _P] + [_I64] * 8 + [_I, _P]),
    "wf_importance_map": (_I, [_I, _P, _P, _I64, _I64, _I64, _P]),
    "wf_sliding_window_stitch": (_I, [_P, _I64, _I64, _P, _P, _P, _P, _I64, _I64, _I64, _I64,
                                      _I64, _I64, _I64, _I64, _P]),
    "wf_tta_merge": (_I, [_P, _P, _I, _P, _I64, _I64, _I64, _I64, _P]),
    "wf_sliding_window_stitch_partial": (_I, [_P, _I64, _I64, _P, _P, _P, _P, _I64, _I64,
                                              _I64, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_sliding_window_normalize": (_I, [_P, _P, _I64, _I64, _I64, _I64, _I64, _P]),
    # training (config 4)
    "wf_window_attention_fwd_train": (_I, [_P, _P, _P, _F, _P, _P, _P, _P, _P, _P, _P, _P,
                                           _I64, _I64, _I64, _I64, _I64, _I64, _I64, _F, _I,
                                           _P]),
    "wf_window_attention_bwd_workspace_bytes": (_I64, [_I64, _I64, _I64, _I64, _I64, _I64,
                                                       _I64]),
    "wf_window_attention_bwd_core": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64,
                                          _I64, _I64, _I64, _I64, _F, _P]),
    "wf_rel_pos_bias_bwd": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _P]),
    "wf_gemm_tn_workspace_bytes": (_I64, [_I64, _I64, _I64]),
    "wf_gemm_tn": (_I, [_P, _I64, _P, _I64, _P, _I64, _I, _P, _I64, _I64, _I64, _P]),
    "wf_colsum_parts": (_I64, [_I64]),
    "wf_colsum": (_I, [_P, _I64, _I64, _P, _I64, _P, _P, _P]),
    "wf_ln_act_fwd": (_I, [_P, _P, _P, _F, _I, _P, _I64, _I64, _P]),
    "wf_ln_bwd_workspace_floats": (_I64, [_I64, _I64]),
    "wf_ln_act_bwd": (_I, [_P, _P, _P, _F, _I, _P, _P, _P, _P, _P, _P, _I64, _I64, _P]),
    "wf_dwt3d_haar_bwd": (_I, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_haar_analysis_ncdhw": (_I, [_P, _I64, _I64, _P, _P, _P, _I64, _I64, _I64, _I64, _I64,
                                    _P]),
    "wf_interp_adjoint_axis": (_I, [_P, _P, _I64, _I64, _I64, _I64, _P, _I64, _P]),
    "wf_interp_adjoint_axis_ac": (_I, [_P, _P, _I64, _I64, _I64, _I64, _P]),
    "wf_dwconv3d_cl": (_I, [_P, _P, _P, _I, _P, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_dwconv_wgrad_ws_floats": (_I64, [_I64] * 5),
    "wf_dwconv3d_wgrad": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_patch_merging_gather": (_I, [_P, _I, _P, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_patch_merging_scatter": (_I, [_P, _I, _P, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_patchify": (_I, [_P, _P, _I, _I64, _I64, _I64, _I64, _I64, _P]),
    "wf_transpose_cs": (_I, [_P, _P, _I64, _I64, _I64, _P]),
}

ABI_VERSION = 18
_lock = threading.Lock()
_lib = None
_err = None


class LibraryMissing(RuntimeError):
    pass


def load(path: str | None = None):
    """Load (once) and return the ctypes library; raises LibraryMissing if unavailable."""
    global _lib, _err
    with _lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            _err = f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            raise LibraryMissing(_err)
        lib = ctypes.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        ver = lib.wf_abi_version()
        if ver != ABI_VERSION:
            raise LibraryMissing(f"{p}: ABI version {ver}, expected {ABI_VERSION} (rebuild)")
        _lib = lib
        return _lib


def call(name: str, *args) -> None:
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.wf_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")


def query(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))
