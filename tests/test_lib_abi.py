"""CPU: the C-ABI library loads and exports every entry point include/waveformer_hip.h declares
(no compute is launched -- there is no GPU here)."""
import ctypes
import os
import re

import pytest

from waveformer_amd import _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                      "waveformer_hip.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(wf_\w+)\s*\(", src, re.M)))


def test_header_and_binding_agree():
    syms = declared_symbols()
    assert len(syms) >= 14
    assert sorted(_lib.SIGNATURES) == syms


def test_library_exports_every_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libwaveformer_hip.so is not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), s
    lib = _lib.load()
    assert lib.wf_abi_version() == _lib.ABI_VERSION


def test_shape_errors_are_reported_without_a_gpu():
    # argument validation runs before any HIP call, so it works on a CPU-only host
    lib = _lib.load()
    rc = lib.wf_dwt3d_haar_fwd(None, None, None, 0.0, None, 1, 6, 3, 4, 4, None)
    assert rc < 0
    assert b"even" in lib.wf_last_error() or b"multiple of 4" in lib.wf_last_error()
    with pytest.raises(RuntimeError, match="wf_proj_out_fwd"):
        _lib.call("wf_proj_out_fwd", None, None, 1, 1e-5, 1, 6, 8, None)
    assert _lib.query("wf_window_attention_workspace_bytes", 1, 48, 32, 32, 32, 0) >= 32768 * 48 * 8


def test_round5_entries_validate_on_the_host():
    # the fused up-sample + depthwise conv refuses a tile whose source span exceeds its staging
    # (an x factor below 2: 40 -> 60 columns, the second tile spans 14 > 12 source columns)
    # before any HIP call; likewise the
    # channel-last proj_out and the LL-only DWT on bad channel counts
    fake = 256  # never dereferenced: validation fails first
    with pytest.raises(RuntimeError, match="source span"):
        _lib.call("wf_upsample_dwconv3d_stats_cl", fake, fake, fake, fake, fake,
                  1, 32, 4, 4, 40, 8, 8, 60, 1, None)
    with pytest.raises(RuntimeError, match="multiple of 32"):
        _lib.call("wf_upsample_dwconv3d_stats_cl", fake, fake, fake, fake, fake,
                  1, 48, 4, 4, 4, 8, 8, 8, 1, None)
    with pytest.raises(RuntimeError, match="multiple of 4"):
        _lib.call("wf_proj_out_cl_fwd", fake, fake, 1e-5, 10, 6, None)
    with pytest.raises(RuntimeError, match="PatchEmbed"):
        _lib.call("wf_patch_embed_ll_fwd", fake, fake, fake, fake, fake, fake, 1e-6, fake,
                  1, 4, 96, 8, 8, 8, None)


def test_no_packed_fp32_in_device_code(tmp_path):
    """the library is built without VOP3P packed-FP32 instructions (the gfx950
    hazard behind round 2's stage-2 corruption).  Disassemble every gfx950 code object embedded
    in the shipped .so and fail on any v_pk_{fma,mul,add}_f32, so a build that drops the
    Makefile's device feature flag cannot ship."""
    import glob
    import shutil
    import subprocess
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not available")
    so = tmp_path / "lib.so"
    shutil.copy(_lib.LIB_PATH, so)
    subprocess.run([objdump, "--offloading", str(so)], cwd=tmp_path, check=True,
                   capture_output=True)
    objs = sorted(glob.glob(str(tmp_path / "lib.so.*gfx950*")))
    assert objs, "no gfx950 code object in the library"
    bad = []
    for o in objs:
        dis = subprocess.run([objdump, "-d", o], check=True, capture_output=True, text=True).stdout
        for line in dis.splitlines():
            if re.search(r"\bv_pk_(fma|mul|add)_f32\b", line):
                bad.append(f"{os.path.basename(o)}: {line.strip()}")
    assert not bad, "packed-FP32 instructions in device code:\n" + "\n".join(bad[:20])
