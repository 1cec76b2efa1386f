"""GPU parity of the general-wavelet kernels (csrc/wavelet.hip; config 5, db1..db4, mode 'zero').

Against PyWavelets' own golden vectors (tests/golden/pywt_dwt3.npz, gen_pywt_vectors.py: Haar,
db2, db3, db4, 1-3 levels, odd sizes) and against the oracle (pinned to the same vectors) on
larger seeded inputs, including non-contiguous detail views and the decoder's concatenation
buffer as the output.  The kernels compute in fp32 (the reference's dtype); tolerance
max |err| <= 2e-6 * max(1, max |ref|) against the float64 golden vectors, rel-L2 <= 1e-6
against the fp32 oracle.  Round trip wavedec3 -> waverec3 reproduces the input (orthogonal
filters) to rel-L2 <= 1e-6 when the size survives the levels.
"""
import numpy as np
import pytest
import torch

from oracle import ref_waveformer as R
from oracle.weight_rule import seeded_randn
from tests import cases as C

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from waveformer_amd import _lib
    _lib.load()
    yield


def _close(got, want):
    want = np.asarray(want)
    got = got.detach().cpu().double().numpy()
    assert got.shape == want.shape
    tol = 2e-6 * max(1.0, float(np.abs(want).max()))
    err = float(np.abs(got - want).max())
    assert err <= tol, (err, tol)


def test_pywt_vectors_on_gpu():
    from waveformer_amd import ops
    z = np.load(C.PYWT_PATH)
    ncase = len([k for k in z.files if k.endswith("_meta")])
    for ci in range(ncase):
        x = torch.from_numpy(z[f"c{ci}_x"]).float().cuda()
        wav = bytes(z[f"c{ci}_wavelet"]).decode()
        for L in range(1, int(z[f"c{ci}_meta"][0]) + 1):
            co = ops.wavedec3(x, wav, L)
            _close(co[0], z[f"c{ci}_L{L}_ll"])
            for li, d in enumerate(co[1:]):
                for k in R.DETAIL_KEYS:
                    _close(d[k], z[f"c{ci}_L{L}_d{li}_{k}"])
            # reconstruct from the float64 golden coefficients (isolates the synthesis)
            gco = [torch.from_numpy(z[f"c{ci}_L{L}_ll"]).float().cuda()] + [
                {k: torch.from_numpy(z[f"c{ci}_L{L}_d{li}_{k}"]).float().cuda()
                 for k in R.DETAIL_KEYS} for li in range(L)]
            _close(ops.waverec3(gco, wav), z[f"c{ci}_L{L}_rec"])


@pytest.mark.parametrize("wav,shape,levels", [
    ("db2", (1, 3, 48, 40, 37), 3),     # config 5's "db2 3-level", odd / ragged sizes
    ("db2", (2, 4, 20, 70, 130), 2),    # several x / y tiles
    ("db1", (1, 2, 33, 17, 9), 3),      # Haar through the general kernel, odd sizes
    ("db3", (1, 2, 25, 26, 27), 2),
    ("db4", (1, 1, 31, 18, 40), 2),
])
def test_wavedec_waverec_vs_oracle(wav, shape, levels):
    from waveformer_amd import ops
    x = seeded_randn(shape, 5) * 2 + 0.3
    ref = R.wavedec3(x, wav, levels)
    got = ops.wavedec3(x.cuda(), wav, levels)
    assert C.rel_l2(got[0], ref[0]) <= 1e-6
    for dg, dr in zip(got[1:], ref[1:]):
        for k in R.DETAIL_KEYS:
            assert tuple(dg[k].shape) == tuple(dr[k].shape)
            assert C.rel_l2(dg[k], dr[k]) <= 1e-6, k
    rec_ref = R.waverec3(ref, wav)
    rec = ops.waverec3(got, wav)
    assert tuple(rec.shape) == tuple(rec_ref.shape)
    assert C.rel_l2(rec, rec_ref) <= 1e-6
    if tuple(rec.shape[-3:]) == shape[-3:]:
        assert C.rel_l2(rec, x) <= 1e-6


def test_waverec_strided_inputs_into_concat_buffer():
    """Channel-last detail views in, the first C channels of a (B, 2C, ...) buffer out."""
    from waveformer_amd import ops
    B, Cc, n = 2, 5, (9, 7, 12)
    cl = [seeded_randn((B,) + n + (Cc,), 40 + i).cuda() for i in range(8)]
    ll = cl[0].permute(0, 4, 1, 2, 3)
    det = {k: cl[i + 1].permute(0, 4, 1, 2, 3) for i, k in enumerate(R.DETAIL_KEYS)}
    want = R.waverec3([ll.cpu().contiguous(), {k: v.cpu().contiguous() for k, v in det.items()}],
                      "db2")
    O = tuple(2 * s - 2 for s in n)
    buf = torch.full((B, 2 * Cc) + O, 7.0, device="cuda")
    ops.waverec3([ll, det], "db2", out=buf[:, :Cc])
    assert C.rel_l2(buf[:, :Cc], want) <= 1e-6
    assert bool((buf[:, Cc:] == 7.0).all())


def test_modules_db2_forward():
    """WaveletTransform3D(wavelet='db2') and UnetrIDWTBlock(wavelet='db2') forward through the
    product modules (the reference modules' wavelet argument, wave_helper.py:344,
    idwt_upsample.py:66)."""
    import waveformer_amd.network_models as NM
    from waveformer_amd.network_models.idwt_upsample import UnetrIDWTBlock
    x = seeded_randn((1, 4, 21, 16, 19), 9)
    ll, yh = NM.WaveletTransform3D(wavelet="db2")(x.cuda(), 2)
    ref = R.wavedec3(x, "db2", 2)
    assert C.rel_l2(ll, ref[0]) <= 1e-6
    for dg, dr in zip(yh, ref[1:]):
        for k in R.DETAIL_KEYS:
            assert C.rel_l2(dg[k], dr[k]) <= 1e-6
    # the IDWT block: conv_lf_block on the LL-shaped input, synthesis, concat, conv_block
    torch.manual_seed(0)
    blk = UnetrIDWTBlock(3, 8, 4, stage=2, hf_refinement=False, wavelet="db2", kernel_size=3,
                         norm_name="instance", res_block=True).eval().cuda()
    inp = seeded_randn((1, 8) + tuple(ref[0].shape[2:]), 11).cuda()
    hf = tuple({k: v[:, :4].contiguous().cuda() for k, v in d.items()} for d in ref[1:])
    O = tuple(2 * s - 2 for s in hf[-1]["aad"].shape[2:])
    skip = seeded_randn((1, 4) + O, 12).cuda()
    with torch.no_grad():
        out = blk(inp, skip, hf)
        lf = blk.conv_lf_block(inp)
        rec = R.waverec3([lf.cpu()] + [{k: v.cpu() for k, v in d.items()} for d in hf], "db2")
        want = blk.conv_block(torch.cat((rec.cuda(), skip), 1))
    assert C.rel_l2(out, want) <= 1e-5
