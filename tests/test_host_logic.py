"""CPU: host-side logic of the product (no kernel launches)."""
import pytest
import torch

import waveformer_amd.network_models as NM
from waveformer_amd import ops
from waveformer_amd.network_models.attention import relative_position_index
from waveformer_amd.network_models.wave_helper import DropPath
from oracle import ref_waveformer as R


@pytest.mark.parametrize("ws", [2, 4, 8])
def test_relative_position_index_equals_oracle(ws):
    assert torch.equal(relative_position_index(ws), R.relative_position_index(ws))


def test_cpu_tensors_fail_loudly():
    x = torch.zeros(1, 4, 4, 4, 8)
    with pytest.raises(RuntimeError, match="GPU only"):
        ops.dwt3d_haar(x)
    blk = NM.Block(8, 1, level=1, img_size=(4, 4, 4)).eval()
    with pytest.raises(RuntimeError, match="GPU only"):
        blk(x)
    enc = NM.MultiscaleTransformer(img_size=(32,) * 3, in_chans=1).eval()
    with torch.no_grad(), pytest.raises(RuntimeError, match="GPU only"):
        enc(torch.zeros(1, 1, 32, 32, 32))


def test_training_path_has_no_cpu_fallback():
    """Under autograd the modules take the HIP training Functions; on CPU tensors they raise
    instead of computing anything on the host."""
    enc = NM.MultiscaleTransformer(img_size=(32,) * 3, in_chans=1)
    with pytest.raises(RuntimeError, match="GPU"):
        enc(torch.zeros(1, 1, 32, 32, 32))


def test_droppath_scale_semantics():
    dp = DropPath(0.25)
    dp.eval()
    assert dp.sample_scale(8, "cpu") is None
    dp.train()
    torch.manual_seed(0)
    s = dp.sample_scale(10000, "cpu")
    vals = s.unique()
    assert vals.numel() == 2 and vals[0] == 0 and abs(vals[1].item() - 1 / 0.75) < 1e-6
    assert abs((s > 0).float().mean().item() - 0.75) < 0.02


def test_block_window_partition_matches_reference_layout():
    blk = NM.Block(8, 1, level=0, img_size=(4, 4, 4))
    x = torch.randn(2, 4, 4, 4, 8)
    assert torch.equal(blk.window_partition(x, 2), R.window_partition(x, 2))


def test_unsupported_wavelet_is_refused():
    wt = NM.WaveletTransform3D(wavelet="db2")
    with pytest.raises(NotImplementedError):
        wt._check()


def test_dicece_loss_vs_reference_monai():
    """waveformer_amd.losses.DiceCELoss against the reference trainer's MONAI DiceCELoss
    (3_train.py:72), value and logits gradient (fixtures from gen_reference_fixtures.py
    --groups loss)."""
    import torch
    from oracle.weight_rule import seeded_randn
    from tests import cases as C
    from waveformer_amd.losses import DiceCELoss
    logits = seeded_randn((2, 4, 8, 8, 8), 30).requires_grad_(True)
    lab = C.g("dicece__labels").long()
    loss = DiceCELoss(to_onehot_y=True, softmax=True)(logits, lab)
    loss.backward()
    assert abs(loss.item() - C.g("dicece__loss").item()) <= 1e-6
    assert C.rel_l2(logits.grad, C.g("dicece__grad")) <= 1e-6
