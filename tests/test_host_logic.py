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


def test_precision_scopes_are_thread_local():
    """an op-group override (fp16 policy -> bf16x3 for 'skip_conv') inside one
    thread's forward must not change the precision another thread's forward sees, and
    overlapping scopes of two threads must not restore each other's value."""
    import threading
    default = ops.get_precision()
    inside, outside = threading.Event(), threading.Event()
    seen = {}

    def a():
        with ops.precision("fp16"):
            with ops.op_precision("skip_conv"):
                seen["a_inner"] = ops.get_precision()
                inside.set()
                outside.wait(10)
            seen["a_after"] = ops.get_precision()

    def b():
        inside.wait(10)
        with ops.precision("fp16"):
            seen["b"] = ops.get_precision()
            seen["b_conv"] = ops.op_prec("conv")
        outside.set()

    ta, tb = threading.Thread(target=a), threading.Thread(target=b)
    ta.start(), tb.start()
    ta.join(20), tb.join(20)
    assert seen == {"a_inner": "bf16x3", "b": "fp16", "b_conv": ops.PRECISIONS["fp16"],
                    "a_after": "fp16"}
    assert ops.get_precision() == default
    with ops.precision("fp16"):
        assert ops.op_prec("attn") == ops.PRECISIONS["bf16x3"]
        with ops.op_precision("conv"):
            assert ops.get_precision() == "fp16"
    assert ops.get_precision() == default


def test_index_formula_tracks_in_place_writes():
    """an in-place write to relative_position_index after the formula check must
    turn the in-kernel formula off (the forward then reads the dense bias built from the
    buffer); loading a state_dict re-validates."""
    a = NM.Attention(48, num_heads=3, qkv_bias=True, window_size=4)
    assert a._formula_valid()
    sd = {k: v.clone() for k, v in a.state_dict().items()}
    a.relative_position_index.fill_(0)
    assert not a._formula_valid()
    a.load_state_dict(sd)
    assert a._formula_valid()
    sd["relative_position_index"] = torch.zeros_like(sd["relative_position_index"])
    a.load_state_dict(sd)
    assert not a._formula_valid()


def test_index_formula_survives_device_moves():
    """A module that loaded a state_dict (buffer version > 0) and is then moved (.to / .cuda:
    a fresh copy of the buffer at version 0) keeps the in-kernel formula -- the round-4
    regression where eager fell back to the dense bias after .cuda() while a torch.compile
    trace kept the formula (test_compile_block_fullgraph_matches_eager)."""
    a = NM.Attention(48, num_heads=3, qkv_bias=True, window_size=4)
    a.load_state_dict({k: v.clone() for k, v in a.state_dict().items()})
    assert a.relative_position_index._version > 0 and a._formula_valid()
    a._apply(lambda t: t.clone())  # what Module.to(device) does to every buffer
    assert a.relative_position_index._version == 0
    assert a._formula_valid()
    a.relative_position_index.fill_(0)
    assert not a._formula_valid()


def test_index_formula_rechecked_when_written_before_a_move():
    """an in-place write followed by a device move (or .float(), which keeps the int
    buffer but adopts its bumped version) must not re-enable the in-kernel formula; a move of
    an unwritten buffer, or a write that restores the formula, keeps / regains it."""
    a = NM.Attention(48, num_heads=3, qkv_bias=True, window_size=4)
    a.relative_position_index.fill_(0)
    a._apply(lambda t: t.clone())  # Module.to(device)
    assert not a._formula_valid()
    b = NM.Attention(48, num_heads=3, qkv_bias=True, window_size=4)
    b.relative_position_index.fill_(0)
    b.float()  # the int buffer is returned unchanged
    assert not b._formula_valid()
    c = NM.Attention(48, num_heads=3, qkv_bias=True, window_size=4)
    good = c.relative_position_index.clone()
    c.relative_position_index.fill_(0)
    c.relative_position_index.copy_(good)
    c._apply(lambda t: t.clone())
    assert c._formula_valid()
    c._apply(lambda t: t.clone())
    assert c._formula_valid()
