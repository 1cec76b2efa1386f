"""Generate golden fixtures by running the REFERENCE implementation itself (CPU, fp32).

    python tests/golden/gen_reference_fixtures.py [--reference /root/reference]

Imports mahfuzalhasan/WaveFormer's `network_models` from the read-only reference checkout
with stand-ins for its four absent third-party imports:
  * torchinfo.summary, ptflops.get_model_complexity_info -- imported but never called;
  * timm.models.layers.{DropPath, to_2tuple, trunc_normal_} -- init helpers + DropPath
    (identity in eval; every fixture runs in eval mode with rule weights);
  * ptwt.{wavedec3, waverec3} -- the repo's wavelet restatement (oracle.ref_waveformer),
    itself pinned to PyWavelets by tests/golden/pywt_dwt3.npz.
Every floating parameter is overwritten by oracle.weight_rule (keyed by state_dict name) and
inputs come from seeded CPU generators, so tests can rebuild the exact same weights/inputs.
Writes tests/golden/ref_fixtures.npz.  Nothing here runs on the GPU box.
"""
from __future__ import annotations

import argparse
import os
import sys
import time
import types
from functools import partial

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import ref_waveformer as R  # noqa: E402
from oracle.weight_rule import apply_rule, seeded_randn  # noqa: E402

# ------------------------------------------------------------------------- stand-ins
def _install_standins():
    ptwt = types.ModuleType("ptwt")

    def wavedec3(data, wavelet, mode="zero", level=None):
        assert mode == "zero"
        return R.wavedec3(data, str(wavelet), level or 1)

    def waverec3(coeffs, wavelet):
        return R.waverec3(coeffs, str(wavelet))

    ptwt.wavedec3, ptwt.waverec3 = wavedec3, waverec3
    sys.modules["ptwt"] = ptwt

    class DropPath(nn.Module):
        def __init__(self, drop_prob=0.0):
            super().__init__()
            self.drop_prob = drop_prob

        def forward(self, x):
            if self.drop_prob == 0.0 or not self.training:
                return x
            keep = 1 - self.drop_prob
            mask = x.new_empty((x.shape[0],) + (1,) * (x.ndim - 1)).bernoulli_(keep)
            return x * mask / keep

    timm = types.ModuleType("timm")
    models = types.ModuleType("timm.models")
    layers = types.ModuleType("timm.models.layers")
    layers.DropPath = DropPath
    layers.to_2tuple = lambda v: tuple(v) if isinstance(v, (tuple, list)) else (v, v)
    layers.trunc_normal_ = nn.init.trunc_normal_
    timm.models, models.layers = models, layers
    sys.modules.update({"timm": timm, "timm.models": models, "timm.models.layers": layers})

    ti = types.ModuleType("torchinfo")
    ti.summary = lambda *a, **k: None
    pf = types.ModuleType("ptflops")
    pf.get_model_complexity_info = lambda *a, **k: (None, None)
    sys.modules.update({"torchinfo": ti, "ptflops": pf})


def _summary(prefix, t, out, nsample=4096, seed=777):
    t = t.detach().contiguous().float()
    flat = t.reshape(-1).double()
    r = seeded_randn(t.shape, seed).reshape(-1).double()
    out[prefix + "__shape"] = np.array(t.shape, dtype=np.int64)
    out[prefix + "__sum"] = np.array([flat.sum().item(), (flat * flat).sum().item(),
                                      (flat * r).sum().item()])
    stride = max(1, flat.numel() // nsample)
    out[prefix + "__sample"] = t.reshape(-1)[::stride][:nsample].numpy()


def _full(prefix, t, out):
    out[prefix] = t.detach().contiguous().float().numpy()


def _hfs(prefix, hfs, out, full=True):
    for li, d in enumerate(hfs):
        for k, v in d.items():
            (_full if full else _summary)(f"{prefix}_{li}_{k}", v, out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--skip-128", action="store_true")
    ap.add_argument("--groups", default="small,128",
                    help="comma list of: small, grad, loss, 128, hf32, 192.  Arrays of groups not listed "
                         "are kept from the existing ref_fixtures.npz")
    args = ap.parse_args()
    groups = set(args.groups.split(","))
    if args.skip_128:
        groups.discard("128")
    sys.dont_write_bytecode = True
    _install_standins()
    sys.path.insert(0, args.reference)
    from network_models import Attention, Block, CCF_FFN, MultiscaleTransformer, PatchMerging, Waveformer  # noqa

    torch.set_num_threads(8)
    torch.set_grad_enabled(False)
    ln6 = partial(nn.LayerNorm, eps=1e-6)
    dst = os.path.join(HERE, "ref_fixtures.npz")
    out = dict(np.load(dst)) if os.path.exists(dst) else {}
    t0 = time.time()
    if "small" in groups:
        _small(out, ln6, Attention, Block, CCF_FFN, MultiscaleTransformer, PatchMerging,
               Waveformer)
    if "hf32" in groups:
        # full model with the high-frequency refinement branch (idwt_upsample.py:39-50, 96-105)
        net = apply_rule(Waveformer(img_size=(32,) * 3, in_chans=4, out_chans=4,
                                    network_config={"transformer": {"hf_refinement": True}})).eval()
        _full("full32hf", net(seeded_randn((1, 4, 32, 32, 32), 23)), out)
    if "grad" in groups:
        with torch.enable_grad():
            _grads(out, ln6, Attention, Block, CCF_FFN, MultiscaleTransformer, PatchMerging,
                   Waveformer)
    if "loss" in groups:
        # 3_train.py:72 DiceCELoss(to_onehot_y=True, softmax=True) (vendored MONAI): value and
        # logits gradient on a seeded (2, 4, 8, 8, 8) batch
        from monai.losses import DiceCELoss
        with torch.enable_grad():
            logits = seeded_randn((2, 4, 8, 8, 8), 30).requires_grad_(True)
            lab = torch.randint(0, 4, (2, 1, 8, 8, 8), generator=torch.Generator().manual_seed(31))
            loss = DiceCELoss(to_onehot_y=True, softmax=True)(logits, lab)
            loss.backward()
        out["dicece__labels"] = lab.to(torch.uint8).numpy()
        out["dicece__loss"] = np.array([loss.item()])
        out["dicece__grad"] = logits.grad.numpy()
    if "128" in groups:
        _big128(out, ln6, MultiscaleTransformer, Waveformer)
    if "192" in groups:
        # config 5: 192^3 x 4 (window 12, N = 1728) encoder summaries and the full model with
        # the HF refinement branch -> labels for the Dice check
        x192 = seeded_randn((1, 4, 192, 192, 192), 5)
        enc = apply_rule(MultiscaleTransformer(img_size=(192,) * 3, in_chans=4, qkv_bias=True,
                                               norm_layer=ln6)).eval()
        t1 = time.time()
        outs, hfs = enc(x192)
        print(f"enc192 {time.time() - t1:.1f}s")
        for i, o in enumerate(outs):
            _summary(f"enc192_out{i}", o, out)
        del enc, outs, hfs
        net = apply_rule(Waveformer(img_size=(192,) * 3, in_chans=4, out_chans=4,
                                    network_config={"transformer": {"hf_refinement": True}})).eval()
        t1 = time.time()
        logits = net(x192)
        print(f"full192hf {time.time() - t1:.1f}s")
        _summary("full192hf", logits, out)
        out["full192hf_labels"] = logits.argmax(1).to(torch.uint8).numpy()

    np.savez_compressed(dst, **out)
    print("wrote", len(out), "arrays in", f"{time.time() - t0:.1f}s")


def _small(out, ln6, Attention, Block, CCF_FFN, MultiscaleTransformer, PatchMerging, Waveformer):
    t0 = time.time()

    # ---- Attention (attention.py:83-104)
    for name, dim, heads, ws, B_ in (("attn_ws8", 48, 3, 8, 1), ("attn_ws2_h1", 48, 1, 2, 4),
                                     ("attn_ws4_h2", 32, 2, 4, 3)):
        m = apply_rule(Attention(dim, num_heads=heads, qkv_bias=True, window_size=ws)).eval()
        x = seeded_randn((B_, ws ** 3, dim), 11)
        _full(name, m(x), out)
        out[name + "__index"] = m.relative_position_index.numpy().astype(np.int16)

    # ---- Block multi-scale, levels 3 / 1 / 0, single-scale level 2 (wave_helper.py:470-549)
    blocks = [("block_l3", 32, 2, 3, 16, True, 1), ("block_l1", 32, 2, 1, 16, True, 1),
              ("block_l0", 32, 2, 0, 8, True, 2), ("block_ss_l2", 32, 2, 2, 16, False, 1)]
    for name, dim, heads, level, img, ms, B in blocks:
        m = apply_rule(Block(dim, heads, qkv_bias=True, norm_layer=ln6, level=level,
                             ms_attention=ms, img_size=(img,) * 3)).eval()
        x = seeded_randn((B, img, img, img, dim), 13)
        r = m(x)
        if isinstance(r, tuple):
            _full(name, r[0], out)
            _hfs(name + "_hf", r[1], out)
        else:
            _full(name, r, out)

    # ---- PatchMerging (Q3) and bare CCF_FFN
    m = apply_rule(PatchMerging(32, norm_layer=ln6)).eval()
    _full("merge", m(seeded_randn((2, 8, 8, 8, 32), 14)), out)
    m = apply_rule(CCF_FFN(32, 128, img_size=(8, 8, 8))).eval()
    _full("ccf_ffn", m(seeded_randn((2, 8, 8, 8, 32), 15)), out)

    # ---- config 1: encoder at 32^3 x 1, heads [1,1,1,1] (head_dim = C)
    enc = apply_rule(MultiscaleTransformer(img_size=(32, 32, 32), in_chans=1, num_heads=[1, 1, 1, 1],
                                           qkv_bias=True, norm_layer=ln6)).eval()
    outs, hfs = enc(seeded_randn((1, 1, 32, 32, 32), 21))
    for i, o in enumerate(outs):
        _full(f"enc32_out{i}", o, out)
    for s, h in enumerate(hfs):
        _hfs(f"enc32_hf{s}", h, out)

    # ---- full model at 32^3 x 4 (default widths / heads)
    net = apply_rule(Waveformer(img_size=(32, 32, 32), in_chans=4, out_chans=4,
                                depths=[2, 2, 2, 2], feat_size=[48, 96, 192, 384],
                                num_heads=[3, 6, 12, 24])).eval()
    _full("full32", net(seeded_randn((1, 4, 32, 32, 32), 22)), out)
    print(f"small fixtures done in {time.time() - t0:.1f}s")

    # ---- state_dict contract (names, shapes, order; int buffers) of the default model and of
    # the hf_refinement variant
    import json
    for tag, kw in (("sd128", dict(img_size=(128,) * 3, in_chans=4, out_chans=4)),
                    ("sd32hf", dict(img_size=(32,) * 3, in_chans=4, out_chans=4,
                                    network_config={"transformer": {"hf_refinement": True}}))):
        sd = Waveformer(**kw).state_dict()
        spec = [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in sd.items()]
        out[tag + "__keys"] = np.frombuffer(json.dumps(spec).encode(), dtype=np.uint8)



def grad_loss(outs):
    """The scalar every gradient fixture differentiates: sum_k <out_k, R_k>, R_k a seeded
    normal cotangent of out_k's shape (seed 900 + k), outputs in the flattened order of
    flat_outputs()."""
    tot = 0.0
    for k, t in enumerate(outs):
        tot = tot + (t * seeded_randn(tuple(t.shape), 900 + k)).sum()
    return tot


def flat_outputs(r):
    """module output -> list of tensors: the main output, then the detail dicts' tensors
    (level-major, ptwt key order) for Blocks; stage outputs then details for the encoder."""
    if isinstance(r, torch.Tensor):
        return [r]
    a, b = r
    if isinstance(a, torch.Tensor):  # Block: (out, tuple of dicts)
        return [a] + [d[k] for d in b for k in sorted(d)]
    return list(a) + [d[k] for h in b for d in h for k in sorted(d)]  # encoder


def _grads(out, ln6, Attention, Block, CCF_FFN, MultiscaleTransformer, PatchMerging,
           Waveformer):
    """Gradient fixtures (config 4's backward): d grad_loss / d input and / d every parameter
    of the reference modules (eval mode, rule weights).  Small modules keep every gradient;
    full32 keeps the input gradient plus a (sum, sum of squares, seeded dot) triple per
    parameter."""
    t0 = time.time()
    cases = []
    for name, dim, heads, ws, B_ in (("attn_ws8", 48, 3, 8, 1), ("attn_ws4_h2", 32, 2, 4, 3)):
        cases.append((name, Attention(dim, num_heads=heads, qkv_bias=True, window_size=ws),
                      (B_, ws ** 3, dim), 11, True))
    for name, dim, heads, level, img, ms, B in (
            ("block_l3", 32, 2, 3, 16, True, 1), ("block_l1", 32, 2, 1, 16, True, 1),
            ("block_l0", 32, 2, 0, 8, True, 2), ("block_ss_l2", 32, 2, 2, 16, False, 1)):
        cases.append((name, Block(dim, heads, qkv_bias=True, norm_layer=ln6, level=level,
                                  ms_attention=ms, img_size=(img,) * 3),
                      (B, img, img, img, dim), 13, True))
    cases.append(("merge", PatchMerging(32, norm_layer=ln6), (2, 8, 8, 8, 32), 14, True))
    cases.append(("ccf_ffn", CCF_FFN(32, 128, img_size=(8, 8, 8)), (2, 8, 8, 8, 32), 15, True))
    cases.append(("enc32h", MultiscaleTransformer(img_size=(32,) * 3, in_chans=4,
                                                  qkv_bias=True, norm_layer=ln6),
                  (1, 4, 32, 32, 32), 24, False))
    cases.append(("full32", Waveformer(img_size=(32, 32, 32), in_chans=4, out_chans=4,
                                       depths=[2, 2, 2, 2], feat_size=[48, 96, 192, 384],
                                       num_heads=[3, 6, 12, 24]), (1, 4, 32, 32, 32), 22, False))
    for name, m, shape, seed, full in cases:
        m = apply_rule(m).eval()
        x = seeded_randn(shape, seed).requires_grad_(True)
        grad_loss(flat_outputs(m(x))).backward()
        out[f"grad_{name}__x"] = x.grad.numpy()
        for pn, p in m.named_parameters():
            if p.grad is None:
                continue
            if full:
                out[f"grad_{name}__{pn}"] = p.grad.numpy()
            else:
                gg = p.grad.double().reshape(-1)
                r = seeded_randn(tuple(p.shape), 777).double().reshape(-1)
                out[f"grad_{name}__{pn}"] = np.array(
                    [gg.sum().item(), (gg * gg).sum().item(), (gg * r).sum().item()])
    print(f"grad fixtures done in {time.time() - t0:.1f}s")


def _big128(out, ln6, MultiscaleTransformer, Waveformer):
    if True:
        # ---- config 2: encoder at 128^3 x 4 (summaries), full model labels
        x128 = seeded_randn((1, 4, 128, 128, 128), 0)
        enc = apply_rule(MultiscaleTransformer(img_size=(128,) * 3, in_chans=4, qkv_bias=True,
                                               norm_layer=ln6)).eval()
        t1 = time.time()
        outs, hfs = enc(x128)
        print(f"enc128 {time.time() - t1:.1f}s")
        for i, o in enumerate(outs):
            _summary(f"enc128_out{i}", o, out)
        for s, h in enumerate(hfs):
            _hfs(f"enc128_hf{s}", h, out, full=False)
        net = apply_rule(Waveformer(img_size=(128,) * 3, in_chans=4, out_chans=4,
                                    depths=[2, 2, 2, 2], feat_size=[48, 96, 192, 384],
                                    num_heads=[3, 6, 12, 24])).eval()
        t1 = time.time()
        logits = net(x128)
        print(f"full128 {time.time() - t1:.1f}s")
        _summary("full128", logits, out)
        out["full128_labels"] = logits.argmax(1).to(torch.uint8).numpy()


if __name__ == "__main__":
    main()
