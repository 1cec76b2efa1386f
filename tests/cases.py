"""Shared parity cases: how to build each module (product side), its rule weights, its seeded
input, the oracle call that restates it, and the golden fixture keys that pin it.

Every case mirrors one block of tests/golden/gen_reference_fixtures.py (same constructor
arguments, seeds and names), so `golden(name)` is what the REFERENCE produced for it.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from functools import partial
from typing import Callable, Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn

from oracle import ref_waveformer as R
from oracle.weight_rule import rule_state_dict, seeded_randn

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN_PATH = os.path.join(HERE, "golden", "ref_fixtures.npz")
PYWT_PATH = os.path.join(HERE, "golden", "pywt_dwt3.npz")
_golden = None


def golden() -> np.lib.npyio.NpzFile:
    global _golden
    if _golden is None:
        _golden = np.load(GOLDEN_PATH)
    return _golden


def g(key: str) -> torch.Tensor:
    return torch.from_numpy(np.array(golden()[key]))


def golden_keys(prefix: str) -> List[str]:
    return [k for k in golden().files if k == prefix or k.startswith(prefix + "_hf")]


def statedict_spec(tag: str):
    return json.loads(bytes(golden()[tag + "__keys"]).decode())


def rel_l2(a: torch.Tensor, b: torch.Tensor) -> float:
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def summary(t: torch.Tensor, nsample: int = 4096, seed: int = 777):
    """Same reduction as gen_reference_fixtures._summary."""
    t = t.detach().contiguous().float().cpu()
    flat = t.reshape(-1).double()
    r = seeded_randn(t.shape, seed).reshape(-1).double()
    stride = max(1, flat.numel() // nsample)
    return (np.array([flat.sum().item(), (flat * flat).sum().item(), (flat * r).sum().item()]),
            t.reshape(-1)[::stride][:nsample])


def dice(a: torch.Tensor, b: torch.Tensor) -> float:
    """light_training/evaluation/metric.py:105-120 semantics: 2|A^B| / (|A|+|B|), 1 if both empty."""
    a = a.bool()
    b = b.bool()
    s = a.sum().item() + b.sum().item()
    if s == 0:
        return 1.0
    return 2.0 * (a & b).sum().item() / s


def brats_regions(labels: torch.Tensor):
    """TC / WT / ET masks from label maps (BraTSTrainer.convert_labels, 3_train.py:104-112:
    TC = {1,3}, WT = {1,2,3}, ET = {3})."""
    return ((labels == 1) | (labels == 3), labels > 0, labels == 3)


@dataclass
class Case:
    name: str
    ctor: Callable[[], nn.Module]
    input_shape: tuple
    seed: int
    oracle: Callable  # (sd, x) -> output (tensor | tuple)
    kind: str = "tensor"  # tensor | block | encoder | summary_encoder | full | labels


def _ln6():
    return partial(nn.LayerNorm, eps=1e-6)


def cases() -> Dict[str, Case]:
    import waveformer_amd.network_models as NM
    c = {}
    for name, dim, heads, ws, B_ in (("attn_ws8", 48, 3, 8, 1), ("attn_ws2_h1", 48, 1, 2, 4),
                                     ("attn_ws4_h2", 32, 2, 4, 3)):
        c[name] = Case(name, partial(NM.Attention, dim, num_heads=heads, qkv_bias=True,
                                     window_size=ws), (B_, ws ** 3, dim), 11,
                       partial(lambda sd, x, h, w: R.attention(sd, "", x, h, w), h=heads, w=ws))
    for name, dim, heads, level, img, ms, B in (
            ("block_l3", 32, 2, 3, 16, True, 1), ("block_l1", 32, 2, 1, 16, True, 1),
            ("block_l0", 32, 2, 0, 8, True, 2), ("block_ss_l2", 32, 2, 2, 16, False, 1)):
        c[name] = Case(name, partial(NM.Block, dim, heads, qkv_bias=True, norm_layer=_ln6(),
                                     level=level, ms_attention=ms, img_size=(img,) * 3),
                       (B, img, img, img, dim), 13,
                       partial(lambda sd, x, h, l, i, m: R.block(sd, "", x, h, l, (i,) * 3, m),
                               h=heads, l=level, i=img, m=ms), "block")
    c["merge"] = Case("merge", partial(NM.PatchMerging, 32, norm_layer=_ln6()), (2, 8, 8, 8, 32),
                      14, lambda sd, x: R.patch_merging(sd, "", x))
    c["ccf_ffn"] = Case("ccf_ffn", partial(NM.CCF_FFN, 32, 128, img_size=(8, 8, 8)),
                        (2, 8, 8, 8, 32), 15, lambda sd, x: R.ccf_ffn(sd, "", x))
    c["enc32"] = Case("enc32", partial(NM.MultiscaleTransformer, img_size=(32,) * 3, in_chans=1,
                                       num_heads=[1, 1, 1, 1], qkv_bias=True, norm_layer=_ln6()),
                      (1, 1, 32, 32, 32), 21,
                      lambda sd, x: R.encoder(sd, x, heads=[1, 1, 1, 1], depths=[2, 2, 2, 2]),
                      "encoder")
    c["full32"] = Case("full32", partial(NM.Waveformer, img_size=(32,) * 3, in_chans=4,
                                         out_chans=4, depths=[2, 2, 2, 2],
                                         feat_size=[48, 96, 192, 384], num_heads=[3, 6, 12, 24]),
                       (1, 4, 32, 32, 32), 22,
                       lambda sd, x: R.waveformer(sd, x, heads=[3, 6, 12, 24], depths=[2] * 4),
                       "full")
    c["full32hf"] = Case("full32hf", partial(NM.Waveformer, img_size=(32,) * 3, in_chans=4,
                                             out_chans=4,
                                             network_config={"transformer": {"hf_refinement": True}}),
                         (1, 4, 32, 32, 32), 23,
                         lambda sd, x: R.waveformer(sd, x, heads=[3, 6, 12, 24], depths=[2] * 4,
                                                    hf_refine=True),
                         "full")
    c["enc128"] = Case("enc128", partial(NM.MultiscaleTransformer, img_size=(128,) * 3,
                                         in_chans=4, qkv_bias=True, norm_layer=_ln6()),
                       (1, 4, 128, 128, 128), 0,
                       lambda sd, x: R.encoder(sd, x, heads=[3, 6, 12, 24], depths=[2] * 4),
                       "summary_encoder")
    c["full128"] = Case("full128", partial(NM.Waveformer, img_size=(128,) * 3, in_chans=4,
                                           out_chans=4, depths=[2, 2, 2, 2],
                                           feat_size=[48, 96, 192, 384],
                                           num_heads=[3, 6, 12, 24]),
                        (1, 4, 128, 128, 128), 0,
                        lambda sd, x: R.waveformer(sd, x, heads=[3, 6, 12, 24], depths=[2] * 4),
                        "labels")
    # config 5: 192^3 x 4 crops, window 12 (N = 1728), HF refinement branch on
    c["enc192"] = Case("enc192", partial(NM.MultiscaleTransformer, img_size=(192,) * 3,
                                         in_chans=4, qkv_bias=True, norm_layer=_ln6()),
                       (1, 4, 192, 192, 192), 5,
                       lambda sd, x: R.encoder(sd, x, heads=[3, 6, 12, 24], depths=[2] * 4),
                       "summary_encoder")
    c["full192hf"] = Case("full192hf", partial(NM.Waveformer, img_size=(192,) * 3, in_chans=4,
                                               out_chans=4,
                                               network_config={"transformer": {"hf_refinement": True}}),
                          (1, 4, 192, 192, 192), 5,
                          lambda sd, x: R.waveformer(sd, x, heads=[3, 6, 12, 24], depths=[2] * 4,
                                                     hf_refine=True),
                          "labels")
    return c


def build(case: Case, device="cpu"):
    """Product module with rule weights (eval) + the rule state_dict for the oracle."""
    m = case.ctor()
    sd = rule_state_dict(m.state_dict())
    m.load_state_dict(sd, strict=True)
    m.eval()
    return m.to(device), sd


def case_input(case: Case) -> torch.Tensor:
    return seeded_randn(case.input_shape, case.seed)


def flatten_output(case: Case, out) -> Dict[str, torch.Tensor]:
    """Map a module/oracle output onto the golden fixture keys of the case."""
    n = case.name
    res: Dict[str, torch.Tensor] = {}
    if case.kind in ("tensor", "full", "labels"):
        res[n] = out
    elif case.kind == "block":
        if isinstance(out, tuple):
            res[n] = out[0]
            for li, d in enumerate(out[1]):
                for k, v in d.items():
                    res[f"{n}_hf_{li}_{k}"] = v
        else:
            res[n] = out
    elif case.kind in ("encoder", "summary_encoder"):
        outs, hfs = out
        for i, o in enumerate(outs):
            res[f"{n}_out{i}"] = o
        for s, h in enumerate(hfs):
            for li, d in enumerate(h):
                for k, v in d.items():
                    res[f"{n}_hf{s}_{li}_{k}"] = v
    return res


# ------------------------------------------------------------------------------------------
# gradient cases (config 4's backward; tests/golden/gen_reference_fixtures.py::_grads)
# ------------------------------------------------------------------------------------------
def grad_loss(outs):
    """sum_k <out_k, R_k>, R_k = seeded_randn(out_k.shape, 900 + k) -- the generator's loss."""
    tot = 0.0
    for k, t in enumerate(outs):
        r = seeded_randn(tuple(t.shape), 900 + k).to(t.device)
        tot = tot + (t * r).sum()
    return tot


def flat_outputs(r):
    """The generator's flat_outputs: main output, then detail tensors (level-major, key order)."""
    if isinstance(r, torch.Tensor):
        return [r]
    a, b = r
    if isinstance(a, torch.Tensor):
        return [a] + [d[k] for d in b for k in sorted(d)]
    return list(a) + [d[k] for h in b for d in h for k in sorted(d)]


@dataclass
class GradCase:
    name: str
    ctor: Callable[[], nn.Module]
    input_shape: tuple
    seed: int
    oracle: Callable  # (sd, x) -> output
    full: bool        # every parameter gradient stored in full (else a summary triple)


def grad_cases() -> Dict[str, GradCase]:
    import waveformer_amd.network_models as NM
    base = cases()
    c: Dict[str, GradCase] = {}
    for n in ("attn_ws8", "attn_ws4_h2", "block_l3", "block_l1", "block_l0", "block_ss_l2",
              "merge", "ccf_ffn"):
        k = base[n]
        c[n] = GradCase(n, k.ctor, k.input_shape, k.seed, k.oracle, True)
    c["enc32h"] = GradCase("enc32h", partial(NM.MultiscaleTransformer, img_size=(32,) * 3,
                                             in_chans=4, qkv_bias=True, norm_layer=_ln6()),
                           (1, 4, 32, 32, 32), 24,
                           lambda sd, x: R.encoder(sd, x, heads=[3, 6, 12, 24], depths=[2] * 4),
                           False)
    k = base["full32"]
    c["full32"] = GradCase("full32", k.ctor, k.input_shape, k.seed, k.oracle, False)
    return c


def grad_summary(gr: torch.Tensor) -> torch.Tensor:
    g = gr.detach().double().cpu().reshape(-1)
    r = seeded_randn(tuple(gr.shape), 777).double().reshape(-1)
    return torch.tensor([g.sum().item(), (g * g).sum().item(), (g * r).sum().item()],
                        dtype=torch.float64)


def oracle_grads(case: GradCase, sd, x):
    """d grad_loss / d (x, every floating state_dict entry) through the oracle on the CPU."""
    sdg = {k: (v.detach().clone().requires_grad_(True) if v.is_floating_point() else v)
           for k, v in sd.items()}
    xg = x.detach().clone().requires_grad_(True)
    grad_loss(flat_outputs(case.oracle(sdg, xg))).backward()
    res = {"x": xg.grad}
    for k, v in sdg.items():
        if v.is_floating_point() and v.grad is not None:
            res[k] = v.grad
    return res
