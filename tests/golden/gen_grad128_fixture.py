"""Config 4 gradient parity at its own size (VERDICT r3 missing #3): d grad_loss / d input and
d / d every parameter of the REFERENCE Waveformer at 128^3 x 4, B = 1 (the shape the train bench
steps, 3_train.py:96-102; full model with the MONAI decoder), eval mode, rule weights, seeded
input 0 -- run on the CPU in this container.

    python tests/golden/gen_grad128_fixture.py [--reference /root/reference]

Uses gen_reference_fixtures.py's stand-ins for the reference's absent third-party imports and
its grad_loss (a seeded normal cotangent of the logits, seed 900).  Writes
tests/golden/grad128_fixture.npz: per parameter the (sum, sum of squares, seeded dot) triple of
tests/cases.grad_summary, and for the input gradient the triple plus a strided 4096-value
sample.  Nothing here runs on the GPU box.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
from oracle.weight_rule import apply_rule, seeded_randn  # noqa: E402
import gen_reference_fixtures as G  # noqa: E402

SHAPE = (1, 4, 128, 128, 128)
SEED = 0
NSAMPLE = 4096


def triple(g: torch.Tensor) -> np.ndarray:
    gg = g.detach().double().reshape(-1)
    r = seeded_randn(tuple(g.shape), 777).double().reshape(-1)
    return np.array([gg.sum().item(), (gg * gg).sum().item(), (gg * r).sum().item()])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    sys.dont_write_bytecode = True
    G._install_standins()
    sys.path.insert(0, args.reference)
    from network_models import Waveformer  # noqa

    torch.set_num_threads(8)
    net = apply_rule(Waveformer(img_size=(128,) * 3, in_chans=4, out_chans=4,
                                depths=[2, 2, 2, 2], feat_size=[48, 96, 192, 384],
                                num_heads=[3, 6, 12, 24])).eval()
    x = seeded_randn(SHAPE, SEED).requires_grad_(True)
    t0 = time.time()
    logits = net(x)
    loss = G.grad_loss(G.flat_outputs(logits))
    loss.backward()
    print(f"forward + backward {time.time() - t0:.1f}s, loss {loss.item():.6e}")
    out = {"loss": np.array([loss.item()]), "x__sum": triple(x.grad)}
    stride = x.grad.numel() // NSAMPLE
    out["x__sample"] = x.grad.reshape(-1)[::stride][:NSAMPLE].numpy().copy()
    out["x__stride"] = np.array([stride])
    n = 0
    for pn, p in net.named_parameters():
        if p.grad is not None:
            out[f"p__{pn}"] = triple(p.grad)
            n += 1
    np.savez_compressed(os.path.join(HERE, "grad128_fixture.npz"), **out)
    print(f"{n} parameter gradients")


if __name__ == "__main__":
    main()
