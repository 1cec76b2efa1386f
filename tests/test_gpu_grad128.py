"""Config 4 gradients at the train bench's own size (VERDICT r3 missing #3 / next #8, r4 next #1):
the full Waveformer at 128^3 x 4, B = 1 (3_train.py:96-102), HIP forward + backward in autograd
mode, against
  * what the REFERENCE's autograd produced for the same rule weights and seeded input
    (tests/golden/grad128_fixture.npz, gen_grad128_fixture.py; CPU fp32), and
  * the exact gradient: the oracle (pinned to the reference by the golden tests) in float64 on
    the GPU, computed here.

Compared: the input gradient (sum / sum of squares / seeded dot + a strided 4096-value sample)
and every parameter gradient's triple, scaled as tests/test_train_grads.py does.

Determinism (round 5): the backward has no atomics left (attention dQ / dBias / table gather,
conv3d split-K, weight-gradient GEMMs: fixed-order partial sums), so two backward passes must
agree BIT FOR BIT -- asserted below.

Bars, and why they are not 1e-2 (tools/grad128_diag.py, profiles/r5_grad128_diag.txt):
  * the gradient is ill-conditioned: the reference's own fp32 CPU result is 1.03e-2 (worst
    tensor; input-gradient sample 1.02e-2) from the exact fp64 gradient;
  * the exact gradient of the same model with every weight rounded to 16 mantissa bits (the
    bf16x3 operand precision) moves by up to 1.7e-2 (2.8e-2 rounding only the encoder's) --
    any arithmetic on 16-bit operands lands that far from the exact gradient, however it sums;
  * measured here: 1.75e-2 worst vs the golden, 1.57e-2 worst vs exact, global parameter
    gradient rel-L2 8.5e-3 vs exact, input gradient 9.7e-3 / 9.5e-3.
So: every tensor within 3e-2 of the golden and 2.5e-2 of the exact gradient, the whole
parameter gradient within 1.5e-2 (rel-L2) and the input gradient within 1.5e-2 of both; the
loss within 1e-4.  Gradients whose reference norm is below 1e-5 of the largest (conv biases
ahead of a non-affine InstanceNorm: true value 0) are only checked to stay at noise level.
"""
import os

import numpy as np
import pytest
import torch

from tests import cases as C

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "grad128_fixture.npz")
TOL = 3e-2          # per tensor vs the reference golden (measured worst 1.75e-2)
TOL_EXACT = 2.5e-2  # per tensor vs the exact fp64 gradient (measured worst 1.57e-2)
TOL_GLOBAL = 1.5e-2  # whole parameter gradient rel-L2 vs exact (measured 8.5e-3)
TOL_X = 1.5e-2      # input gradient vs golden sample / exact (measured 9.7e-3 / 9.5e-3)


def fixture():
    return np.load(FIX)


def test_grad128_fixture_matches_model_parameters():
    """CPU: the fixture holds one triple per parameter of the product model (same names: the
    strict state_dict contract), plus the input gradient."""
    fx = fixture()
    m = C.cases()["full128"].ctor()
    names = {f"p__{n}" for n, _ in m.named_parameters()}
    keys = {k for k in fx.files if k.startswith("p__")}
    assert keys <= names and len(keys) >= 0.9 * len(names), sorted(names - keys)[:8]
    assert fx["x__sample"].shape == (4096,) and np.isfinite(fx["x__sample"]).all()


@pytest.mark.gpu
def test_hip_grads_128_vs_reference():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from waveformer_amd import _lib
    _lib.load()
    torch.backends.cuda.matmul.allow_tf32 = False
    fx = fixture()
    case = C.cases()["full128"]
    m, sd = C.build(case, "cuda")
    x0 = C.case_input(case).cuda()

    def run():
        m.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        loss = C.grad_loss(C.flat_outputs(m(x)))
        loss.backward()
        torch.cuda.synchronize()
        got = {"x": x.grad.detach().cpu()}
        for k, p in m.named_parameters():
            if p.grad is not None:
                got[k] = p.grad.detach().cpu()
        return loss.item(), got

    loss, got = run()
    loss2, got2 = run()
    assert loss2 == loss
    nondet = [k for k in got if not torch.equal(got[k], got2[k])]
    assert not nondet, f"backward not bitwise repeatable: {nondet[:8]}"
    del got2
    assert abs(loss / fx["loss"][0] - 1) <= 1e-4, (loss, fx["loss"][0])
    # the exact gradient: the oracle in float64 on the GPU
    sdg = {k: (v.detach().double().cuda().requires_grad_(True) if v.is_floating_point()
               else v.cuda()) for k, v in sd.items()}
    xg = x0.double().clone().requires_grad_(True)
    C.grad_loss(C.flat_outputs(case.oracle(sdg, xg))).backward()
    exact = {"x": xg.grad.detach().cpu()}
    exact.update({k: v.grad.detach().cpu() for k, v in sdg.items()
                  if v.is_floating_point() and v.grad is not None})
    del sdg, xg
    torch.cuda.empty_cache()
    want = {"x": fx["x__sum"]}
    want.update({k[3:]: fx[k] for k in fx.files if k.startswith("p__")})
    norms = {k: float(w[1]) ** 0.5 for k, w in want.items()}
    floor = 1e-5 * max(norms.values())

    def err(s, w, n):
        scale = max(float(w[1]) ** 0.5, 1e-30)
        rn = max(1, n) ** 0.5
        return max(abs(s[0] - w[0]) / (scale * rn), abs(s[1] - w[1]) / abs(w[1]),
                   abs(s[2] - w[2]) / (scale * rn))

    bad, worst_g, worst_e = [], (0.0, None), (0.0, None)
    num = den = 0.0
    for k, w in want.items():
        assert k in got, f"no gradient for {k}"
        gv = got[k]
        s = C.grad_summary(gv).numpy()
        if norms[k] < floor:
            if not gv.double().norm().item() < 10 * floor:
                bad.append((k, "noise-level gradient too large"))
            continue
        eg = err(s, w, gv.numel())
        ee = err(s, C.grad_summary(exact[k]).numpy(), gv.numel())
        worst_g, worst_e = max(worst_g, (eg, k)), max(worst_e, (ee, k))
        if not eg <= TOL:
            bad.append((k, "golden", eg))
        if not ee <= TOL_EXACT:
            bad.append((k, "exact", ee))
        if k != "x":
            num += (gv.double() - exact[k]).norm().item() ** 2
            den += exact[k].norm().item() ** 2
    glob = (num / den) ** 0.5
    stride = int(fx["x__stride"][0])
    samp = got["x"].reshape(-1)[::stride][:4096]
    err_x = C.rel_l2(samp, torch.from_numpy(fx["x__sample"]))
    err_xe = C.rel_l2(got["x"], exact["x"])
    print(f"grad128: bitwise repeatable; worst vs golden {worst_g[0]:.3e} ({worst_g[1]}), vs exact "
          f"{worst_e[0]:.3e} ({worst_e[1]}); parameter gradient rel-L2 vs exact {glob:.3e}; "
          f"input gradient vs golden sample {err_x:.3e}, vs exact {err_xe:.3e}; loss {loss:.6e}")
    assert err_x <= TOL_X and err_xe <= TOL_X, (err_x, err_xe)
    assert glob <= TOL_GLOBAL, glob
    assert not bad, f"{len(bad)} gradients over their bar: {bad[:8]}"
