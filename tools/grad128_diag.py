"""Config-4 gradient diagnostics at 128^3 x 4: how much of the HIP backward's
distance from the reference's CPU fp32 gradients (tests/golden/grad128_fixture.npz) is run-to-run
spread and how much is systematic.

  * P1, P2: the HIP forward + backward (autograd mode, bf16x3 forward) run twice on the same
    weights and input -- their distance is the run-to-run spread;
  * O64: the oracle (oracle/ref_waveformer.py) in float64 on the GPU -- the rounding-free
    gradient both fp32 computations approximate;
  * G: the reference's own CPU fp32 gradients (summaries).

Per tensor the error is the test's metric (tests/test_gpu_grad128.py).  Prints the worst tensors
and the column maxima; --json writes every row.
    python tools/grad128_diag.py [--no-oracle] [--json out.json]
"""
import argparse
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests import cases as C  # noqa: E402
from tests.test_gpu_grad128 import fixture  # noqa: E402


def summ(t: torch.Tensor) -> np.ndarray:
    return C.grad_summary(t).numpy()


def err(s, w, n):
    """test_gpu_grad128's metric: summary s against reference summary w of an n-element tensor."""
    scale = max(float(w[1]) ** 0.5, 1e-30)
    rn = max(1, n) ** 0.5
    return max(abs(s[0] - w[0]) / (scale * rn), abs(s[1] - w[1]) / max(abs(w[1]), 1e-300),
               abs(s[2] - w[2]) / (scale * rn))


def product_run(m, x0):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--json", default=None)
    ap.add_argument("--round-weights", action="store_true",
                    help="also run the fp64 oracle with every weight rounded to a bf16 hi + lo "
                         "pair (16 mantissa bits): the gradients' sensitivity to bf16x3 operands")
    ap.add_argument("--round-scope", default="all", choices=["all", "encoder", "decoder"],
                    help="which weights --round-weights rounds")
    args = ap.parse_args()
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    from waveformer_amd import _lib
    _lib.load()
    fx = fixture()
    case = C.cases()["full128"]
    m, sd = C.build(case, "cuda")
    x0 = C.case_input(case).cuda()
    runs = []
    for r in range(args.runs):
        loss, got = product_run(m, x0)
        runs.append((loss, {k: (summ(v), v.numel(), v) for k, v in got.items()}))
        print(f"product run {r}: loss {loss:.9e}", flush=True)
    want = {"x": fx["x__sum"]}
    want.update({k[3:]: fx[k] for k in fx.files if k.startswith("p__")})
    stride = int(fx["x__stride"][0])
    o64 = None
    if not args.no_oracle:
        sdg = {k: (v.detach().double().cuda().requires_grad_(True) if v.is_floating_point()
                   else v.cuda()) for k, v in sd.items()}
        xg = x0.double().clone().requires_grad_(True)
        lo = C.grad_loss(C.flat_outputs(case.oracle(sdg, xg)))
        lo.backward()
        torch.cuda.synchronize()
        print(f"oracle fp64 loss {lo.item():.9e}  (reference fp32 CPU {fx['loss'][0]:.9e})",
              flush=True)
        o64 = {"x": xg.grad.detach().cpu()}
        for k, v in sdg.items():
            if v.is_floating_point() and v.grad is not None:
                o64[k] = v.grad.detach().cpu()
        o64 = {k: (summ(v), v.numel(), v) for k, v in o64.items()}
    o64r = None
    if not args.no_oracle and args.round_weights:
        def r16(t):
            hi = t.float().to(torch.bfloat16).float()
            lo = (t.float() - hi).to(torch.bfloat16).float()
            return (hi.double() + lo.double())
        def pick(k):
            enc = k.startswith("waveformer_encoder.")
            return args.round_scope == "all" or (enc == (args.round_scope == "encoder"))
        sdr = {k: ((r16(v) if pick(k) else v.double()).cuda().requires_grad_(True)
                   if v.is_floating_point() else v.cuda()) for k, v in sd.items()}
        xr = x0.double().clone().requires_grad_(True)
        C.grad_loss(C.flat_outputs(case.oracle(sdr, xr))).backward()
        torch.cuda.synchronize()
        o64r = {"x": xr.grad.detach().cpu()}
        for k, v in sdr.items():
            if v.is_floating_point() and v.grad is not None:
                o64r[k] = v.grad.detach().cpu()
        o64r = {k: (summ(v), v.numel(), v) for k, v in o64r.items()}
    rows = []
    norms = {k: float(w[1]) ** 0.5 for k, w in want.items()}
    floor = 1e-5 * max(norms.values())
    for k, w in want.items():
        if norms[k] < floor:
            continue
        s1, n, t1 = runs[0][1][k]
        row = {"tensor": k, "norm": norms[k], "P1_G": err(s1, w, n)}
        if len(runs) > 1:
            s2, _, t2 = runs[1][1][k]
            row["P2_G"] = err(s2, w, n)
            row["P1_P2"] = err(s2, s1, n)
            row["P1_P2_rel_l2"] = C.rel_l2(t2, t1)
        if o64 is not None:
            so, _, to = o64[k]
            row["P1_O64"] = err(s1, so, n)
            row["G_O64"] = err(w, so, n)
            row["P1_O64_rel_l2"] = C.rel_l2(t1, to)
        if o64r is not None:
            row["O64r_O64"] = err(o64r[k][0], o64[k][0], n)
        rows.append(row)
    # input-gradient strided sample
    samp_g = torch.from_numpy(fx["x__sample"])
    xs = {"P1_G": C.rel_l2(runs[0][1]["x"][2].reshape(-1)[::stride][:4096], samp_g)}
    if len(runs) > 1:
        xs["P1_P2"] = C.rel_l2(runs[1][1]["x"][2], runs[0][1]["x"][2])
    if o64 is not None:
        xs["O64_G"] = C.rel_l2(o64["x"][2].reshape(-1)[::stride][:4096].float(), samp_g)
        xs["P1_O64"] = C.rel_l2(runs[0][1]["x"][2], o64["x"][2])
    cols = [c for c in ("P1_G", "P2_G", "P1_P2", "P1_P2_rel_l2", "P1_O64", "G_O64",
                        "P1_O64_rel_l2", "O64r_O64") if c in rows[0]]
    key = "P1_O64" if "P1_O64" in rows[0] else "P1_G"
    rows.sort(key=lambda r: -r[key])
    print(f"{'tensor':66s} " + " ".join(f"{c:>13s}" for c in cols))
    for r in rows[:30]:
        print(f"{r['tensor'][:66]:66s} " + " ".join(f"{r[c]:13.3e}" for c in cols))
    print("max " + " ".join(f"{c}={max(r[c] for r in rows):.3e}" for c in cols))
    print("input-gradient sample rel-L2:", {k: f"{v:.3e}" for k, v in xs.items()})
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"rows": rows, "x": xs, "losses": [r[0] for r in runs]}, f, indent=1)


if __name__ == "__main__":
    main()
