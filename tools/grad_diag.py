"""Per-tensor gradient errors of one grad case on the GPU: the product modules and the oracle run
on the GPU (plain torch, fp32, MIOpen convs), both against the reference's golden gradients.
    python tools/grad_diag.py full32"""
import sys

import torch

sys.path.insert(0, ".")
from tests import cases as C  # noqa: E402
from tests.test_train_grads import _golden_grads  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "full32"
torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
from waveformer_amd import _lib  # noqa: E402
_lib.load()
case = C.grad_cases()[name]
m = case.ctor()
sd = C.rule_state_dict(m.state_dict())
m.load_state_dict(sd, strict=True)
m = m.eval().cuda()
x = C.seeded_randn(case.input_shape, case.seed).cuda().requires_grad_(True)
C.grad_loss(C.flat_outputs(m(x))).backward()
got = {"x": x.grad.cpu()}
for k, p in m.named_parameters():
    if p.grad is not None:
        got[k] = p.grad.cpu()
sdg = {k: v.cuda() for k, v in sd.items()}
og = {k: v.cpu() for k, v in C.oracle_grads(case, sdg, x.detach()).items()}
want = _golden_grads(name)


def err(gv, w):
    if w.dim() == 1 and w.numel() == 3 and gv.numel() != 3:
        s = C.grad_summary(gv)
        scale = max(abs(w[1].item()) ** 0.5, 1e-30)
        return max(abs(s[0] - w[0]).item() / (scale * max(1, gv.numel()) ** 0.5),
                   abs(s[1] - w[1]).item() / max(abs(w[1].item()), 1e-30),
                   abs(s[2] - w[2]).item() / (scale * max(1, gv.numel()) ** 0.5))
    return C.rel_l2(gv.reshape(w.shape), w)


rows = []
for k, w in want.items():
    rows.append((k, err(got[k], w) if k in got else float("nan"),
                 err(og[k], w) if k in og else float("nan"),
                 (w[1].item() ** 0.5) if (w.dim() == 1 and w.numel() == 3) else w.double().norm().item()))
print(f"{'tensor':70s} {'product':>10s} {'oracle@gpu':>10s} {'norm':>10s}")
for k, a, b, n in rows:
    print(f"{k:70s} {a:10.2e} {b:10.2e} {n:10.2e}")
