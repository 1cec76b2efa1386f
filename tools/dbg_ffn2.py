"""Determinism / parity of the stage-2 CCF_FFN (C 96, hidden 384) under NaN-filled free memory."""
import sys

import torch

sys.path.insert(0, ".")
import waveformer_amd.network_models as NM  # noqa: E402
from oracle import ref_waveformer as R  # noqa: E402
from oracle.weight_rule import rule_state_dict  # noqa: E402
from waveformer_amd import _lib, ops  # noqa: E402

_lib.load()
torch.manual_seed(0)
for (B, S) in [(1, 32), (2, 16), (1, 16)]:
    mlp = NM.CCF_FFN(96, 384, img_size=(S, S, S))
    sd = rule_state_dict(mlp.state_dict())
    mlp.load_state_dict(sd)
    mlp = mlp.eval().cuda()
    norm2 = torch.nn.LayerNorm(96, eps=1e-6).cuda()
    x = torch.randn(B, S, S, S, 96, device="cuda")
    outs = []
    for it in range(4):
        junk = torch.full((4 * 1024 ** 3 // 4,), float("nan"), device="cuda")
        del junk
        with torch.no_grad():
            st = ops.msfuse([], x, 1e-6)[1]
            outs.append(ops.ccf_ffn(x, st, norm2, mlp))
        torch.cuda.synchronize()
    d = max((o - outs[0]).abs().max().item() for o in outs[1:])
    with torch.no_grad():
        xc = x.cpu()
        n2 = torch.nn.functional.layer_norm(xc, [96], norm2.weight.cpu(), norm2.bias.cpu(), 1e-6)
        ref = xc + R.ccf_ffn(sd, "", n2)
    e = float((outs[0].cpu() - ref).norm() / ref.norm())
    print(f"B={B} S={S}: run-to-run max diff {d:.3e} nan {bool(torch.isnan(outs[0]).any())} "
          f"rel-L2 vs oracle {e:.3e}", flush=True)
