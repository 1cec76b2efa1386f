"""Run-to-run determinism of PatchMerging 1 -> 2 (C = 48) at 64^3: the same call N times, rows
that differ from the first run, and the distance of each run from the fp64 oracle per row.
    WF_MERGE_RES=0|1 python tools/merge_det.py [runs]"""
import sys

import torch

sys.path.insert(0, ".")
from tests import test_gpu_parity as T  # noqa: E402
from tests import cases as C  # noqa: E402
from oracle import ref_waveformer as R  # noqa: E402
from oracle.weight_rule import rule_state_dict, seeded_randn  # noqa: E402
import waveformer_amd.network_models as NM  # noqa: E402
from waveformer_amd import ops  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
m = NM.PatchMerging(48, norm_layer=C._ln6())
sd = rule_state_dict(m.state_dict())
m.load_state_dict(sd)
m = m.cuda()
x = seeded_randn((1, 64, 64, 64, 48), 62) * 1.5 + 0.25
ref = R.patch_merging({k: v.double() for k, v in sd.items()}, "", x.double()).reshape(-1, 96)
xc = x.cuda()
outs = []
with torch.no_grad(), ops.precision("bf16x3"):
    for _ in range(runs):
        outs.append(ops.patch_merging(xc, m.norm, m.reduction).cpu().reshape(-1, 96))
for i, o in enumerate(outs):
    rows = (o != outs[0]).any(-1)
    err = ((o.double() - ref).norm(dim=-1) / ref.norm(dim=-1))
    print(f"run {i}: rows != run 0: {int(rows.sum())}  max row rel err vs fp64 {float(err.max()):.3e}"
          f"  mean {float(err.mean()):.3e}")
