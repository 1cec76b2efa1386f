"""Print the measured rel-L2 (vs the reference's golden outputs) of every module case and the
full-model Dice at 128^3 / 192^3 for one precision -- the numbers the test bounds are set from.
usage: python tools/prec_errs.py fp16"""
import sys

import torch

sys.path.insert(0, ".")
from tests import cases as C  # noqa: E402
from waveformer_amd import _lib, ops  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp16"
_lib.load()
for name in ["attn_ws8", "attn_ws2_h1", "attn_ws4_h2", "merge", "ccf_ffn", "block_l3", "block_l1",
             "block_l0", "block_ss_l2", "enc32", "full32", "full32hf"]:
    case = C.cases()[name]
    m, sd = C.build(case, "cuda")
    with torch.no_grad(), ops.precision(prec):
        out = m(C.case_input(case).cuda())
    got = C.flatten_output(case, out)
    worst = max((C.rel_l2(got[k], C.g(k)), k) for k in got)
    print(f"{prec} {name:12s} {case.kind:8s} worst rel-L2 {worst[0]:.3e} ({worst[1]})", flush=True)
for name, key in (("full128", "full128_labels"), ("full192hf", "full192hf_labels")):
    case = C.cases()[name]
    m, _ = C.build(case, "cuda")
    with torch.no_grad(), ops.precision(prec):
        lab = m(C.case_input(case).cuda()).argmax(1).cpu()
    ref = C.g(key).long()
    d = [C.dice(a, b) for a, b in zip(C.brats_regions(lab), C.brats_regions(ref))]
    print(f"{prec} {name} Dice TC/WT/ET {d}", flush=True)
    del m
    torch.cuda.empty_cache()
