"""enc128 outputs vs the reference summaries: per key, the norm ratio and the seeded-dot error
relative to the test bound (tests/test_gpu_parity.py::test_encoder128_vs_reference_summaries),
plus a checksum so two runs (e.g. WF_GEMM_NO_LNW=1) can be compared."""
import math
import sys

import torch

sys.path.insert(0, ".")
from tests import cases as C  # noqa: E402
from waveformer_amd import _lib  # noqa: E402

_lib.load()
case = C.cases()["enc128"]
m, _ = C.build(case, "cuda")
with torch.no_grad():
    outs, hfs = m(C.case_input(case).cuda())
flat = C.flatten_output(case, (outs, hfs))
for k, t in flat.items():
    sums, sample = C.summary(t)
    ref = C.golden()[k + "__sum"]
    tol = 2e-3 if "_hf" in k else 2e-4
    nr = abs(math.sqrt(sums[1]) / math.sqrt(ref[1]) - 1) / tol
    dr = abs(sums[2] - ref[2]) / (10 * tol * math.sqrt(ref[1]))
    sr = C.rel_l2(sample, C.g(k + "__sample")) / tol
    flag = " <-- FAIL" if max(nr, dr, sr) > 1 else ""
    print(f"{k:24s} norm {nr:6.3f} dot {dr:6.3f} sample {sr:6.3f} (fraction of bound) "
          f"sum {float(t.double().sum()):+.6e}{flag}")
