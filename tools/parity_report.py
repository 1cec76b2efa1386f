"""Print rel-L2 errors of every parity case (HIP path vs oracle and vs reference golden)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import cases as C  # noqa: E402


def main(names):
    allc = C.cases()
    for name in names or [n for n in allc if n not in ("enc128", "full128")]:
        case = allc[name]
        m, sd = C.build(case, "cuda")
        x = C.case_input(case)
        with torch.no_grad():
            out = m(x.cuda())
            ora = case.oracle(sd, x)
        got, want = C.flatten_output(case, out), C.flatten_output(case, ora)
        for k in sorted(got):
            gk = k if k in C.golden().files else None
            e_g = C.rel_l2(got[k], C.g(gk)) if gk else float("nan")
            print(f"{k:28s} vs_oracle {C.rel_l2(got[k], want[k]):.3e}  vs_ref {e_g:.3e}  "
                  f"absmax {want[k].abs().max().item():.3e}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
