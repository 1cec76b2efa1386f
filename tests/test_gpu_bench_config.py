"""Parity of the benched configuration itself (bench.py's default line): the 128^3 x 4 encoder
at B = 8 per GPU, replayed from a HIP graph as bench.py times it.

  * volume 0 is the enc128 input (seed 0, rule weights): every output and high-frequency band
    of it is checked against the REFERENCE's own summaries (tests/golden/ref_fixtures.npz,
    same bars as test_encoder128_vs_reference_summaries: 2e-4, 2e-3 for the detail bands);
  * volumes 1..7 are seeded noise; every volume of the B = 8 graph replay must equal its own
    eager B = 1 forward in FULL (every output tensor and detail band) to rel-L2 <= 1e-6 -- the
    window / batch / stride indexing only B = 8 exercises (B * nW window rows, the 1.6 GB
    FFN workspaces, the 8-volume grids) against the path the golden tests pin.
"""
import math

import pytest
import torch

from oracle.weight_rule import seeded_randn
from tests import cases as C

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from waveformer_amd import _lib
    _lib.load()
    yield


def _flat(case, out):
    return C.flatten_output(case, out)


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def test_encoder128_b8_graph_replay_vs_b1_and_reference():
    case = C.cases()["enc128"]
    m, _ = C.build(case, "cuda")
    B = 8
    x = torch.cat([C.case_input(case), seeded_randn((B - 1, 4, 128, 128, 128), 4242)]).cuda()

    def step():
        with torch.no_grad():
            return m(x)

    step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        static = step()
    for t in _flat(case, static).values():  # the replays below must recompute every output
        t.zero_()
    graph.replay()
    graph.replay()
    torch.cuda.synchronize()
    got = _flat(case, static)

    # volume 0 against the reference's summaries of enc128
    for k, t in got.items():
        v0 = t[0:1]
        assert tuple(v0.shape) == tuple(C.golden()[k + "__shape"]), k
        sums, sample = C.summary(v0)
        ref = C.golden()[k + "__sum"]
        tol = 2e-3 if "_hf" in k else 2e-4
        assert abs(math.sqrt(sums[1]) / math.sqrt(ref[1]) - 1) <= tol, k
        assert abs(sums[2] - ref[2]) <= 10 * tol * math.sqrt(ref[1]), k
        assert C.rel_l2(sample, C.g(k + "__sample")) <= tol, k

    # the graph replay against a second, eager B = 8 forward: bit-identical (same kernels, same
    # launch shapes); on a mismatch the message names the tensor and the differing region, so
    # the failing run itself says which side and where
    with torch.no_grad():
        eager = _flat(case, m(x))
    for k, t in got.items():
        assert torch.equal(t, eager[k]), f"graph replay vs eager B=8, {k}: {_region(t, eager[k])}"

    # every volume against its own B = 1 eager forward, full tensors
    worst = 0.0
    for b in range(B):
        with torch.no_grad():
            one = _flat(case, m(x[b:b + 1].contiguous()))
        for k, t in got.items():
            e = _rel(t[b:b + 1], one[k])
            worst = max(worst, e)
            assert e <= 1e-6, (b, k, e, _region(t[b:b + 1], one[k]), _region(eager[k][b:b + 1], one[k]))
    print(f"B=8 graph vs B=1 eager: worst rel-L2 {worst:.3e}")


def _region(a, b):
    """Extent of the elements that differ between two (B, C, D, H, W) tensors: samples,
    channel / z / y / x ranges, count, max difference."""
    d = (a.double() - b.double()).abs()
    nz = (d > 0).nonzero()
    if nz.numel() == 0:
        return "identical"
    lo, hi = nz.min(0).values.tolist(), nz.max(0).values.tolist()
    ax = "bczyx" if a.dim() == 5 else "".join(str(i) for i in range(a.dim()))
    ext = ", ".join(f"{n} {l}-{h}" for n, l, h in zip(ax, lo, hi))
    return f"{nz.shape[0]} elements, {ext}, max {d.max().item():.3e}"
