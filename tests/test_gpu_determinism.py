"""Run-to-run determinism of the encoder forward (the benched path) with the caching
allocator's free memory filled with NaN before every run: a kernel that reads memory it did
not write shows up as NaN, a race as a bitwise difference between runs.  (The encoder's
inference kernels use no atomics; the decoder's split-K convolution and InstanceNorm moments
do, and are not covered here.)"""
import pytest
import torch

from tests import cases as C

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from waveformer_amd import _lib
    _lib.load()
    yield


def _flat(r):
    outs, hfs = r
    return list(outs) + [d[k] for h in hfs for d in h for k in sorted(d)]


@pytest.mark.parametrize("prec", ["bf16x3", "fp16"])
def test_encoder128_bitwise_deterministic_under_nan_filled_memory(prec):
    from waveformer_amd import ops
    case = C.cases()["enc128"]
    m, _ = C.build(case, "cuda")
    x = torch.cat([C.case_input(case)] * 2).cuda()
    runs = []
    for _ in range(3):
        junk = torch.full((3 * 1024 ** 3 // 4,), float("nan"), device="cuda")
        del junk
        with torch.no_grad(), ops.precision(prec):
            runs.append([t.clone() for t in _flat(m(x))])
        torch.cuda.synchronize()
    for t in runs[0]:
        assert not torch.isnan(t).any()
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)


def test_encoder128_independent_of_lds_garbage():
    """A kernel that reads LDS it did not write computes on whatever the previous workgroup on
    that CU left there.  Every library launch of the encoder forward is preceded, on the same
    stream, by NaN-pattern LDS-poisoning workgroups of several sizes (wf_debug_poison_lds), and
    the forward is repeated with poisoning workgroups running concurrently on a side stream:
    the outputs must stay bitwise equal to an undisturbed forward."""
    from waveformer_amd import _lib, ops
    case = C.cases()["enc128"]
    m, _ = C.build(case, "cuda")
    x = torch.cat([C.case_input(case)] * 2).cuda()
    with torch.no_grad():
        ref = [t.clone() for t in _flat(m(x))]
    torch.cuda.synchronize()
    sizes = [16 * 1024, 48 * 1024, 96 * 1024, 160 * 1024]
    real_call = _lib.call
    n = [0]

    def poisoned_call(name, *args):
        if name != "wf_debug_poison_lds":
            lb = sizes[n[0] % len(sizes)]
            n[0] += 1
            real_call("wf_debug_poison_lds", 2048, lb, ops._stream())
        return real_call(name, *args)

    _lib.call = poisoned_call
    try:
        with torch.no_grad():
            got = [t.clone() for t in _flat(m(x))]
        torch.cuda.synchronize()
    finally:
        _lib.call = real_call
    assert n[0] > 50
    for a, b in zip(ref, got):
        assert torch.equal(a, b)

    side = torch.cuda.Stream()
    main = torch.cuda.current_stream()
    side.wait_stream(main)
    with torch.cuda.stream(side):
        for i in range(400):
            _lib.call("wf_debug_poison_lds", 512, sizes[i % len(sizes)], ops._stream())
    with torch.no_grad():
        got = [t.clone() for t in _flat(m(x))]
    main.wait_stream(side)
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
