"""Weight updates between forwards reach the kernels.

The MFMA kernels read derived forms of the fp32 parameters (bf16 hi / lo planes, packed conv
weights, dense relative-position biases).  They are rebuilt at the start of every top-level
forward (ops.weight_scope: one launch for all split weights), never cached across forwards, so
a write through `.data` -- which bumps no version counter (EMA, weight surgery, re-init) --
is seen by the next forward, eagerly and in a replayed HIP graph.  Checked bit-for-bit against
a fresh model loaded with the updated weights.
"""
from functools import partial

import pytest
import torch
import torch.nn as nn

from oracle.weight_rule import rule_state_dict, seeded_randn

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from waveformer_amd import _lib
    _lib.load()
    yield


def _encoder():
    import waveformer_amd.network_models as NM
    m = NM.MultiscaleTransformer(img_size=(32,) * 3, in_chans=4, qkv_bias=True,
                                 norm_layer=partial(nn.LayerNorm, eps=1e-6))
    m.load_state_dict(rule_state_dict(m.state_dict()), strict=True)
    return m.eval().cuda()


def _touch(m):
    """Rewrite split-operand weights of every kind through .data (no version bump)."""
    names = ["block1.0.attn.qkv.weight", "block1.1.mlp.pwconv.weight", "block2.0.mlp.fc.weight",
             "downsample_1.reduction.weight", "block4.1.attn.proj.weight",
             "block3.0.attn.relative_position_bias_table"]
    params = dict(m.named_parameters())
    for n in names:
        p = params[n]
        v0 = p._version
        p.data.copy_(p.data * 1.25 + 0.01)
        assert p._version == v0  # the case a version-keyed cache misses
    return names


def _flat(r):
    outs, hfs = r
    return list(outs) + [d[k] for h in hfs for d in h for k in sorted(d)]


def test_data_write_between_forwards_is_seen():
    m = _encoder()
    x = seeded_randn((1, 4, 32, 32, 32), 71).cuda()
    with torch.no_grad():
        before = _flat(m(x))
        _touch(m)
        after = _flat(m(x))
        fresh = _encoder()
        fresh.load_state_dict(m.state_dict())
        want = _flat(fresh(x))
    assert not torch.equal(before[0], after[0])
    for a, b in zip(after, want):
        assert torch.equal(a, b)


def test_data_write_seen_by_graph_replay():
    m = _encoder()
    x = seeded_randn((1, 4, 32, 32, 32), 72).cuda()
    with torch.no_grad():
        m(x)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m(x)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            static = _flat(m(x))
        g.replay()
        torch.cuda.synchronize()
        before = [t.clone() for t in static]
        _touch(m)
        g.replay()
        torch.cuda.synchronize()
        fresh = _encoder()
        fresh.load_state_dict(m.state_dict())
        want = _flat(fresh(x))
    assert not torch.equal(before[0], static[0])
    for a, b in zip(static, want):
        assert torch.equal(a, b)


def test_arenas_bounded_over_fresh_threads():
    """one weight arena per thread identity, never freed.  Forwards on six
    short-lived threads, one after another: the arenas of ended threads are retired at the next
    scope entry, so the model holds at most this thread's and the last worker's.  Every thread
    computes the same output."""
    import threading

    from waveformer_amd import ops
    m = _encoder()
    x = seeded_randn((1, 4, 32, 32, 32), 73).cuda()
    with torch.no_grad():
        want = _flat(m(x))
    outs, errs = [], []

    def work():
        try:
            with torch.no_grad():
                outs.append(_flat(m(x)))
            torch.cuda.synchronize()
        except Exception as e:  # surfaced below
            errs.append(e)

    for _ in range(6):
        t = threading.Thread(target=work)
        t.start()
        t.join()
        assert ops.arena_count(m) <= 2
    assert not errs, errs
    with torch.no_grad():
        m(x)  # the main thread's next forward retires the last worker's arena
    assert ops.arena_count(m) == 1
    for o in outs:
        for a, b in zip(o, want):
            assert torch.equal(a, b)
