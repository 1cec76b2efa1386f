"""Which op spends config 5's Dice margin?  Runs the full 192^3 Waveformer with the HF branch
(the reference's 192^3 labels, tests/golden) at fp16 with ONE op group switched to the
fp32-faithful bf16x3 arithmetic, and at bf16x3 with one group switched to fp16, and prints
Dice TC/WT/ET for each.  Groups: attn (window attention), ffn (CCF_FFN), merge
(PatchMerging), conv (decoder 3x3x3 convolutions), linear (decoder 1x1 GEMMs), embed.
usage: python tools/prec_attrib.py [full192hf|full128] [conv]   (conv: per-layer attribution)"""
import sys

import torch

sys.path.insert(0, ".")
from tests import cases as C  # noqa: E402
from waveformer_amd import _lib, ops  # noqa: E402

SPLIT, FP16 = ops.PRECISIONS["bf16x3"], ops.PRECISIONS["fp16"]
GROUPS = {"attn": ["window_attention"], "ffn": ["ccf_ffn_raw"], "merge": ["_patch_merging_raw"],
          "conv": ["conv3d_k3"], "linear": ["linear_rows"]}


def patched(group, prec_name):
    """Wrap the ops of `group` so they run at `prec_name` whatever the global precision."""
    saved = {}
    for fn in GROUPS[group]:
        orig = getattr(ops, fn)
        saved[fn] = orig
        pid = ops.PRECISIONS[prec_name]

        def w(*a, _o=orig, _fn=fn, **kw):
            if _fn in ("window_attention", "ccf_ffn_raw"):
                kw["prec"] = pid
                return _o(*a, **kw)
            if _fn == "_patch_merging_raw":
                a = list(a)
                a[6] = pid
                return _o(*a, **kw)
            with ops.precision(prec_name):
                return _o(*a, **kw)
        setattr(ops, fn, w)
    return saved


def restore(saved):
    for k, v in saved.items():
        setattr(ops, k, v)


def dice(case_name, base, group=None, other=None):
    case = C.cases()[case_name]
    m, _ = C.build(case, "cuda")
    saved = patched(group, other) if group else {}
    try:
        with torch.no_grad(), ops.precision(base):
            lab = m(C.case_input(case).cuda()).argmax(1).cpu()
    finally:
        restore(saved)
    ref = C.g(case_name + "_labels").long()
    d = [C.dice(a, b) for a, b in zip(C.brats_regions(lab), C.brats_regions(ref))]
    del m
    torch.cuda.empty_cache()
    return d


def conv_layers(case_name="full192hf"):
    """Per-call attribution of the decoder convolutions: all ops fp16 except conv call i at
    bf16x3, and all bf16x3 except conv call i at fp16 -- which layers spend the margin."""
    case = C.cases()[case_name]
    m, _ = C.build(case, "cuda")
    ref = C.g(case_name + "_labels").long()
    orig = ops.conv3d_k3
    calls = []

    def counting(*a, **kw):
        calls.append(tuple(a[0].shape) + (a[1].shape[0],))
        return orig(*a, **kw)
    ops.conv3d_k3 = counting
    with torch.no_grad(), ops.precision("fp16"):
        m(C.case_input(case).cuda())
    ops.conv3d_k3 = orig
    n = len(calls)
    for base, other in (("fp16", "bf16x3"), ("bf16x3", "fp16")):
        for i in range(n):
            cnt = [0]

            def w(*a, _i=i, **kw):
                j = cnt[0]
                cnt[0] += 1
                if j == _i:
                    with ops.precision(other):
                        return orig(*a, **kw)
                return orig(*a, **kw)
            ops.conv3d_k3 = w
            try:
                with torch.no_grad(), ops.precision(base):
                    lab = m(C.case_input(case).cuda()).argmax(1).cpu()
            finally:
                ops.conv3d_k3 = orig
            d = [C.dice(a, b) for a, b in zip(C.brats_regions(lab), C.brats_regions(ref))]
            print(f"{case_name} {base}, conv call {i} {calls[i]} at {other}: delta "
                  f"{1 - min(d):.2e}", flush=True)


def combos(case_name="full192hf"):
    """fp16 with attention + a set of conv calls (by call index) at bf16x3."""
    sets = {"A attn+conv{2,4,6}": ({2, 4, 6}, []), "B attn+conv{2..7}": (set(range(2, 8)), []),
            "C attn+conv{2,4,6}+merge": ({2, 4, 6}, ["merge"]),
            "D attn+conv{2,4,6}+merge+ffn": ({2, 4, 6}, ["merge", "ffn"]),
            "E attn+all conv": (set(range(64)), [])}
    case = C.cases()[case_name]
    m, _ = C.build(case, "cuda")
    ref = C.g(case_name + "_labels").long()
    orig = ops.conv3d_k3
    for name, (cs, extra) in sets.items():
        cnt = [0]

        def w(*a, _cs=cs, **kw):
            j = cnt[0]
            cnt[0] += 1
            if j in _cs:
                with ops.precision("bf16x3"):
                    return orig(*a, **kw)
            return orig(*a, **kw)
        saved = patched("attn", "bf16x3")
        for g in extra:
            saved.update(patched(g, "bf16x3"))
        ops.conv3d_k3 = w
        try:
            with torch.no_grad(), ops.precision("fp16"):
                lab = m(C.case_input(case).cuda()).argmax(1).cpu()
        finally:
            ops.conv3d_k3 = orig
            restore(saved)
        d = [C.dice(a, b) for a, b in zip(C.brats_regions(lab), C.brats_regions(ref))]
        print(f"{case_name} fp16 {name}: Dice {[round(v, 6) for v in d]} delta {1 - min(d):.2e}",
              flush=True)


if __name__ == "__main__":
    _lib.load()
    name = sys.argv[1] if len(sys.argv) > 1 else "full192hf"
    if len(sys.argv) > 2 and sys.argv[2] == "conv":
        conv_layers(name)
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[2] == "combos":
        combos(name)
        sys.exit(0)
    for base, other in (("fp16", "bf16x3"), ("bf16x3", "fp16")):
        d = dice(name, base)
        print(f"{name} all {base}: Dice {[round(v, 6) for v in d]} delta {1 - min(d):.2e}", flush=True)
        for g in GROUPS:
            d = dice(name, base, g, other)
            print(f"{name} {base} with {g} at {other}: Dice {[round(v, 6) for v in d]} "
                  f"delta {1 - min(d):.2e}", flush=True)
