"""Scan gfx950 device assembly (hipcc --cuda-device-only -S) for register write-after-read
patterns the compiler's hazard recognizer does not pad:

  ds      : an LDS write with more than 64 bits of data (ds_write_b96/b128, ds_write2*_b64)
            followed within WIN instructions by an instruction that writes one of its DATA
            VGPRs (the round-3 stage-2 corruption: gemm_lnw<SPLIT,3>'s staging loop,
            `ds_write2st64_b64 v4, v[8:9], v[2:3]` then `v_add_u32 v2, ...`);
  vmem    : the same after a >64-bit global/buffer store;
  mfma_ab : an MFMA followed within WIN instructions by a write of one of its A / B VGPRs.

usage: python tools/isa_hazard_scan.py [WIN] file.s ...   (prints per kernel counts + examples)
"""
import re
import sys


def regs(s):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]", s):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", s):
        out.add(int(m.group(1)))
    return out


def operands(t):
    parts = t.split(None, 1)
    if len(parts) < 2:
        return []
    return [o.strip() for o in re.split(r",(?![^\[]*\])", parts[1])]


WIDE_DS = re.compile(r"^ds_(write|store)(_b96|_b128|2st64_b64|2_b64)\b")
WIDE_VM = re.compile(r"^(global|buffer|flat)_store_(dwordx3|dwordx4|b96|b128)\b")
NO_DST = re.compile(r"^(s_|ds_write|ds_store|global_store|buffer_store|flat_store|v_cmp|v_cmpx|;)")


def dst_regs(t):
    """VGPRs an instruction writes (first operand of VALU / loads / ds_read / mfma)."""
    if NO_DST.match(t) or not (t.startswith("v_") or "_load" in t or t.startswith("ds_read")
                               or t.startswith("ds_bpermute") or t.startswith("ds_swizzle")):
        return set()
    ops = operands(t)
    return regs(ops[0]) if ops else set()


def scan(path, win):
    kern, res = None, {}
    raw = open(path).read().split("\n")
    lines = [l.split(";")[0].strip() if not l.strip().startswith(";") else "" for l in raw]
    insts = []
    for i, l in enumerate(raw):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            kern = m.group(1)
            continue
        t = lines[i]
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        insts.append((kern, i + 1, t))
    for k, (kern, ln, t) in enumerate(insts):
        kind, data = None, set()
        if WIDE_DS.match(t):
            kind = "ds"
            for o in operands(t)[1:]:
                data |= regs(o)
        elif WIDE_VM.match(t):
            kind = "vmem"
            ops = operands(t)
            data = regs(ops[1]) if t.startswith("global") or t.startswith("flat") else regs(ops[0])
        elif t.startswith("v_mfma"):
            kind = "mfma_ab"
            ops = operands(t)
            data = regs(ops[1]) | regs(ops[2])
        if not kind:
            continue
        n = 0
        for kern2, ln2, u in insts[k + 1:]:
            if kern2 != kern:
                break
            if u.startswith("s_nop"):
                n += int(u.split()[1]) + 1
            else:
                n += 1
            if n > win:
                break
            if dst_regs(u) & data:
                r = res.setdefault(kern, {}).setdefault(kind, [])
                r.append(f"{ln}: {t}  ->  {ln2}: {u}")
                break
    return res


if __name__ == "__main__":
    args = sys.argv[1:]
    win = int(args.pop(0)) if args and args[0].isdigit() else 2
    total = {}
    for p in args:
        for kern, kinds in scan(p, win).items():
            print(f"{p}: {kern}")
            for kind, ex in kinds.items():
                total[kind] = total.get(kind, 0) + len(ex)
                print(f"  {kind}: {len(ex)}   e.g. {ex[0]}")
    print("TOTAL", total)
