"""Mean per launch of the SQ counters collected by tools/pmc_sq_b8.sh, plus the derived issue /
wait fractions.  Units (MI355X_MICROARCH.md, 's_memtime tick vs SQ PMC units'): SQ_WAVE_CYCLES,
SQ_WAIT_*, SQ_ACTIVE_INST_* count quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE
count cycles (GRBM summed over the 8 XCDs).  VALU issue-busy uses the 2-cycle SIMD-32 throughput
of a wave64 v_fma_f32 (constants table), i.e. SQ_INSTS_VALU x 2 / (1024 SIMDs x cycles).

    python tools/pmc_summary_sq.py gpurun_out/TAG_p REGEX
"""
import collections
import csv
import glob
import re
import sys


def main(prefix, rx):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{prefix}*/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if not re.search(rx, r["Kernel_Name"]):
                continue
            per[(r["Counter_Name"], r.get("Dispatch_Id", ""))] += float(r["Counter_Value"])
        for (k, _), v in per.items():
            acc[k].append(v)
    m = {k: sum(v) / len(v) for k, v in acc.items()}
    for k in sorted(m):
        print(f"{k:28s} {m[k]:18.1f}  (n={len(acc[k])})")
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc:
        valu = m.get("SQ_INSTS_VALU", 0) - m.get("SQ_INSTS_MFMA", 0)
        print(f"# cycles per launch (GRBM_GUI_ACTIVE/8)   {cyc:.0f}")
        print(f"# VALU issue-busy (2 cyc/instr, non-MFMA)  {valu * 2 / 1024 / cyc:.3f}")
        print(f"# MFMA pipe busy (BUSY_CYCLES/1024 SIMDs)  {m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / 1024 / cyc:.3f}")
        print(f"# LDS array busy (IDX_ACTIVE/256 CUs)      {m.get('SQ_LDS_IDX_ACTIVE', 0) / 256 / cyc:.3f}")
    wc = m.get("SQ_WAVE_CYCLES", 0)
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            print(f"# {k:24s} / WAVE_CYCLES  {m.get(k, 0) / wc:.3f}")
    if m.get("SQ_INSTS_LDS"):
        print(f"# LDS bank-conflict cycles per LDS instr  {m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_INSTS_LDS']:.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
