"""VALU issue fraction and MFMA-pipe busy per kernel from one rocprofv3 --pmc pass
(SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE) of a command, written
to a JSON summary that bench.py reads (roofline.valu_issue_frac, mfma_busy_frac).

    python tools/pmc_valu.py gpurun_out/TAG_pmc_valu OUT.json BATCH

valu_issue_frac = (SQ_INSTS_VALU - SQ_INSTS_MFMA) x 2 cycles / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8):
the share of a SIMD's VALU issue capacity the launch used, at the SIMD-32 throughput of a
wave64 v_fma_f32 -- 2 cycles per wave-instruction with two or more waves on the SIMD
(MI355X_MICROARCH.md, per-instruction constants; one wave alone issues at most every 4).
Round 3 priced it at 4 cycles, which doubled the fraction.
mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8).
For each kernel the largest launch is reported."""
import collections
import csv
import glob
import json
import sys


def main(root, out_path, batch):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"].split("(")[0], r.get("Dispatch_Id", ""))
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    best = {}
    for (name, _), c in per.items():
        if not c.get("GRBM_GUI_ACTIVE"):
            continue
        if name not in best or c["GRBM_GUI_ACTIVE"] > best[name]["GRBM_GUI_ACTIVE"]:
            best[name] = dict(c)
    kernels = {}
    for name, c in best.items():
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        valu = c.get("SQ_INSTS_VALU", 0.0) - c.get("SQ_INSTS_MFMA", 0.0)
        kernels[name] = {"valu_insts_per_launch": valu, "mfma_insts_per_launch": c.get("SQ_INSTS_MFMA", 0.0),
                         "cycles_per_xcd": cyc, "valu_issue_frac": round(valu / 1024 * 2 / cyc, 4),
                         "valu_cycles_per_inst": 2}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            kernels[name]["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / cyc, 4)
    json.dump({"per_gpu_batch": batch, "source": root, "kernels": kernels}, open(out_path, "w"), indent=1)
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["cycles_per_xcd"])[:12]:
        print(f"{v['valu_issue_frac']:6.3f}  {v['cycles_per_xcd']:12.0f} cyc  {k[:80]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]))
