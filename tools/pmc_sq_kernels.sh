#!/bin/bash
# SQ stall breakdown per kernel instance (name + grid) of every kernel matching REGEX under a
# driver (default tools/enc_drv.py, ITERS=1): two counter passes, mean per launch, derived
#   wait% = SQ_WAIT_ANY / SQ_WAVE_CYCLES, inst% = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES,
#   valu% = SQ_INSTS_VALU x 2 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), mfma% = MFMA busy / (1024 x GRBM / 8),
#   ldsc = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS.
#   tools/pmc_sq_kernels.sh TAG REGEX [DRIVER]
set -o pipefail
TAG=$1; RX=$2; DRV=${3:-tools/enc_drv.py}
export TMPDIR=/tmp ITERS=${ITERS:-1}
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${TAG}_p1 -o run -- python $DRV > gpurun_out/${TAG}_p1.log 2>&1 || { tail -5 gpurun_out/${TAG}_p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${TAG}_p2 -o run -- python $DRV > gpurun_out/${TAG}_p2.log 2>&1 || { tail -5 gpurun_out/${TAG}_p2.log; exit 1; }
python - "$TAG" <<'PY'
import collections, csv, glob, sys
tag = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/{tag}_p*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    key = {}
    for r in csv.DictReader(open(f)):
        d = (f, r["Dispatch_Id"])
        per[d, r["Counter_Name"]] += float(r["Counter_Value"])
        key[d] = (r["Kernel_Name"].split("(")[0][:60], r["Grid_Size"], r.get("VGPR_Count", "?"))
    for (d, c), v in per.items():
        acc[key[d]][c].append(v)
print(f"{'kernel':60s} {'grid':>9s} {'vgpr':>4s} {'wait%':>6s} {'inst%':>6s} {'valu%':>6s} {'mfma%':>6s} {'ldsc':>5s} {'vmemc/w':>8s} {'gui_us':>7s}")
for k, cs in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("GRBM_GUI_ACTIVE", [0]))):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    g = m.get("GRBM_GUI_ACTIVE", 0) / 8 or 1
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k[0]:60s} {k[1]:>9s} {k[2]:>4s} {100*m.get('SQ_WAIT_ANY',0)/wc:6.1f} {100*m.get('SQ_WAIT_INST_ANY',0)/wc:6.1f} "
          f"{100*m.get('SQ_INSTS_VALU',0)*2/(1024*g):6.1f} {100*m.get('SQ_VALU_MFMA_BUSY_CYCLES',0)/(1024*g):6.1f} "
          f"{m.get('SQ_LDS_BANK_CONFLICT',0)/(m.get('SQ_INSTS_LDS',0) or 1):5.2f} "
          f"{m.get('SQ_INST_CYCLES_VMEM',0)/(m.get('SQ_WAVES',0) or 1):8.1f} {g/2400:7.1f}")
PY
