#!/bin/bash
# SQ stall breakdown of the whole-FFN kernel (regex $2) under tools/kbench_ffn_fused.py: two passes
set -o pipefail
TAG=$1; RX=$2
export TMPDIR=/tmp
export ITERS=3
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${TAG}_p1 -o run -- python tools/kbench_ffn_fused.py 0 > gpurun_out/${TAG}_p1.log 2>&1 || { tail -5 gpurun_out/${TAG}_p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${TAG}_p2 -o run -- python tools/kbench_ffn_fused.py 0 > gpurun_out/${TAG}_p2.log 2>&1 || { tail -5 gpurun_out/${TAG}_p2.log; exit 1; }
python - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/{tag}_p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
