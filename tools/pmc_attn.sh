#!/bin/bash
# Attention core under tools/kbench_attn.py: kernel trace, HBM traffic (FETCH / WRITE), SQ
# issue counters.  One counter set per rocprofv3 run.
set -o pipefail
TAG=${1:-pa}
export TMPDIR=/tmp ITERS=3
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- python tools/kbench_attn.py > gpurun_out/${TAG}_kt.log 2>&1 || { tail -5 gpurun_out/${TAG}_kt.log; exit 1; }
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex attn_ --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python tools/kbench_attn.py > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pmc $i failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done
python - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/{tag}_p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
tr = glob.glob(f"gpurun_out/{tag}_kt/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(tr[0])):
    print(r["Name"][:70], r["Calls"], r["AverageNs"])
PY
