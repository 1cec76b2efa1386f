#!/bin/bash
# conv3d_k3 at the decoder shapes (timing), then SQ counter passes on shape $2 (default 2:
# B=2 96->48 at 128^3) -- one counter set per rocprofv3 run.
set -o pipefail
TAG=${1:-cv}; IDX=${2:-2}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/kbench_conv_hip.py > gpurun_out/${TAG}_kb.txt 2>&1 || { tail -20 gpurun_out/${TAG}_kb.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_kb.txt
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT" "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU"; do
  i=$((i+1))
  ITERS=3 timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex conv3d_k3_kernel --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python tools/kbench_conv_hip.py $IDX > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pmc set $i failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
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
PY
