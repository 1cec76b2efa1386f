#!/bin/bash
# SQ counters of two encoder kernels: the stage-2 depthwise conv (kbench_ffn at C=96, S=32)
# and the attention core (encoder bench, eager).  One counter set per rocprofv3 run.
set -o pipefail
TAG=${1:-pe}
export TMPDIR=/tmp
mkdir -p gpurun_out
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT"
C2="SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VMEM_WR"
i=0
for set in "$C1" "$C2"; do
  i=$((i+1))
  C=96 S=32 ITERS=3 timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex dwconv3d_kernel --output-format csv -d gpurun_out/${TAG}_dw$i -o run -- python tools/kbench_ffn.py > gpurun_out/${TAG}_dw$i.log 2>&1 || { echo "dw pmc $i failed"; tail -5 gpurun_out/${TAG}_dw$i.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex attn_core_kernel --output-format csv -d gpurun_out/${TAG}_at$i -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_at$i.log 2>&1 || { echo "attn pmc $i failed"; tail -5 gpurun_out/${TAG}_at$i.log; exit 1; }
done
python - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
for part in ("dw", "at"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/{tag}_{part}*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(part)
    for k, v in sorted(acc.items()):
        print(f"  {k:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
