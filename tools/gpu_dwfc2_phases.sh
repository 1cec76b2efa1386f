#!/bin/bash
# ffn_dwfc2 phase attribution: the B = 8 stage-2 FFN with phases of the fused kernel skipped
# (WF_FFN_DBG bits: 1 scatter, 2 LN2, 4 fc, 8 fetch/commit; results invalid), kernel trace.
set -o pipefail
TAG=${1:-dwfc2ph}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for d in ${DBGS:-0 1 2 4 8 6 15}; do
  WF_FFN_DBG=$d B=8 C=${KC:-96} S=${KS:-32} ITERS=10 timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/p$d -o run -- python3 tools/kbench_ffn.py > $OUT/p$d.log 2>&1 \
    || { tail -20 $OUT/p$d.log; exit 1; }
  f=$(find $OUT/p$d -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$d" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "dwfc" in r["Name"]:
        print(f'dbg {sys.argv[2]:>2}: {float(r["AverageNs"]) / 1e3:8.1f} us  {r["Name"][:60]}')
PY
done
