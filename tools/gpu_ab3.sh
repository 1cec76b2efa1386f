#!/bin/bash
# Interleaved A/B (3 rounds) of stage-1 FFN back-half variants at B = 8 under a kernel trace.
# Each argument is LIB[:ENV=VAL]; e.g. abso/libwf_pk.so abso/libwf_pk.so:WF_FFN_DWFC_WS=1
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2 3; do
  k=0
  for spec in "$@"; do
    k=$((k+1))
    lib=${spec%%:*}; envs=""; [ "$spec" != "$lib" ] && envs=${spec#*:}
    d=gpurun_out/${TAG}_v${k}_$rep
    env $envs WAVEFORMER_HIP_LIB=$PWD/$lib B=8 C=${KC:-48} S=${KS:-64} ITERS=10 timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $d -o run -- python3 tools/kbench_ffn.py > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    python3 - "$f" "$spec" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "dwfc" in r["Name"] or "gemm" in r["Name"]:
        print(f'{sys.argv[2]:45s} {float(r["AverageNs"]) / 1e3:8.1f} us  {r["Name"][:50]}')
PY
  done
done
