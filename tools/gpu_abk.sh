#!/bin/bash
# Interleaved A/B (3 rounds) of library builds / env switches on one driver under a kernel trace:
#   tools/gpu_abk.sh TAG DRIVER.py REGEX LIB[:ENV=VAL] ...
# prints the average duration of every kernel whose name matches REGEX, per variant and round.
set -o pipefail
TAG=$1; DRV=$2; RX=$3; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2 3; do
  k=0
  for spec in "$@"; do
    k=$((k+1))
    lib=${spec%%:*}; envs=""; [ "$spec" != "$lib" ] && envs=${spec#*:}
    d=gpurun_out/${TAG}_v${k}_$rep
    env $envs WAVEFORMER_HIP_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $d -o run -- python3 $DRV > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    python3 - "$f" "$spec" "$RX" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], r["Name"]):
        print(f'{sys.argv[2]:52s} {float(r["AverageNs"]) / 1e3:8.1f} us x{r["Calls"]:>4s}  {r["Name"][:60]}')
PY
  done
done
