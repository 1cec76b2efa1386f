#!/bin/bash
# Interleaved bench A/B of environment settings: tools/gpu_benchab.sh TAG ROUNDS "ENV1" "ENV2" ...
# ("-" = no extra setting).  Each run: bench.py --steps 150 (encoder, B = 8), value printed.
set -o pipefail
TAG=$1; R=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    [ "$e" = "-" ] && e="WF_NONE=1"
    env $e timeout -k 10 200 python -u bench.py --steps ${STEPS:-150} --warmup 10 --cpu-baseline 0 --parity 0 --op-timers 0 ${BENCH_ARGS} > gpurun_out/${TAG}_${r}_$i.json 2> gpurun_out/${TAG}_${r}_$i.err || { tail -20 gpurun_out/${TAG}_${r}_$i.err; exit 1; }
    echo "round $r [$e] $(python tools/bench_line.py gpurun_out/${TAG}_${r}_$i.json)"
  done
done
