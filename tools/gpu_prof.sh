#!/bin/bash
# Kernel trace of the default bench step: warm-up + graph replays only (no op-timer repeats).
# Usage: tools/gpu_prof.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-prof}
shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 --parity 0 --op-timers 0 "$@" > gpurun_out/${TAG}_prof.log 2>&1 || { tail -30 gpurun_out/${TAG}_prof.log; exit 1; }
tail -1 gpurun_out/${TAG}_prof.log | cut -c1-200
f=$(ls gpurun_out/${TAG}_prof/*kernel_trace.csv | head -1)
python tools/kstats.py "$f" ${NK:-30} > gpurun_out/${TAG}_kstats.txt
cat gpurun_out/${TAG}_kstats.txt
