#!/bin/bash
# Sliding-window (config 3) bench + kernel-trace profile of it.
set -o pipefail
TAG=${1:-swp}
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/${TAG}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u bench.py --workload sliding --steps 3 --warmup 1 > gpurun_out/${TAG}_sliding.json 2> gpurun_out/${TAG}_sliding.err || { tail -30 gpurun_out/${TAG}_sliding.err; exit 1; }
cat gpurun_out/${TAG}_sliding.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python -u bench.py --workload sliding --steps 1 --warmup 1 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -30 gpurun_out/${TAG}_prof.log; exit 1; }
head -30 gpurun_out/${TAG}_prof/run_kernel_stats.csv | cut -c1-200
