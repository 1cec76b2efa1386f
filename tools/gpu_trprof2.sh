#!/bin/bash
# kernel-trace profile of the config-4 train step (B=1, MIOpen find, 2 timed steps)
set -o pipefail
TAG=${1:-tp}
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/${TAG}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 800 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python -u bench.py --workload train --steps 2 --warmup 1 --batch 1 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -30 gpurun_out/${TAG}_prof.log; exit 1; }
grep "metric" gpurun_out/${TAG}_prof.log | cut -c1-300
