#!/bin/bash
# Config-4 train bench variants: immediate mode with MIOpen's naive conv solvers disabled
# (B=2), then find mode (B=1).
set -o pipefail
TAG=${1:-tt}
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/${TAG}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW=0 \
  timeout -k 10 480 python -u bench.py --workload train --steps 3 --warmup 1 --batch 2 --miopen-find 0 > gpurun_out/${TAG}_imm.json 2> gpurun_out/${TAG}_imm.err
echo "immediate rc=$?"; grep -v amdgpu gpurun_out/${TAG}_imm.err | tail -4; cat gpurun_out/${TAG}_imm.json
timeout -k 10 480 python -u bench.py --workload train --steps 3 --warmup 1 --batch 1 --miopen-find 1 > gpurun_out/${TAG}_find.json 2> gpurun_out/${TAG}_find.err
echo "find rc=$?"; grep -v amdgpu gpurun_out/${TAG}_find.err | tail -4; cat gpurun_out/${TAG}_find.json
