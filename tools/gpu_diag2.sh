#!/bin/bash
# full32 gradient diagnosis, then the config-4 probe with channels_last_3d decoder convs.
set -o pipefail
TAG=${1:-dg}
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/${TAG}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u tools/grad_diag.py full32 > gpurun_out/${TAG}_diag.txt 2>&1 || { tail -20 gpurun_out/${TAG}_diag.txt; exit 1; }
WF_CL3D=1 timeout -k 10 700 python -u tools/train_probe.py 1 3 > gpurun_out/${TAG}_cl.txt 2>&1 || { tail -20 gpurun_out/${TAG}_cl.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_cl.txt
