#!/bin/bash
# Config-4 probe: decoder convs with channels_last_3d, then MIOpen find (cudnn.benchmark).
set -o pipefail
TAG=${1:-cl}
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/${TAG}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
WF_CL3D=1 timeout -k 10 500 python -u tools/train_probe.py 1 2 > gpurun_out/${TAG}_cl.txt 2>&1 || { tail -20 gpurun_out/${TAG}_cl.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_cl.txt
WF_CL3D=1 WF_CUDNN_BENCH=1 timeout -k 10 500 python -u tools/train_probe.py 1 2 > gpurun_out/${TAG}_clb.txt 2>&1 || { tail -20 gpurun_out/${TAG}_clb.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_clb.txt
