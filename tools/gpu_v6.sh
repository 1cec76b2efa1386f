#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab.sh v6 WF_GEMM_NO_KC || exit $?
timeout -k 10 300 python tools/kbench_conv.py > gpurun_out/v6_conv.txt 2>&1
cat gpurun_out/v6_conv.txt
