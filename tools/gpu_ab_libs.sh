#!/bin/bash
# parity on the in-tree library, then a kernel-trace A/B of library variants on the encoder driver
# usage: tools/gpu_ab_libs.sh TAG "PYTEST_K_EXPR" abso/A.so abso/B.so ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; KX=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "$KX" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -20 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.txt
bash tools/gpu_ab.sh $TAG tools/enc_drv.py "$@"
