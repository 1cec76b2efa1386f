#!/bin/bash
# General-wavelet kernel tests + per-tensor gradient diagnosis of the full model.
set -o pipefail
TAG=${1:-wv}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wavelets.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_pytest.txt
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 400 python -u tools/grad_diag.py full32 > gpurun_out/${TAG}_diag.txt 2>&1 || { tail -20 gpurun_out/${TAG}_diag.txt; exit 1; }
cat gpurun_out/${TAG}_diag.txt
