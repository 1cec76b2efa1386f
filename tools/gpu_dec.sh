#!/bin/bash
# Decoder conv stack: op tests, model-level parity, then full-model forward timing.
set -o pipefail
TAG=${1:-dec}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_decoder.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?
tail -25 gpurun_out/${TAG}_pytest.txt
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "full or module" > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?
tail -8 gpurun_out/${TAG}_parity.txt
exit $rc
