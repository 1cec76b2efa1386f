#!/bin/bash
set -o pipefail
TAG=${1:-cv}
timeout -k 10 300 python -u -m pytest tests/test_gpu_decoder.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.txt
tools/pmc_conv.sh ${TAG} 2
