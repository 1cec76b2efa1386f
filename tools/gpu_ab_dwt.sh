#!/bin/bash
set -o pipefail
TAG=${1:-ad}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "dwt or block or enc" > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_new.json 2>/dev/null || exit 1
WF_NOTHING=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_old.json 2>/dev/null || exit 1
python tools/bench_line.py gpurun_out/${TAG}_new.json gpurun_out/${TAG}_old.json
