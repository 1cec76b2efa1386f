#!/bin/bash
# parity (encoder + attention + training grads) and the encoder bench's attention timing
set -o pipefail
TAG=${1:-aa}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_train_grads.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_new.json 2>/dev/null || exit 1
python tools/bench_line.py gpurun_out/${TAG}_new.json
