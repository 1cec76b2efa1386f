#!/bin/bash
# depthwise-conv kernel change: parity of its users + encoder bench + kernel stats
set -o pipefail
TAG=${1:-dw}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decoder.py tests/test_train_grads.py -x -q --timeout 200 --timeout-method thread -m gpu -k "block or enc or ffn or dwconv or Projection or module or stage" > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_new.json 2>/dev/null || exit 1
cat gpurun_out/${TAG}_new.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-160; grep -i dwconv "$f" | cut -c1-160
