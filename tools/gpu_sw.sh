#!/bin/bash
# config-3 GPU check: sliding-window parity tests, the encoder bench (driver line), the
# sliding-window bench, and a kernel trace of the encoder bench.
set -o pipefail
TAG=${1:-sw1}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sliding_window.py -x -v --timeout 120 \
  --timeout-method thread -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 400 python bench.py --workload sliding --steps 3 --warmup 1 > gpurun_out/${TAG}_sliding.json 2> gpurun_out/${TAG}_sliding.err || { tail -20 gpurun_out/${TAG}_sliding.err; exit 1; }
cat gpurun_out/${TAG}_sliding.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
echo done
