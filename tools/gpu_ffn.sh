#!/bin/bash
# fused-FFN GPU check: the FFN / module / Dice parity tests, the bench and a kernel trace
set -o pipefail
TAG=${1:-ffn1}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "ccf_ffn or module_vs or full_model_128 or encoder128" > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
echo done
