#!/bin/bash
# full -m gpu suite, then bench + kernel trace
set -o pipefail
TAG=${1:-v10}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.txt
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" gpurun_out/${TAG}_pytest.txt | head -20; exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --batch 4 > gpurun_out/${TAG}_bench_b4.json 2> gpurun_out/${TAG}_bench_b4.err || exit 1
cat gpurun_out/${TAG}_bench_b4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --batch 4 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
echo done
