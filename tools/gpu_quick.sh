#!/bin/bash
# quick GPU check: a pytest -k selection, then the bench and a kernel trace
set -o pipefail
TAG=$1; SEL=$2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu -k "$SEL" > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
python tools/kstats.py gpurun_out/${TAG}_prof/run_kernel_trace.csv > gpurun_out/${TAG}_kstats.txt; head -16 gpurun_out/${TAG}_kstats.txt
