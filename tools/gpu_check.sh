#!/bin/bash
# Quick GPU iteration: the parity tests matching $2 (pytest -k), then a short B=8 bench line.
# Usage: tools/gpu_check.sh TAG "pytest -k expression" [extra bench args]
set -o pipefail
TAG=${1:-chk}
K=${2:-ccf_ffn}
shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_config.py -k "$K" > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_pytest.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --cpu-baseline 0 --parity 0 "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python tools/bench_line.py gpurun_out/${TAG}_bench.json
