#!/bin/bash
# decoder op tests (incl. the up-sampling adjoint), training gradient parity, config-4 bench
set -o pipefail
TAG=${1:-t3}
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/${TAG}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_decoder.py tests/test_train_grads.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.txt
timeout -k 10 700 python -u bench.py --workload train --steps 3 --warmup 1 --batch 1 > gpurun_out/${TAG}_train.json 2> gpurun_out/${TAG}_train.err || { tail -20 gpurun_out/${TAG}_train.err; exit 1; }
cut -c1-400 gpurun_out/${TAG}_train.json
