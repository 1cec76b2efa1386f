#!/bin/bash
# Training path on one GPU: gradient parity tests, then a short config-4 train bench.
#   tools/gpu_train.sh TAG [BATCH]
set -o pipefail
TAG=${1:-tr}; BATCH=${2:-2}
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/${TAG}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_train_grads.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?
tail -25 gpurun_out/${TAG}_pytest.txt
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 900 python -u bench.py --workload train --steps 3 --warmup 2 --batch $BATCH > gpurun_out/${TAG}_train.json 2> gpurun_out/${TAG}_train.err || { tail -30 gpurun_out/${TAG}_train.err; exit 1; }
cat gpurun_out/${TAG}_train.json
