#!/bin/bash
# Training path: gradient parity tests, then a rocprofv3 kernel-trace of tools/train_probe.py.
#   tools/gpu_trprof.sh TAG [BATCH]
set -o pipefail
TAG=${1:-trp}; BATCH=${2:-1}
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/${TAG}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_train_grads.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_pytest.txt
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python -u tools/train_probe.py $BATCH > gpurun_out/${TAG}_prof.log 2>&1 || { tail -30 gpurun_out/${TAG}_prof.log; exit 1; }
grep "^it \|peak" gpurun_out/${TAG}_prof.log
head -25 gpurun_out/${TAG}_prof/run_kernel_stats.csv | cut -c1-220
