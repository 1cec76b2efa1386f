#!/bin/bash
# One GPU session: tests, bench variants, kernel-trace profile.  Usage: tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.txt
# test failures (1) still let the bench run; a crash, abort or time limit ends the call
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --batch 4 > gpurun_out/${TAG}_bench_b4.json 2> gpurun_out/${TAG}_bench_b4.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 8 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_bench_b8.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 4 --cpu-baseline 0 --parity 0 --precision bf16 > gpurun_out/${TAG}_bench_b4_bf16.json 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --batch 4 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_prof.log 2>&1
echo done
