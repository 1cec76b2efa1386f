#!/bin/bash
# bench + kernel trace + PMC (FETCH_SIZE / WRITE_SIZE) first, then the encoder parity suite
set -o pipefail
TAG=${1:-v9}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --batch 4 > gpurun_out/${TAG}_bench_b4.json 2> gpurun_out/${TAG}_bench_b4.err || exit 1
cat gpurun_out/${TAG}_bench_b4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --batch 4 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python bench.py --steps 2 --warmup 1 --batch 4 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python bench.py --steps 2 --warmup 1 --batch 4 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_pmc_write.log 2>&1 || exit 1
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write gpurun_out/${TAG}_pmc.json
timeout -k 10 560 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.txt
exit $rc
