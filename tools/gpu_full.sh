#!/bin/bash
# Round checkpoint on one GPU: full -m gpu suite, bench (B=4 with cpu_baseline + parity),
# kernel-trace profile, and FETCH_SIZE / WRITE_SIZE PMC passes -> profiles/TAG_pmc.json.
#   tools/gpu_full.sh TAG
set -o pipefail
TAG=${1:-full}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_pmc_write.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write gpurun_out/${TAG}_pmc.json
echo done
