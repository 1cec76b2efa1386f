#!/bin/bash
# B=8 (new bench default): PMC traffic passes, then the default bench line (reads the PMC
# summary from profiles/), then the kernel trace of the same command
set -o pipefail
TAG=${1:-v11}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_pmc_write.log 2>&1 || exit 1
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write gpurun_out/${TAG}_pmc.json 8 || exit 1
cp gpurun_out/${TAG}_pmc.json profiles/r1_${TAG}_pmc.json
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
echo done
