#!/bin/bash
# Round evidence on one GPU, in the order the bench line needs it:
#   1. FETCH_SIZE / WRITE_SIZE PMC passes of the default bench (eager launches, B = 8)
#      -> profiles/TAG_pmc.json (bench.py reads roofline.traffic from it)
#   2. the default bench line (parity + cpu_baseline) -> gpurun_out/TAG_bench.json
#   3. a replay-only kernel trace + summary (tools/gpu_prof.sh) -> gpurun_out/TAG_kstats.txt
#   tools/gpu_evidence.sh TAG
set -o pipefail
TAG=${1:-evidence}
export TMPDIR=/tmp
mkdir -p gpurun_out profiles
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --parity 0 --graph 0 --op-timers 0 > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --parity 0 --graph 0 --op-timers 0 > gpurun_out/${TAG}_pmc_write.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write profiles/${TAG}_pmc.json 8 || exit 1
cp profiles/${TAG}_pmc.json gpurun_out/
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
bash tools/gpu_prof.sh ${TAG} > /dev/null || exit 1
head -12 gpurun_out/${TAG}_kstats.txt
