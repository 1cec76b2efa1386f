#!/bin/bash
# The round's committed measurements: replay-only kernel trace of the default encoder bench,
# the config-5 (192^3 fp16, HF refinement) line + its trace, the attention SQ / HBM counters,
# and the FETCH / WRITE passes of the default bench at B = 8 (roofline.traffic).
#   tools/gpu_profile_round.sh TAG
set -o pipefail
TAG=${1:-r2}
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_prof.sh ${TAG}enc || exit 1
bash tools/gpu_prof.sh ${TAG}c5 --workload full --img 192 --precision fp16 || exit 1
timeout -k 10 300 python bench.py --workload full --img 192 --precision fp16 > gpurun_out/${TAG}_c5_bench.json 2> gpurun_out/${TAG}_c5_bench.err || { tail -5 gpurun_out/${TAG}_c5_bench.err; exit 1; }
bash tools/pmc_attn.sh ${TAG}att > gpurun_out/${TAG}att_summary.txt 2>&1 || { tail -5 gpurun_out/${TAG}att_summary.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_pmc_write.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write gpurun_out/${TAG}_pmc.json 8
cat gpurun_out/${TAG}att_summary.txt
echo done
