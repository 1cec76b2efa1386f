#!/bin/bash
# Round 6 final tree: FETCH / WRITE / VALU counter passes of the default bench (the PMC summaries
# bench.py reads for roofline.traffic / valu_issue_frac).
set -o pipefail
TAG=${1:-r6z}
export TMPDIR=/tmp
mkdir -p gpurun_out
BQ="python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --parity 0 --graph 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- $BQ > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- $BQ > gpurun_out/${TAG}_pmc_write.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write gpurun_out/${TAG}_pmc.json 8 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_pmc_valu -o run -- $BQ > gpurun_out/${TAG}_pmc_valu.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_valu.log; exit 1; }
python tools/pmc_valu.py gpurun_out/${TAG}_pmc_valu gpurun_out/${TAG}_valu.json 8 | tee gpurun_out/${TAG}_valu.txt || exit 1
