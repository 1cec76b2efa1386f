#!/bin/bash
# The round's committed measurements: replay-only kernel trace of the default encoder bench,
# the config-5 (192^3 fp16, HF refinement) line + its trace, the attention SQ / HBM counters,
# the FETCH / WRITE passes of the default bench at B = 8 (roofline.traffic) and the VALU pass
# (roofline.valu_issue_frac).  Counter passes run before the bench lines that read them only
# if their JSON summaries are copied into profiles/ first (a second call).
#   tools/gpu_profile_round.sh TAG
set -o pipefail
TAG=${1:-r3}
export TMPDIR=/tmp
mkdir -p gpurun_out
BQ="python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --parity 0 --graph 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- $BQ > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- $BQ > gpurun_out/${TAG}_pmc_write.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write gpurun_out/${TAG}_pmc.json 8 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_pmc_valu -o run -- $BQ > gpurun_out/${TAG}_pmc_valu.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_valu.log; exit 1; }
python tools/pmc_valu.py gpurun_out/${TAG}_pmc_valu gpurun_out/${TAG}_valu.json 8 | tee gpurun_out/${TAG}_valu.txt || exit 1
bash tools/pmc_attn.sh ${TAG}att > gpurun_out/${TAG}att_summary.txt 2>&1 || { tail -5 gpurun_out/${TAG}att_summary.txt; exit 1; }
bash tools/gpu_prof.sh ${TAG}enc > /dev/null || exit 1
bash tools/gpu_prof.sh ${TAG}c5 --workload full --img 192 --precision fp16 > /dev/null || exit 1
head -25 gpurun_out/${TAG}enc_kstats.txt
cat gpurun_out/${TAG}att_summary.txt
echo done
