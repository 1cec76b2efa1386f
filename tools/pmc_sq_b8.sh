#!/bin/bash
# SQ issue / wait / LDS counters of one kernel (regex $2) of the stage-1 CCF_FFN at B = 8 under
# tools/kbench_ffn.py, one rocprofv3 --pmc pass per counter set; prints means per launch.
set -o pipefail
TAG=$1; RX=$2
export TMPDIR=/tmp B=${B:-8} ITERS=${ITERS:-6}
mkdir -p gpurun_out
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python tools/kbench_ffn.py > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done
python tools/pmc_summary_sq.py gpurun_out/${TAG}_p "$RX"
