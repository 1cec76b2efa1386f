#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ITERS=5 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/kt -o run -- python tools/kbench_ffn.py > gpurun_out/pmc/kt.log 2>&1 || exit 1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" ; do
  i=$((i+1))
  ITERS=3 timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python tools/kbench_ffn.py > gpurun_out/pmc/p$i.log 2>&1 || echo "pmc set $i failed: $set"
done
echo pmc done
