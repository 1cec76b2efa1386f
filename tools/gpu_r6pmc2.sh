#!/bin/bash
# Round 6 end: FETCH_SIZE / WRITE_SIZE passes (separate runs) of the encoder driver on the final
# tree, summarised per kernel by tools/pmc_traffic.py (the late-round kernels: patch_embed_ll v2,
# the split-K gemm_kc, the narrow depthwise conv).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ITERS=2 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r6pmc2_fetch -o run -- python3 tools/enc_drv.py > gpurun_out/r6pmc2_fetch.log 2>&1 || { tail -5 gpurun_out/r6pmc2_fetch.log; exit 1; }
ITERS=2 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r6pmc2_write -o run -- python3 tools/enc_drv.py > gpurun_out/r6pmc2_write.log 2>&1 || { tail -5 gpurun_out/r6pmc2_write.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/r6pmc2_fetch gpurun_out/r6pmc2_write gpurun_out/r6pmc2_pmc.json 8
