#!/bin/bash
# Round 6: merge_res waves per workgroup 12 (shipped) / 8 / 6 / 4 (second pass), encoder driver kernel trace x3.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_abk.sh r6ap_mr tools/enc_drv.py 'merge_res' waveformer_amd/libwaveformer_hip.so abv/libwf_mr8.so abv/libwf_mr6.so abv/libwf_mr4.so 2>&1 | tee gpurun_out/r6ap_mr_ab.txt
