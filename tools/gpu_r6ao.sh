#!/bin/bash
# Round 6: merge_res waves per workgroup 12 (shipped) / 16 / 8, encoder driver kernel trace x3.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_abk.sh r6ao_mr tools/enc_drv.py 'merge_res' waveformer_amd/libwaveformer_hip.so abv/libwf_mr16.so abv/libwf_mr8.so 2>&1 | tee gpurun_out/r6ao_mr_ab.txt
