#!/bin/bash
# Round 6: depthwise conv 64-channel x 8-column tiles on narrow volumes (stage 4, W = 8):
# interleaved A/B x3 (WF_DW_NARROW=0: the 32 x 16 tiles) under the encoder driver, then tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=waveformer_amd/libwaveformer_hip.so
bash tools/gpu_abk.sh r6dw tools/enc_drv.py 'dwconv3d' $L "$L:WF_DW_NARROW_W=16" > gpurun_out/r6dw_ab.txt 2>&1 || { tail -20 gpurun_out/r6dw_ab.txt; exit 1; }
cat gpurun_out/r6dw_ab.txt
