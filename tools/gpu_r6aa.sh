#!/bin/bash
# Round 6: stage-3/4 depthwise z-segment length (WF_DW_ZSMIN 8 / 4 / 2), A/B x3 under the encoder.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=waveformer_amd/libwaveformer_hip.so
bash tools/gpu_abk.sh r6aa_dw tools/enc_drv.py 'dwconv3d' $L $L:WF_DW_ZSMIN=4 $L:WF_DW_ZSMIN=2 2>&1 | tee gpurun_out/r6aa_dw_ab.txt
