#!/bin/bash
# Round 6: depthwise-conv z-segment length at the stage-3 / 4 shapes (768 workgroups = 1.5
# residency rounds at 2 per CU): interleaved A/B x3 under the encoder driver.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=waveformer_amd/libwaveformer_hip.so
bash tools/gpu_abk.sh r6dz tools/enc_drv.py 'dwconv3d' $L "$L:WF_DW_ZS=16" "$L:WF_DW_ZS=4" > gpurun_out/r6dz_ab.txt 2>&1 || { tail -20 gpurun_out/r6dz_ab.txt; exit 1; }
cat gpurun_out/r6dz_ab.txt
