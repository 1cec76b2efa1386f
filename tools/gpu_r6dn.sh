#!/bin/bash
# Round 6: depthwise conv 64-channel x 8-column tiles on narrow volumes (stage 4, W = 8):
# interleaved A/B x3 (WF_DW_NARROW=0: the 32 x 16 tiles) under the encoder driver, then tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=waveformer_amd/libwaveformer_hip.so
bash tools/gpu_abk.sh r6dn tools/enc_drv.py 'dwconv3d' "$L:WF_DW_NARROW=0" $L > gpurun_out/r6dn_ab.txt 2>&1 || { tail -20 gpurun_out/r6dn_ab.txt; exit 1; }
cat gpurun_out/r6dn_ab.txt
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6dn_pytest.txt 2>&1 || { tail -30 gpurun_out/r6dn_pytest.txt; exit 1; }
tail -1 gpurun_out/r6dn_pytest.txt
