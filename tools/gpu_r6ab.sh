#!/bin/bash
# Round 6: four-row msfuse (A/B x3 against the row kernel, WF_MSF_COAL=0) + parity tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=waveformer_amd/libwaveformer_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "msfuse or block or enc or full" --timeout 300 --timeout-method thread > gpurun_out/r6ab_pytest.txt 2>&1 || { tail -30 gpurun_out/r6ab_pytest.txt; exit 1; }
tail -2 gpurun_out/r6ab_pytest.txt
bash tools/gpu_abk.sh r6ab_msf tools/enc_drv.py 'msfuse' $L:WF_MSF_COAL=0 $L 2>&1 | tee gpurun_out/r6ab_msf_ab.txt
