#!/bin/bash
# Round 6: the kept gemm_kc change (6-tile chunks for costly loaders, split-K on the stage-4 fc)
# against the HEAD build, interleaved x3 under the encoder driver; then the final-tree steps.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_abk.sh r6ks4 tools/enc_drv.py 'gemm_kc' waveformer_amd/libwf_base.so waveformer_amd/libwaveformer_hip.so "waveformer_amd/libwaveformer_hip.so:WF_KC_NTMAX=12 WF_KC_GELU_WIDE=1" > gpurun_out/r6ks4_ab.txt 2>&1 || { tail -20 gpurun_out/r6ks4_ab.txt; exit 1; }
grep -h "encoder B=" gpurun_out/r6ks4_v*.log
bash tools/gpu_final.sh r6ks4
