#!/bin/bash
# Round 6: gemm_kc column-chunk width x split-K on the small-grid shapes (stages 3 / 4):
# interleaved A/B x3 under the encoder driver.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=waveformer_amd/libwf_ks.so
bash tools/gpu_abk.sh r6ks2 tools/enc_drv.py 'gemm_kc' "$L:WF_KC_SPLIT=1" "$L:WF_KC_SPLIT=1 WF_KC_MINNT=6" "$L:WF_KC_MINNT=6" "$L:WF_KC_MINNT=8" 2>&1 | tee gpurun_out/r6ks2_ab.txt
