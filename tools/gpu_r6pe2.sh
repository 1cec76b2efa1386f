#!/bin/bash
# Round 6: PatchEmbed + LL v2 (no LDS row tile) -- parity first, then interleaved A/B x3 against
# the v1 row-tile kernel (WF_PE_LL_V1=1), then the final-tree steps.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "patch_embed_ll or hf_skip" tests/test_gpu_bench_config.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6pe2_pytest1.txt 2>&1 || { tail -30 gpurun_out/r6pe2_pytest1.txt; exit 1; }
tail -1 gpurun_out/r6pe2_pytest1.txt
L=waveformer_amd/libwaveformer_hip.so
bash tools/gpu_abk.sh r6pe2 tools/enc_drv.py 'patch_embed' "$L:WF_PE_LL_V1=1" $L > gpurun_out/r6pe2_ab.txt 2>&1 || { tail -20 gpurun_out/r6pe2_ab.txt; exit 1; }
cat gpurun_out/r6pe2_ab.txt
bash tools/gpu_final.sh r6pe2
