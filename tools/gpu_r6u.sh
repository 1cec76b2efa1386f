#!/bin/bash
# Round 6: attention with four query sub-tiles per wave (A/B x3); ffn_dwfc2 LN2 on eight waves
# (A/B x3, stage-2 shape); proj_out tile pitch (SQ of the proj_out launches) + parity tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_abk.sh r6u_attn tools/kbench_attn.py attn_tbl abv/libwf_attn_nq4.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/r6u_attn_ab.txt || exit 1
B=8 C=96 S=32 ITERS=10 bash tools/gpu_abk.sh r6u_dw2 tools/kbench_ffn.py ffn_dwfc2 abv/libwf_dwfc2_ln4.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/r6u_dwfc2_ab.txt || exit 1
bash tools/pmc_sq_kernels.sh r6u_sq 'proj_out|ffn_dwfc2' 2>&1 | tee gpurun_out/r6u_sq.txt || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6u_pytest.txt 2>&1 || { tail -30 gpurun_out/r6u_pytest.txt; exit 1; }
tail -2 gpurun_out/r6u_pytest.txt
