#!/bin/bash
# Round 6, first GPU call: stage-1 FFN parity with the swizzled tb4 h2 rows, an interleaved A/B
# against the round-5 library, and SQ counters of the FFN back halves (tb4 + ffn_dwfc2).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "ccf_ffn_stage1 or ccf_ffn_stage2" > gpurun_out/r6b_pytest.txt 2>&1 || { tail -30 gpurun_out/r6b_pytest.txt; exit 1; }
tail -3 gpurun_out/r6b_pytest.txt
bash tools/gpu_ab3.sh r6b_tb4 abv/libwf_r5.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/r6b_tb4_ab.txt || exit 1
bash tools/pmc_sq_kernels.sh r6b_sq "ffn_dwfc_tb4" 2>&1 | tee gpurun_out/r6b_sq.txt
