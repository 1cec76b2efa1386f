#!/bin/bash
# Round 6: dot2 probe, parity file, attention + stage-1 FFN A/B against the round-5 library.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/bin/probe_dot2 > gpurun_out/r6c_probe.txt 2>&1; cat gpurun_out/r6c_probe.txt; grep -q "SGPR-constant form 0 of" gpurun_out/r6c_probe.txt || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r6c_pytest.txt 2>&1 || { tail -30 gpurun_out/r6c_pytest.txt; exit 1; }
tail -3 gpurun_out/r6c_pytest.txt
bash tools/gpu_abk.sh r6c_attn tools/kbench_attn.py attn_tbl abv/libwf_r5.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/r6c_attn_ab.txt || exit 1
B=8 C=48 S=64 ITERS=10 bash tools/gpu_abk.sh r6c_ffn tools/kbench_ffn.py tb4 abv/libwf_r5.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/r6c_ffn_ab.txt
