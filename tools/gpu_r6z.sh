#!/bin/bash
# Round 6: gemm_kc prefetch depth 4 on small grids (A/B x3 against WF_KC_PD=2 under the encoder
# driver) + parity tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_abk.sh r6z_kc tools/enc_drv.py 'gemm_kc' waveformer_amd/libwaveformer_hip.so:WF_KC_PD=2 waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/r6z_kc_ab.txt || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_config.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6z_pytest.txt 2>&1 || { tail -30 gpurun_out/r6z_pytest.txt; exit 1; }
tail -2 gpurun_out/r6z_pytest.txt
