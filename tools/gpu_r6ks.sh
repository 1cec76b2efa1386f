#!/bin/bash
# Round 6: gemm_kc split-K on the small-grid CCF_FFN fc (stages 3 / 4): interleaved A/B x3 under
# the encoder driver (WF_KC_SPLIT=1 = no split) + parity tests on the split-K build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_abk.sh r6ks tools/enc_drv.py 'gemm_kc' waveformer_amd/libwf_ks.so:WF_KC_SPLIT=1 waveformer_amd/libwf_ks.so 2>&1 | tee gpurun_out/r6ks_ab.txt || exit 1
WAVEFORMER_HIP_LIB=$PWD/waveformer_amd/libwf_ks.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_config.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6ks_pytest.txt 2>&1 || { tail -30 gpurun_out/r6ks_pytest.txt; exit 1; }
tail -2 gpurun_out/r6ks_pytest.txt
