#!/bin/bash
# parity of the gemm_rows 12-wave / gemm_kc deep-prefetch variants, then a kernel-trace A/B of the encoder
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
WF_ROWS_WAVES=12 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_config.py tests/test_gpu_determinism.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab1_pytest.txt 2>&1 || { tail -20 gpurun_out/ab1_pytest.txt; exit 1; }
tail -1 gpurun_out/ab1_pytest.txt
bash tools/gpu_envab.sh ab1 tools/enc_drv.py "WF_KC_DEPTH=1" "WF_KC_DEPTH=3" "WF_ROWS_WAVES=12" 
