#!/bin/bash
# Round 6: gemm_tn on an XCD-contiguous grid: config-4 step A/B x3 (WF_TN_XCD=0 vs default) under
# a kernel trace (gemm_tn kernels), then the training tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=waveformer_amd/libwaveformer_hip.so
bash tools/gpu_abk.sh r6ag_tn tools/_trdrv.py 'gemm_tn_kernel' $L:WF_TN_XCD=0 $L 2>&1 | tee gpurun_out/r6ag_tn_ab.txt || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_grad128.py tests/test_gpu_ddp.py tests/test_train_grads.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6ag_pytest.txt 2>&1 || { tail -30 gpurun_out/r6ag_pytest.txt; exit 1; }
tail -2 gpurun_out/r6ag_pytest.txt
