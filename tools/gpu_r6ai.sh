#!/bin/bash
# Round 6: norm_act backward apply with a fixed channel quad per thread (A/B x3 under the
# config-4 step vs the committed build) + training tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_abk.sh r6ai_na tools/_trdrv.py 'norm_act_bwd' abv/libwf_naold.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/r6ai_na_ab.txt || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_grad128.py tests/test_gpu_ddp.py tests/test_train_grads.py tests/test_gpu_decoder.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6ai_pytest.txt 2>&1 || { tail -30 gpurun_out/r6ai_pytest.txt; exit 1; }
tail -2 gpurun_out/r6ai_pytest.txt
