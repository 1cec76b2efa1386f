#!/bin/bash
# Round 6: conv3d_k3w weights staged by LDS-DMA into a double buffer vs through registers
# : conv parity tests, interleaved kernel bench x3, config-4 step kernel trace A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_grad128.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6ak_pytest.txt 2>&1 || { tail -30 gpurun_out/r6ak_pytest.txt; exit 1; }
tail -2 gpurun_out/r6ak_pytest.txt
for rep in 1 2 3; do
  for lib in abv/libwf_c3wreg.so waveformer_amd/libwaveformer_hip.so; do
    echo "== $lib rep $rep"
    WAVEFORMER_HIP_LIB=$PWD/$lib timeout -k 10 200 python3 tools/kbench_conv_ab.py || exit 1
  done
done 2>&1 | tee gpurun_out/r6ak_kbench.txt || exit 1
bash tools/gpu_abk.sh r6ak_tr tools/_trdrv.py 'conv3d_k3' abv/libwf_c3wreg.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/r6ak_tr_ab.txt
