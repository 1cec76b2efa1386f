#!/bin/bash
# Round 6: conv3d_k3w with several tiles per workgroup (next tile's first step fetched under the
# current tile's last MFMAs, the epilogue after the next tile's first commit) vs the committed
# one-tile kernel: conv parity tests, interleaved kernel bench, config-4 step kernel trace A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_grad128.py tests/test_gpu_config3.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6an_pytest.txt 2>&1 || { tail -30 gpurun_out/r6an_pytest.txt; exit 1; }
tail -2 gpurun_out/r6an_pytest.txt
for rep in 1 2; do
  for spec in abv/libwf_c3w_head.so:1 waveformer_amd/libwaveformer_hip.so:1 waveformer_amd/libwaveformer_hip.so:2 waveformer_amd/libwaveformer_hip.so:4; do
    lib=${spec%%:*}; t=${spec#*:}
    echo "== $lib TPW=$t rep $rep"
    WAVEFORMER_HIP_LIB=$PWD/$lib WF_C3W_TPW=$t timeout -k 10 200 python3 tools/kbench_conv_ab.py || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r6an_kbench.txt || exit 1
bash tools/gpu_abk.sh r6an_tr tools/_trdrv.py 'conv3d_k3w' abv/libwf_c3w_head.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/r6an_tr_ab.txt
