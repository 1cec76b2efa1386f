#!/bin/bash
# Round 6: conv3d_k3 fused statistics: fp64 atomics removed (timing-only build) vs shipped,
# both with STATS=1, plus STATS=0 on the shipped build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for spec in abv/libwf_noatom.so:1 waveformer_amd/libwaveformer_hip.so:1 waveformer_amd/libwaveformer_hip.so:0; do
    lib=${spec%%:*}; st=${spec#*:}
    echo "== $lib STATS=$st rep $rep"
    WAVEFORMER_HIP_LIB=$PWD/$lib STATS=$st timeout -k 10 200 python3 tools/kbench_conv_ab.py || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r6am_noatom.txt
