#!/bin/bash
# Round 6: cost of the fused InstanceNorm statistics (fp64 atomics) in conv3d_k3: kbench with
# STATS=1 / 0 interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for st in 1 0; do
    echo "== STATS=$st rep $rep"
    STATS=$st timeout -k 10 200 python3 tools/kbench_conv_ab.py || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r6al_stats.txt
