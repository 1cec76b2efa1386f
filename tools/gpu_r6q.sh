#!/bin/bash
# Round 6: wide conv at 48 / 96 channels under bf16x3 at the config-4 shapes (A/B x3);
# wgrad with the dot2 split (A/B vs the committed build) + its SQ pass.
set -o pipefail
export TMPDIR=/tmp ITERS=6
export SHAPES="bf16x3,4,48,48,128;bf16x3,4,96,48,128;bf16x3,4,96,96,64;bf16x3,4,192,96,64;bf16x3,4,48,48,64"
mkdir -p gpurun_out
for r in 1 2 3; do
  echo "== new gating"; timeout -k 10 120 python tools/kbench_conv_shapes.py || exit 1
  echo "== round-5 gating (Cin >= 89)"; WF_CONV_WIDE_MINCIN=89 timeout -k 10 120 python tools/kbench_conv_shapes.py || exit 1
done
for r in 1 2 3; do
  echo "== wgrad dot2 split"; timeout -k 10 120 python tools/kbench_wgrad.py 4 || exit 1
  echo "== wgrad committed"; WAVEFORMER_HIP_LIB=$PWD/abv/libwf_wgrad_old.so timeout -k 10 120 python tools/kbench_wgrad.py 4 || exit 1
done
bash tools/pmc_sq_kernels.sh r6q_wg 'conv3d_wgrad|conv3d_k3' tools/kbench_wgrad.py
