#!/bin/bash
# Round 6: SQ pass over the decoder convolutions at the config-3/4 shapes (bf16x3).
set -o pipefail
export TMPDIR=/tmp ITERS=2
export SHAPES="bf16x3,4,48,48,128;bf16x3,4,96,48,128;bf16x3,4,96,96,64"
mkdir -p gpurun_out
bash tools/pmc_sq_kernels.sh r6ah_conv 'conv3d_k3' tools/kbench_conv_shapes.py 2>&1 | tee gpurun_out/r6ah_conv_sq.txt
