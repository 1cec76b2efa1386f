#!/bin/bash
# Round 6: the wide-chunk conv at 48 input channels under bf16x3 (WF_CONV_WIDE_MINCIN), A/B x3.
set -o pipefail
export TMPDIR=/tmp ONLY=3,4 ITERS=8
mkdir -p gpurun_out
for r in 1 2 3; do
  echo "== default"; timeout -k 10 120 python tools/kbench_conv_ab.py || exit 1
  echo "== wide at Cin >= 8"; WF_CONV_WIDE_MINCIN=8 timeout -k 10 120 python tools/kbench_conv_ab.py || exit 1
done
