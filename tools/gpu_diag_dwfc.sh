#!/bin/bash
# dwfc z-segment length A/B (WF_DWFC_MINBLK) and phase attribution (WF_DWFC_DIAG)
set -o pipefail
export TMPDIR=/tmp
for mb in 1024 512 256 2048; do
  echo "minblk=$mb"
  WF_DWFC_MINBLK=$mb ITERS=30 timeout -k 10 120 python tools/kbench_ffn.py 2>&1 | tail -1 || exit 1
done
for mb in 1024 512; do
  echo "minblk=$mb diag=15"
  WF_DWFC_DIAG=15 WF_DWFC_MINBLK=$mb ITERS=30 timeout -k 10 120 python tools/kbench_ffn.py 2>&1 | tail -1 || exit 1
done
