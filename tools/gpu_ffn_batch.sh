#!/bin/bash
# stage-1 CCF_FFN kernel times per batch size (does h1 stay in the Infinity Cache at small B?)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 1 2 4 8; do
  B=$b ITERS=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ffnb_$b -o run -- python tools/kbench_ffn.py > gpurun_out/ffnb_$b.log 2>&1 || { tail -20 gpurun_out/ffnb_$b.log; exit 1; }
  echo "== B=$b"; grep ccf_ffn gpurun_out/ffnb_$b.log
  f=$(ls gpurun_out/ffnb_$b/*kernel_trace.csv | head -1); python tools/kstats.py $f 4
done
