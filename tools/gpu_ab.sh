#!/bin/bash
# A/B of library variants on one kernel driver: tools/gpu_ab.sh TAG DRIVER.py VAR1.so VAR2.so ...
# (rocprofv3 kernel trace per variant, kstats summary per variant; env passes through)
set -o pipefail
TAG=$1; DRV=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for so in "$@"; do
  n=$(basename $so .so)
  WAVEFORMER_HIP_LIB=$PWD/$so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$n -o run -- python $DRV > gpurun_out/${TAG}_$n.log 2>&1 || { tail -20 gpurun_out/${TAG}_$n.log; exit 1; }
  echo "== $n"; tail -2 gpurun_out/${TAG}_$n.log
  f=$(ls gpurun_out/${TAG}_$n/*kernel_trace.csv | head -1); python tools/kstats.py $f ${NK:-8}
done
