#!/bin/bash
# A/B of environment settings on one kernel driver: tools/gpu_envab.sh TAG DRIVER.py "ENV1" "ENV2" ...
# (each setting in its own process under rocprofv3 --kernel-trace; kstats per setting)
set -o pipefail
TAG=$1; DRV=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$i -o run -- python $DRV > gpurun_out/${TAG}_$i.log 2>&1 || { tail -20 gpurun_out/${TAG}_$i.log; exit 1; }
  echo "== $e"
  f=$(ls gpurun_out/${TAG}_$i/*kernel_trace.csv | head -1); python tools/kstats.py $f ${NK:-3}
done
