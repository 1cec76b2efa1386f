#!/bin/bash
# A/B of gemm_lnw variant libraries under tools/lnw_stress.py (one process per library)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  WAVEFORMER_HIP_LIB=$PWD/abso/libwf_$v.so timeout -k 10 150 python -u tools/lnw_stress.py \
    > gpurun_out/lnw_$v.txt 2>&1 || { echo "variant $v failed rc=$?"; tail -5 gpurun_out/lnw_$v.txt; exit 1; }
  grep RESULT gpurun_out/lnw_$v.txt
done
