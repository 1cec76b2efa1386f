#!/bin/bash
# A/B of the fused FFN back halves between library builds: stage-1 (C 48, 64^3) and stage-2
# (C 96, 32^3) B = 8 launches under a kernel trace, alternated.  usage: gpu_ffn_ab.sh TAG A.so B.so
set -o pipefail
TAG=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    WAVEFORMER_HIP_LIB=$PWD/$lib KC=48 KS=64 DBGS=0 bash tools/gpu_dwfc2_phases.sh ${TAG}_${n}_s1_$rep | sed "s/^/$n stage1 /" || exit 1
    WAVEFORMER_HIP_LIB=$PWD/$lib KC=96 KS=32 DBGS=0 bash tools/gpu_dwfc2_phases.sh ${TAG}_${n}_s2_$rep | sed "s/^/$n stage2 /" || exit 1
  done
done
