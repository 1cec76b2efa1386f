#!/bin/bash
# Round 6 experiment: split-K on the PatchMerging gemm_kc launches (library-owned scratch, eager
# driver only), interleaved x3 against the current library.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
E=waveformer_amd/libwf_exp.so
bash tools/gpu_abk.sh r6ms tools/enc_drv.py 'gemm_kc' waveformer_amd/libwaveformer_hip.so "$E:WF_MERGE_SPLIT_EXP=1 WF_KC_SPLIT_ANY=1" "$E:WF_MERGE_SPLIT_EXP=1 WF_KC_SPLIT_ANY=1 WF_KC_SPLIT_MINSTEPS=3" > gpurun_out/r6ms_ab.txt 2>&1 || { tail -20 gpurun_out/r6ms_ab.txt; exit 1; }
grep -h "encoder B=" gpurun_out/r6ms_v*.log
