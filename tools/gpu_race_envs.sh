#!/bin/bash
# concurrent two-stream encoder forwards (tools/race_arena.py, separate modules) under the
# library's A/B switches: which kernel's replacement makes the concurrent runs exact?
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for e in "WF_X=0" "WF_FFN_DWFC_CLASSIC=1" "WF_ATTN_TILED=1" "WF_GEMM_NO_LNW=1" "WF_PE_ONESHOT=1" "WF_GEMM_NO_KC=1"; do
  env $e ONLY_SEP=1 REPS=4 timeout -k 10 200 python -u tools/race_arena.py > gpurun_out/race_env.txt 2>&1 || { tail -5 gpurun_out/race_env.txt; exit 1; }
  echo "$e: $(grep 'runs differ' gpurun_out/race_env.txt)"
done
