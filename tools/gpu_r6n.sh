#!/bin/bash
# Round 6: attention row sums on the VALU (A/B) + its parity under the attention tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6n}
bash tools/gpu_abk.sh ${T}_attn tools/kbench_attn.py attn_tbl abv/libwf_attn_vsum.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/${T}_attn_ab.txt || exit 1
WAVEFORMER_HIP_LIB=$PWD/abv/libwf_attn_vsum.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "attn or attention or block or enc" --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest.txt
