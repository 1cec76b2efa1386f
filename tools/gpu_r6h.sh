#!/bin/bash
# Round 6: full GPU suite; attention staging A/B; which GEMMs of the train step still fall back.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6h}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest.txt
bash tools/gpu_abk.sh ${T}_attn tools/kbench_attn.py attn_tbl abv/libwf_attn_head.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/${T}_attn_ab.txt || exit 1
WF_GEMM_FALLBACK_TRACE=1 timeout -k 10 300 python tools/train_mm_probe.py > gpurun_out/${T}_mm_probe.txt 2>&1 || { tail -20 gpurun_out/${T}_mm_probe.txt; exit 1; }
grep -B2 -A8 "GEMM fallback" gpurun_out/${T}_mm_probe.txt | head -60
bash tools/gpu_abk.sh ${T}_nt tools/enc_drv.py 'gemm_rows' abv/libwf_ntstore.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/${T}_nt_ab.txt || exit 1
timeout -k 10 300 python bench.py --workload sliding --steps 5 --warmup 2 > gpurun_out/${T}_sliding.json 2> gpurun_out/${T}_sliding.log || { tail -20 gpurun_out/${T}_sliding.log; exit 1; }
cut -c1-300 gpurun_out/${T}_sliding.json; grep -o '"sliding_window_stitch": {[^}]*}' gpurun_out/${T}_sliding.json
