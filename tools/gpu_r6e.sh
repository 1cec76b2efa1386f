#!/bin/bash
# Round 6: full GPU suite, attention A/B (round 5 / one sub-tile / query pairs), config-4 bench
# line + kernel trace, config-3 stitch / DWT rooflines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6e_pytest.txt 2>&1 || { tail -40 gpurun_out/r6e_pytest.txt; exit 1; }
tail -3 gpurun_out/r6e_pytest.txt
bash tools/gpu_abk.sh r6e_attn tools/kbench_attn.py attn_tbl abv/libwf_r5.so abv/libwf_qp0.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/r6e_attn_ab.txt || exit 1
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 > gpurun_out/r6e_train.json 2> gpurun_out/r6e_train.log || { tail -20 gpurun_out/r6e_train.log; exit 1; }
cat gpurun_out/r6e_train.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6e_trtrace -o run -- python bench.py --workload train --steps 4 --warmup 2 > gpurun_out/r6e_trtrace.log 2>&1 || { tail -20 gpurun_out/r6e_trtrace.log; exit 1; }
f=$(ls gpurun_out/r6e_trtrace/*kernel_trace.csv | head -1); python tools/kstats.py $f 45 > gpurun_out/r6e_train_kstats.txt; head -50 gpurun_out/r6e_train_kstats.txt
echo "Cijk launches: $(grep -c Cijk $f)"
timeout -k 10 300 python bench.py --workload sliding --steps 5 --warmup 2 > gpurun_out/r6e_sliding.json 2> gpurun_out/r6e_sliding.log || { tail -20 gpurun_out/r6e_sliding.log; exit 1; }
cat gpurun_out/r6e_sliding.json
