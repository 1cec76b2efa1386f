#!/bin/bash
# Round 6: full GPU suite, attention A/B (round 5 / one sub-tile / query pairs), encoder bench
# + replay trace, config-4 bench line + kernel trace, config-3 line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6f}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -3 gpurun_out/${T}_pytest.txt
bash tools/gpu_abk.sh ${T}_attn tools/kbench_attn.py attn_tbl abv/libwf_r5.so abv/libwf_qp0.so waveformer_amd/libwaveformer_hip.so 2>&1 | tee gpurun_out/${T}_attn_ab.txt || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { tail -20 gpurun_out/${T}_bench.log; exit 1; }
cut -c1-400 gpurun_out/${T}_bench.json
bash tools/gpu_prof.sh ${T}_enc > gpurun_out/${T}_enc_prof.txt 2>&1 || { tail -20 gpurun_out/${T}_enc_prof.txt; exit 1; }
head -40 gpurun_out/${T}_enc_kstats.txt
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 > gpurun_out/${T}_train.json 2> gpurun_out/${T}_train.log || { tail -20 gpurun_out/${T}_train.log; exit 1; }
cat gpurun_out/${T}_train.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trtrace -o run -- python bench.py --workload train --steps 4 --warmup 2 > gpurun_out/${T}_trtrace.log 2>&1 || { tail -20 gpurun_out/${T}_trtrace.log; exit 1; }
f=$(ls gpurun_out/${T}_trtrace/*kernel_trace.csv | head -1); python tools/kstats.py $f 45 > gpurun_out/${T}_train_kstats.txt; head -30 gpurun_out/${T}_train_kstats.txt
echo "Cijk launches: $(grep -c Cijk $f)"
timeout -k 10 300 python bench.py --workload sliding --steps 5 --warmup 2 > gpurun_out/${T}_sliding.json 2> gpurun_out/${T}_sliding.log || { tail -20 gpurun_out/${T}_sliding.log; exit 1; }
cat gpurun_out/${T}_sliding.json
