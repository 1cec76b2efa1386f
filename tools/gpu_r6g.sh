#!/bin/bash
# Round 6: full GPU suite; config-4 line, trace and library-GEMM probe; config-3 line; encoder line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6g}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -3 gpurun_out/${T}_pytest.txt
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 > gpurun_out/${T}_train.json 2> gpurun_out/${T}_train.log || { tail -20 gpurun_out/${T}_train.log; exit 1; }
cut -c1-330 gpurun_out/${T}_train.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trtrace -o run -- python bench.py --workload train --steps 4 --warmup 2 > gpurun_out/${T}_trtrace.log 2>&1 || { tail -20 gpurun_out/${T}_trtrace.log; exit 1; }
f=$(ls gpurun_out/${T}_trtrace/*kernel_trace.csv | head -1); python tools/kstats.py $f 60 > gpurun_out/${T}_train_kstats.txt; head -12 gpurun_out/${T}_train_kstats.txt
echo "Cijk launches: $(grep -c Cijk $f || true)"
timeout -k 10 300 python tools/train_mm_probe.py > gpurun_out/${T}_mm_probe.txt 2>&1 || { tail -20 gpurun_out/${T}_mm_probe.txt; exit 1; }
head -30 gpurun_out/${T}_mm_probe.txt
timeout -k 10 300 python bench.py --workload sliding --steps 5 --warmup 2 > gpurun_out/${T}_sliding.json 2> gpurun_out/${T}_sliding.log || { tail -20 gpurun_out/${T}_sliding.log; exit 1; }
cut -c1-300 gpurun_out/${T}_sliding.json; grep -o '"sliding_window_stitch": {[^}]*}' gpurun_out/${T}_sliding.json
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { tail -20 gpurun_out/${T}_bench.log; exit 1; }
cut -c1-300 gpurun_out/${T}_bench.json
