#!/bin/bash
# Round 6: config-4 ATen folds (unbound DWT bands, no materialized workspace gradients, DiceCE
# one-hot / sums, cached index grouping): full GPU suite, train line, ATen attribution, trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6l}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest.txt
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 > gpurun_out/${T}_train.json 2> gpurun_out/${T}_train.log || { tail -20 gpurun_out/${T}_train.log; exit 1; }
cut -c1-330 gpurun_out/${T}_train.json
timeout -k 10 300 python tools/train_native_probe.py > gpurun_out/${T}_native.txt 2>&1 || { tail -20 gpurun_out/${T}_native.txt; exit 1; }
head -30 gpurun_out/${T}_native.txt | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trtrace -o run -- python bench.py --workload train --steps 4 --warmup 2 > gpurun_out/${T}_trtrace.log 2>&1 || { tail -20 gpurun_out/${T}_trtrace.log; exit 1; }
f=$(ls gpurun_out/${T}_trtrace/*kernel_trace.csv | head -1); python tools/kstats.py $f 60 > gpurun_out/${T}_train_kstats.txt; head -5 gpurun_out/${T}_train_kstats.txt
echo "Cijk launches: $(grep -c Cijk $f || true)"
