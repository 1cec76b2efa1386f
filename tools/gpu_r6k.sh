#!/bin/bash
# Round 6: ATen device time of the config-4 step by origin; stitch wave-uniform batches.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6k}
timeout -k 10 300 python tools/train_native_probe.py > gpurun_out/${T}_native.txt 2>&1 || { tail -20 gpurun_out/${T}_native.txt; exit 1; }
head -50 gpurun_out/${T}_native.txt | cut -c1-220
timeout -k 10 400 python -u -m pytest tests/test_gpu_sliding_window.py tests/test_gpu_config3.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest.txt
timeout -k 10 300 python bench.py --workload sliding --steps 5 --warmup 2 > gpurun_out/${T}_sliding.json 2> gpurun_out/${T}_sliding.log || { tail -20 gpurun_out/${T}_sliding.log; exit 1; }
cut -c1-200 gpurun_out/${T}_sliding.json; grep -o '"sliding_window_stitch": {[^}]*}' gpurun_out/${T}_sliding.json
