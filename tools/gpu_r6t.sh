#!/bin/bash
# Round 6: config-4 and config-3 lines after the conv / wgrad changes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6t}
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 > gpurun_out/${T}_train.json 2> gpurun_out/${T}_train.log || { tail -20 gpurun_out/${T}_train.log; exit 1; }
cut -c1-330 gpurun_out/${T}_train.json
timeout -k 10 300 python bench.py --workload sliding --steps 5 --warmup 2 > gpurun_out/${T}_sliding.json 2> gpurun_out/${T}_sliding.log || { tail -20 gpurun_out/${T}_sliding.log; exit 1; }
cut -c1-200 gpurun_out/${T}_sliding.json; grep -o '"conv3d_k3": {[^}]*}' gpurun_out/${T}_sliding.json
