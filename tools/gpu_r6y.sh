#!/bin/bash
# Round 6 final tree: the driver's steps (GPU tests, smoke, default bench), the default bench
# under a kernel trace (its rocprof summary), and the config 3 / 4 / 5 lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6y}
bash tools/gpu_final.sh ${T} || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_benchprof -o run -- python bench.py > gpurun_out/${T}_benchprof.json 2> gpurun_out/${T}_benchprof.log || { tail -20 gpurun_out/${T}_benchprof.log; exit 1; }
cut -c1-200 gpurun_out/${T}_benchprof.json
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 > gpurun_out/${T}_train.json 2> gpurun_out/${T}_train.log || { tail -20 gpurun_out/${T}_train.log; exit 1; }
cut -c1-250 gpurun_out/${T}_train.json
timeout -k 10 300 python bench.py --workload sliding --steps 5 --warmup 2 > gpurun_out/${T}_sliding.json 2> gpurun_out/${T}_sliding.log || { tail -20 gpurun_out/${T}_sliding.log; exit 1; }
cut -c1-200 gpurun_out/${T}_sliding.json
timeout -k 10 400 python bench.py --workload full --img 192 --precision fp16 > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.log || { tail -20 gpurun_out/${T}_c5.log; exit 1; }
cut -c1-200 gpurun_out/${T}_c5.json
