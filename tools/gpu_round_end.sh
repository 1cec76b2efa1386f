#!/bin/bash
# Round-end evidence on the final tree: the driver's three GPU steps (pytest -m gpu, smoke,
# bench), a rocprofv3 kernel-trace + stats run of the bench command, then configs 5 / 3 / 4.
#   tools/gpu_round_end.sh TAG
set -o pipefail
TAG=${1:-end}
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_final.sh ${TAG} || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --cpu-baseline 0 > gpurun_out/${TAG}_bench_under_rocprof.json 2> gpurun_out/${TAG}_prof.err || { tail -20 gpurun_out/${TAG}_prof.err; exit 1; }
cut -c1-200 gpurun_out/${TAG}_bench_under_rocprof.json
bash tools/gpu_configs.sh ${TAG}
