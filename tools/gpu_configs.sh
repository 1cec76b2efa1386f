#!/bin/bash
# The non-default bench lines on the current tree: config 5 (192^3 fp16 full model + HF),
# config 3 (sliding window), config 4 (train step, B=4).  Each under its own time limit;
# the first failure ends the script.   tools/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-cfg}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload full --img 192 --precision fp16 > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 1; }
cut -c1-400 gpurun_out/${TAG}_c5.json
timeout -k 10 400 python -u bench.py --workload sliding > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
cut -c1-400 gpurun_out/${TAG}_c3.json
timeout -k 10 500 python -u bench.py --workload train > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err || { tail -20 gpurun_out/${TAG}_c4.err; exit 1; }
cut -c1-400 gpurun_out/${TAG}_c4.json
