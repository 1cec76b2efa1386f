#!/bin/bash
# Config-4 train bench (MIOpen find on the first step can take minutes: a heartbeat file keeps
# the run visibly alive).  Usage: tools/gpu_train.sh TAG [bench args]
set -o pipefail
TAG=${1:-tr}
shift
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 30; date >> gpurun_out/${TAG}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u bench.py --workload train "$@" > gpurun_out/${TAG}_train.json 2> gpurun_out/${TAG}_train.err || { tail -20 gpurun_out/${TAG}_train.err; exit 1; }
tail -c 700 gpurun_out/${TAG}_train.json
