#!/bin/bash
# What the driver runs at round end: smoke(), then the default bench (N=1, no flags).
set -o pipefail
TAG=${1:-dr}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${TAG}_smoke.txt 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
start=$(date +%s)
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - start )) s"
python tools/bench_line.py gpurun_out/${TAG}_bench.json
