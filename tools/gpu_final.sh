#!/bin/bash
# round-end rehearsal on the final tree: the driver's three GPU steps in its order
set -o pipefail
TAG=${1:-final}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -20 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json
