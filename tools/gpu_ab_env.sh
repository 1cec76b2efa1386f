#!/bin/bash
# A/B of env-selected kernel variants: pytest -k selection once, then one bench per variant
#   tools/gpu_ab_env.sh TAG "pytest -k" "VAR=a" "VAR=b" ...
set -o pipefail
TAG=$1; SEL=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu -k "$SEL" > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.txt
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_b$i.json 2> gpurun_out/${TAG}_b$i.err || { tail -20 gpurun_out/${TAG}_b$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_b$i.json')); r=d['roofline']; print('$v', round(d['value'],1), 'vol/s', r['kernel'], r['avg_launch_us'], 'us', r['frac'])"
done
