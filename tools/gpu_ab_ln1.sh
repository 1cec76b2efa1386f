#!/bin/bash
# encoder parity + A/B of the split pwconv LayerNorm (stages 3/4)
set -o pipefail
TAG=${1:-ab}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_train_grads.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_new.json 2>/dev/null || exit 1
WF_FFN_NO_SPLIT_LN1=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_old.json 2>/dev/null || exit 1
python -c "
import json
for n in ('new','old'):
    d=json.load(open('gpurun_out/${TAG}_'+n+'.json')); print(n, round(d['value'],1), round(d['ms_per_step'],3))"
