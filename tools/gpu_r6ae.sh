#!/bin/bash
# Round 6: NCDHW IDWT with the XCD-aware (row, channel block) grid: tests, bench line rooflines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decoder.py -m gpu -x -q -k "idwt or IDWT or waverec or hf" --timeout 300 --timeout-method thread > gpurun_out/r6ae_pytest.txt 2>&1 || { tail -30 gpurun_out/r6ae_pytest.txt; exit 1; }
tail -2 gpurun_out/r6ae_pytest.txt
timeout -k 10 300 python bench.py --steps 30 --cpu-baseline 0 > gpurun_out/r6ae_bench.json 2> gpurun_out/r6ae_bench.err || { tail -20 gpurun_out/r6ae_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r6ae_bench.json').read().strip().splitlines()[-1])
print(round(d['value'],1)); [print(k, v.get('frac'), v.get('avg_launch_us')) for k, v in d['rooflines'].items()]"
