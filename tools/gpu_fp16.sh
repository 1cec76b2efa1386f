#!/bin/bash
# fp16 (config 5) check: measured errors per module case + Dice, the fp16 parity tests, then the
# 192^3 full-model fp16 bench line.  Usage: tools/gpu_fp16.sh TAG
set -o pipefail
TAG=${1:-f16}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/prec_errs.py fp16 > gpurun_out/${TAG}_errs.txt 2>&1
rc=$?; cat gpurun_out/${TAG}_errs.txt | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "fp16 or attention_vs_oracle or stage1_fused" > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?; tail -15 gpurun_out/${TAG}_pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --workload full --img 192 --precision fp16 --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
