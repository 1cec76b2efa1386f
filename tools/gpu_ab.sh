#!/bin/bash
# Parity suite + FFN microbench + bench A/B of env-gated variants + kernel trace.
# Usage: tools/gpu_ab.sh TAG [VAR1 VAR2 ...]   (each VAR is set to 1 for one extra bench run)
set -o pipefail
TAG=${1:-ab}
shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x --durations=15 > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?
tail -22 gpurun_out/${TAG}_pytest.txt
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 200 python tools/kbench_ffn.py > gpurun_out/${TAG}_ffn.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_ffn.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --batch 4 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_bench_b4.json 2> gpurun_out/${TAG}_bench_b4.err || exit 1
for V in "$@"; do
  env $V=1 timeout -k 10 400 python bench.py --steps 20 --warmup 5 --batch 4 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_bench_b4_${V}.json 2>&1 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --batch 4 --cpu-baseline 0 --parity 0 --graph 0 > gpurun_out/${TAG}_prof.log 2>&1
echo done
