#!/bin/bash
# Round-5 GPU session: the -m gpu suite, the config-4 gradient diagnostics at 128^3, and a
# kernel trace of the config-4 train step.  Stops at the first step that ends in anything other
# than success or ordinary test failures (exit 0 / 1): a time limit, abort or fault.
#   tools/gpu_r5.sh TAG [suite|diag|train ...]
set -o pipefail
TAG=${1:-g5}; shift
STEPS=${@:-suite diag train}
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/${TAG}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
for s in $STEPS; do
  case $s in
    suite)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1
      rc=$?; tail -4 gpurun_out/${TAG}_pytest.txt; ok $rc || exit $rc ;;
    diag)
      timeout -k 10 500 python -u tools/grad128_diag.py --json gpurun_out/${TAG}_diag.json > gpurun_out/${TAG}_diag.txt 2>&1
      rc=$?; tail -40 gpurun_out/${TAG}_diag.txt; ok $rc || exit $rc ;;
    train)
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_tr -o run -- python -u bench.py --workload train --steps 6 --warmup 2 --cpu-baseline 0 --parity 0 > gpurun_out/${TAG}_tr.json 2> gpurun_out/${TAG}_tr.err
      rc=$?; tail -3 gpurun_out/${TAG}_tr.err; python tools/bench_line.py gpurun_out/${TAG}_tr.json
      f=$(ls gpurun_out/${TAG}_tr/*kernel_trace.csv 2>/dev/null | head -1)
      [ -n "$f" ] && python tools/kstats.py $f 40 > gpurun_out/${TAG}_tr_kstats.txt && head -42 gpurun_out/${TAG}_tr_kstats.txt
      ok $rc || exit $rc ;;
  esac
done
