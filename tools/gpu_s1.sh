set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
WF_PU_CHUNK=65536 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py -k "projection" > gpurun_out/s1_pytest.txt 2>&1 || { tail -30 gpurun_out/s1_pytest.txt; exit 1; }
tail -1 gpurun_out/s1_pytest.txt
for v in "WF_PU_CHUNK=0" "WF_PU_CHUNK=131072" "WF_PU_CHUNK=65536" "WF_PU_CHUNK=262144" "WF_PU_CHUNK=0" "WF_PU_CHUNK=131072" "WF_PU_CHUNK=65536"; do
  env $v timeout -k 10 300 python -u bench.py --workload full --img 192 --precision fp16 --cpu-baseline 0 --parity 0 --op-timers 0 > gpurun_out/s1_c5.json 2>gpurun_out/s1_c5.err || { tail -5 gpurun_out/s1_c5.err; exit 1; }
  echo "c5 $v $(python tools/bench_line.py gpurun_out/s1_c5.json | cut -c1-80)"
done
