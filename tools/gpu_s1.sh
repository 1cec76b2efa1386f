set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_parity.py -k "upsample or projection or full_model or linear or gemm" > gpurun_out/s1_pytest.txt 2>&1 || { tail -30 gpurun_out/s1_pytest.txt; exit 1; }
tail -1 gpurun_out/s1_pytest.txt
for v in "WF_CAT_DIRECT=1" "WF_CAT_DIRECT=0" "WF_CAT_DIRECT=1" "WF_CAT_DIRECT=0"; do
  env $v timeout -k 10 300 python -u bench.py --workload full --img 192 --precision fp16 --cpu-baseline 0 --parity 0 --op-timers 0 > gpurun_out/s1_c5.json 2>gpurun_out/s1_c5.err || { tail -5 gpurun_out/s1_c5.err; exit 1; }
  echo "c5 $v $(python tools/bench_line.py gpurun_out/s1_c5.json | cut -c1-80)"
done
for v in "WF_CAT_DIRECT=1" "WF_CAT_DIRECT=0"; do
  env $v timeout -k 10 300 python -u bench.py --workload sliding --steps 10 --cpu-baseline 0 --parity 0 --op-timers 0 > gpurun_out/s1_c3.json 2>gpurun_out/s1_c3.err || { tail -5 gpurun_out/s1_c3.err; exit 1; }
  echo "c3 $v $(python tools/bench_line.py gpurun_out/s1_c3.json | cut -c1-80)"
done
