set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "X=1" "WF_HF_SKIP=0" "WF_CONV_WIDE=0" "X=1" "WF_HF_SKIP=0" "WF_CONV_WIDE=0"; do
  env $v timeout -k 10 300 python -u bench.py --workload sliding --steps 10 --cpu-baseline 0 --parity 0 --op-timers 0 > gpurun_out/s1_c3.json 2>gpurun_out/s1_c3.err || { tail -5 gpurun_out/s1_c3.err; exit 1; }
  echo "$v $(python tools/bench_line.py gpurun_out/s1_c3.json | cut -c1-80)"
done
