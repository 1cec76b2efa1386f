set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0 1 0 1 0; do
  WF_HF_SKIP=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --parity 0 --op-timers 0 --steps 300 > gpurun_out/s1_b$v.json 2>gpurun_out/s1_b$v.err || exit 1
  echo "HF_SKIP=$v $(python tools/bench_line.py gpurun_out/s1_b$v.json | cut -c1-80)"
done
