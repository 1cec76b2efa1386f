#!/bin/bash
# per-op determinism + short bench for library variants (abso/libwf_<v>.so)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  export WAVEFORMER_HIP_LIB=$PWD/abso/libwf_$v.so
  timeout -k 10 300 python -u tools/op_determinism.py > gpurun_out/opdet_$v.txt 2>&1 || { echo "opdet $v rc=$?"; tail -5 gpurun_out/opdet_$v.txt; exit 1; }
  grep SUMMARY gpurun_out/opdet_$v.txt
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --parity 0 --cpu-baseline 0 > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || { echo "bench $v rc=$?"; tail -5 gpurun_out/bench_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_$v.json')); print('$v', round(d['value'],1), 'vol/s', {k: v['avg_launch_us'] for k, v in d.get('rooflines', {}).items()}, d['roofline']['avg_launch_us'])"
done
