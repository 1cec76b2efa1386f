set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --precision bf16 --cpu-baseline 0 > gpurun_out/s2_bench_bf16.json 2> gpurun_out/s2_bench_bf16.err || { tail -20 gpurun_out/s2_bench_bf16.err; exit 1; }
python tools/bench_line.py gpurun_out/s2_bench_bf16.json 2>/dev/null || tail -c 1500 gpurun_out/s2_bench_bf16.json
bash tools/gpu_prof.sh s2bf16 --precision bf16
