set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_config.py > gpurun_out/s1_pytest.txt 2>&1 || { tail -30 gpurun_out/s1_pytest.txt; exit 1; }
tail -1 gpurun_out/s1_pytest.txt
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --parity 1 --steps 200 > gpurun_out/s1_bp.json 2>gpurun_out/s1_bp.err || exit 1
python tools/bench_line.py gpurun_out/s1_bp.json | cut -c1-80
python -c "import json; print(json.load(open('gpurun_out/s1_bp.json'))['parity'])"
