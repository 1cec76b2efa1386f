set -o pipefail
mkdir -p gpurun_out
T=${1:-g5g}
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_ddp.py tests/test_gpu_grad128.py -m gpu -s > gpurun_out/${T}_pytest.txt 2>&1; rc=$?; grep -E "grad128:|DDP vs|passed|failed|Error" gpurun_out/${T}_pytest.txt | tail -8; [ $rc -le 1 ] || exit $rc
tools/gpu_r5.sh $T train
