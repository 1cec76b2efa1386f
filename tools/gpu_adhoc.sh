set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ddp.py tests/test_gpu_grad128.py tests/test_train_grads.py -s > gpurun_out/g5f_pytest.txt 2>&1; rc=$?; grep -E "grad128:|DDP vs|PASS|FAIL|passed|failed" gpurun_out/g5f_pytest.txt | tail -20; exit $rc
