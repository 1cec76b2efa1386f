set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp ITERS=4
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py > gpurun_out/s1_pytest.txt 2>&1 || { tail -30 gpurun_out/s1_pytest.txt; exit 1; }
tail -1 gpurun_out/s1_pytest.txt
for v in "WF_CONV_WIDE=1" "WF_CONV_WIDE=0" "WF_CONV_WIDE=1" "WF_CONV_WIDE=0"; do
  echo "== $v"; env $v timeout -k 10 120 python tools/kbench_conv_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
done
