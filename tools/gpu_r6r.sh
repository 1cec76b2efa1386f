#!/bin/bash
# Round 6: wgrad with the XOR-swizzled g tile (A/B vs the committed build, x3) + SQ pass;
# decoder / training tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  echo "== wgrad XCD grid"; timeout -k 10 120 python tools/kbench_wgrad.py 4 || exit 1
  echo "== wgrad committed"; WAVEFORMER_HIP_LIB=$PWD/abv/libwf_wgrad_old.so timeout -k 10 120 python tools/kbench_wgrad.py 4 || exit 1
done
bash tools/pmc_sq_kernels.sh r6af_wg 'conv3d_wgrad' tools/kbench_wgrad.py || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_grad128.py tests/test_gpu_ddp.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6af_pytest.txt 2>&1 || { tail -30 gpurun_out/r6af_pytest.txt; exit 1; }
tail -2 gpurun_out/r6af_pytest.txt
