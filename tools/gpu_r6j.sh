#!/bin/bash
# Round 6: stitch batched-load paths (tests + config-3 stitch roofline); SQ pass over the
# stage-1 streaming kernels and the stage-2 FFN back half.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6j}
timeout -k 10 400 python -u -m pytest tests/test_gpu_sliding_window.py tests/test_gpu_config3.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest.txt
timeout -k 10 300 python bench.py --workload sliding --steps 5 --warmup 2 > gpurun_out/${T}_sliding.json 2> gpurun_out/${T}_sliding.log || { tail -20 gpurun_out/${T}_sliding.log; exit 1; }
cut -c1-200 gpurun_out/${T}_sliding.json; grep -o '"sliding_window_stitch": {[^}]*}' gpurun_out/${T}_sliding.json
bash tools/pmc_sq_kernels.sh ${T}_sq 'msfuse|merge_res|patch_embed|dwt3d_haar|ffn_dwfc2|proj_out|pw2' 2>&1 | tee gpurun_out/${T}_sq.txt
