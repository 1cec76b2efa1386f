#!/bin/bash
# Stage-2 CCF_FFN fused back half (ffn_dwfc2_kernel): parity tests, then the B = 8 stage-2 FFN
# timed fused vs staged, then a kernel trace of the fused one.  usage: tools/gpu_dwfc2.sh TAG
set -o pipefail
TAG=${1:-dwfc2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "ccf_ffn" > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
for v in fused staged; do
  if [ $v = staged ]; then export WF_FFN_NO_DWFC=1; else unset WF_FFN_NO_DWFC; fi
  B=8 C=96 S=32 ITERS=20 timeout -k 10 200 python -u tools/kbench_ffn.py > $OUT/kb_$v.txt 2>&1 \
    || { tail -20 $OUT/kb_$v.txt; exit 1; }
  echo "$v: $(tail -1 $OUT/kb_$v.txt)"
done
unset WF_FFN_NO_DWFC
B=8 C=96 S=32 ITERS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
  -- python3 tools/kbench_ffn.py > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'{float(r["AverageNs"]) / 1e3:9.1f} us x {r["Calls"]:>4}  {r["Name"][:90]}')
EOF
