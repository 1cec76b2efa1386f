#!/bin/bash
# Stitch counters under tools/kbench_stitch.py: kernel trace, FETCH / WRITE passes (raw, 4-B
# lane reads are uncalibrated), SQ stall breakdown.   tools/pmc_stitch.sh TAG
set -o pipefail
T=$1
export TMPDIR=/tmp ITERS=5
mkdir -p gpurun_out
timeout -k 10 120 python tools/kbench_stitch.py || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex stitch --output-format csv -d gpurun_out/${T}_f -o run -- python tools/kbench_stitch.py > gpurun_out/${T}_f.log 2>&1 || { tail -5 gpurun_out/${T}_f.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex stitch --output-format csv -d gpurun_out/${T}_w -o run -- python tools/kbench_stitch.py > gpurun_out/${T}_w.log 2>&1 || { tail -5 gpurun_out/${T}_w.log; exit 1; }
python - "$T" <<'PY'
import collections, csv, glob, sys
t = sys.argv[1]
for c, d in (("FETCH_SIZE", "f"), ("WRITE_SIZE", "w")):
    per = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/{t}_{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c:
                per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = sorted(per.values())
    print(f"{c}: median {v[len(v) // 2] / 1e3:.1f} MB per launch over {len(v)} launches (raw KB counter)")
PY
bash tools/pmc_sq_kernels.sh ${T}_sq stitch tools/kbench_stitch.py
