"""Per-launch-site times of the gemm_kc family in encoder-driver kernel traces: launches of one
forward are numbered in order (a split-K reduce is added to the GEMM launch before it), averaged
over the forwards and rounds of each variant.  usage: kc_positions.py TAG NVARIANTS"""
import csv, glob, re, sys, collections
tag, nv = sys.argv[1], int(sys.argv[2])
RX = re.compile(r"gemm_kc")
for v in range(1, nv + 1):
    sites = collections.defaultdict(list)
    names = {}
    for f in sorted(glob.glob(f"gpurun_out/{tag}_v{v}_*/run_kernel_trace.csv")):
        rows = [r for r in csv.DictReader(open(f))]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        # forwards start at each patch_embed launch
        fwd, seq = -1, []
        for r in rows:
            n = r["Kernel_Name"]
            if "patch_embed" in n:
                fwd += 1
                seq = []
            if fwd < 0 or not RX.search(n):
                continue
            t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            if "reduce" in n and seq:
                sites[(f, fwd, len(seq) - 1)].append(t)
                continue
            seq.append(n)
            i = len(seq) - 1
            names[i] = (re.sub(r"\(wf::GemmArgs\)|void wf::|, false, 0, 8>", "", n)[:24],
                        r["Grid_Size_X"] + "x" + r["Grid_Size_Y"] + "x" + r["Grid_Size_Z"],
                        r["Workgroup_Size_X"])
            sites[(f, fwd, i)].append(t)
    per = collections.defaultdict(list)
    for (_, fw, i), ts in sites.items():
        if fw >= 3:  # skip the warm-up forwards
            per[i].append(sum(ts))
    print(f"--- variant {v}")
    tot = 0
    for i in sorted(per):
        m = sum(per[i]) / len(per[i])
        tot += m
        print(f"  {i:2d} {names[i][0]:24s} {names[i][1]:>14s} {m:7.1f} us")
    print(f"  total {tot:.1f} us per forward")
