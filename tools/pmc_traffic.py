"""HBM traffic per launch from two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of
the same command, written to a JSON summary that bench.py reads (roofline.traffic).

    python tools/pmc_traffic.py gpurun_out/TAG_pmc_fetch gpurun_out/TAG_pmc_write OUT.json

Per MI355X_MICROARCH.md (HBM [CDNA4]): FETCH_SIZE and WRITE_SIZE are kilobytes at the L2's
memory side (Infinity-Cache hits included); on gfx950 FETCH_SIZE reports half the bytes of a
16 B/lane streaming read, and WRITE_SIZE is exact for 16 B/lane stores.  Other access widths
are uncalibrated (the guide says so), so the x2 read correction is applied ONLY to the kernels
listed in WIDE16 -- their bulk reads are 16 B per lane (f32x4 / b128 loads, checked in the
source) -- and every other kernel's FETCH_SIZE is reported raw with rule "raw-uncalibrated"
(the old scalar IDWT read its bands 4 B per lane and the blanket x2
inflated its traffic to 1.44x).  Each kernel's entry records the rule it got.
For each kernel the largest launch (max fetch) is reported, and under "by_grid" the largest
launch of each launch shape (grid size in work-items): bench.py keys its traffic by the shape
of the launch it times when it knows it."""
import collections
import csv
import glob
import json
import sys


def load(root, counter):
    """{kernel name: [(grid size in work-items, counter value summed over the dispatch's
    XCD / instance rows), ...]}, one entry per dispatch."""
    out = collections.defaultdict(list)
    grid = {}
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0]
            key = (name, r.get("Dispatch_Id", ""))
            out[key].append(float(r["Counter_Value"]))
            grid[key] = int(float(r.get("Grid_Size", 0) or 0))
    per = collections.defaultdict(list)
    for key, v in out.items():
        per[key[0]].append((grid[key], sum(v)))
    return per


# kernels whose bulk reads are 16 B per lane (name prefixes; see the module docstring)
WIDE16 = ("dwt3d_haar_fwd_kernel", "idwt3d_haar_cl4_kernel", "idwt3d_haar_nc4_kernel",
          "msfuse_row_kernel", "ffn_dwfc_sb_kernel", "ffn_dwfc_ws_kernel", "ffn_dwfc2_kernel",
          "gemm_rows_kernel", "gemm_kc_kernel", "gemm_lnw_kernel", "dwconv_ln_gelu_kernel",
          "proj_out_kernel", "ffn_dwfc_tb4_kernel", "ffn_dwfc_tb_kernel", "attn_tbl_kernel",
          "merge_res_kernel", "pw2_res_kernel")


def rule_of(name):
    short = name.split("<")[0].split("::")[-1].strip()
    return "x2-fetch-16B" if short.startswith(WIDE16) else "raw-uncalibrated"


def main():
    fetch_root, write_root, dst = sys.argv[1], sys.argv[2], sys.argv[3]
    batch = int(sys.argv[4]) if len(sys.argv) > 4 else 4  # bench --batch of the PMC passes
    fetch, write = load(fetch_root, "FETCH_SIZE"), load(write_root, "WRITE_SIZE")
    kernels = {}
    for name, fv in fetch.items():
        if "rocclr" in name or "at::native" in name:
            continue
        wv = write.get(name, [(0, 0.0)])
        rule = rule_of(name)
        k = 2 if rule == "x2-fetch-16B" else 1
        f_kb, w_kb = max(v for _, v in fv), max(v for _, v in wv)
        # per launch shape (grid size in work-items): the largest launch of each, so a bench
        # roofline can take the entry of ITS launch rather than the kernel name's largest
        shapes = {}
        for g in sorted({g for g, _ in fv}):
            fg = max(v for gg, v in fv if gg == g)
            wg = max((v for gg, v in wv if gg == g), default=0.0)
            shapes[str(g)] = {"launches": sum(1 for gg, _ in fv if gg == g),
                              "hbm_bytes_per_launch": int(k * fg * 1024 + wg * 1024)}
        kernels[name] = {
            "launches": len(fv),
            "fetch_size_kb_largest": f_kb,
            "write_size_kb_largest": w_kb,
            "rule": rule,
            "hbm_bytes_per_launch_largest": int(k * f_kb * 1024 + w_kb * 1024),
            "by_grid": shapes,
        }
    json.dump({"source": [fetch_root, write_root], "per_gpu_batch": batch,
               "correction": "bytes = k * FETCH_SIZE[KB] * 1024 + WRITE_SIZE[KB] * 1024, k = 2 for "
                             "rule x2-fetch-16B (gfx950 FETCH_SIZE halving of 16 B/lane reads, "
                             "MI355X_MICROARCH.md), k = 1 for raw-uncalibrated",
               "kernels": kernels}, open(dst, "w"), indent=1)
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch_largest"])[:12]:
        print(f"{v['hbm_bytes_per_launch_largest'] / 1e6:10.1f} MB  {k}")


if __name__ == "__main__":
    main()
