#!/bin/bash
# Build variants/var_time.so: the current library with s_memtime phase probes in the
# wave-specialised ffn_dwfc kernel (WF_FFN_DBG=16 enables them; tools/dwfc_phase_times.py
# reads them).  The probes are never part of the product library.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/wf_timing
rm -rf $T && mkdir -p $T/waveformer_amd $T/include
cp -r $R/waveformer_amd/csrc $T/waveformer_amd/csrc
cp $R/include/waveformer_hip.h $T/include/
python3 - $T/waveformer_amd/csrc/ffn_dwfc.hip <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
def rep(a, b):
    global s
    assert s.count(a) == 1, a
    s = s.replace(a, b)
rep("template <int P, typename T>\n__global__ __launch_bounds__(768, 1) void ffn_dwfc_ws_kernel(DwFcArgs a) {",
    "__device__ long long g_wf_tbuf[64];\ntemplate <int P, typename T>\n__global__ __launch_bounds__(768, 1) void ffn_dwfc_ws_kernel(DwFcArgs a) {")
rep("    for (int p = z0 - 1; p <= z1 + 1; ++p) {\n      const bool live = p <= z1;",
    "    const bool tm = (a.dbg & 16) && blockIdx.x == 517 && (tid == 0 || tid == 320);\n    long long ta[4] = {0, 0, 0, 0};\n    for (int p = z0 - 1; p <= z1 + 1; ++p) {\n      long long c0 = __builtin_readcyclecounter();\n      const bool live = p <= z1;")
rep("      if (live && dscat) rows(cur, 0, a.ws_split);\n      __syncthreads();  // 1 -> 2",
    "      if (live && dscat) rows(cur, 0, a.ws_split);\n      long long c1 = __builtin_readcyclecounter();\n      __syncthreads();  // 1 -> 2\n      long long c2 = __builtin_readcyclecounter();")
rep("      __syncthreads();  // 2 -> next 1\n    }\n    return;",
    "      long long c3 = __builtin_readcyclecounter();\n      __syncthreads();  // 2 -> next 1\n      long long c4 = __builtin_readcyclecounter();\n      ta[0] += c1 - c0; ta[1] += c2 - c1; ta[2] += c3 - c2; ta[3] += c4 - c3;\n    }\n    if (tm)\n      for (int i = 0; i < 4; ++i) g_wf_tbuf[(tid ? 16 : 0) + i] = ta[i];\n    return;")
rep("  for (int p = z0 - 1; p <= z1 + 1; ++p) {\n    const int zo = p - 2;  // output plane this iteration finishes",
    "  const bool tmE = (a.dbg & 16) && blockIdx.x == 517 && (tid == NE || tid == NE + 320);\n  long long tb[4] = {0, 0, 0, 0};\n  for (int p = z0 - 1; p <= z1 + 1; ++p) {\n    long long c0 = __builtin_readcyclecounter();\n    const int zo = p - 2;  // output plane this iteration finishes")
rep("    __syncthreads();  // 1 -> 2: LN rows of tile (p-2) visible",
    "    long long c1 = __builtin_readcyclecounter();\n    __syncthreads();  // 1 -> 2: LN rows of tile (p-2) visible\n    long long c2 = __builtin_readcyclecounter();")
rep("    __syncthreads();  // 2 -> next 1\n  }\n}",
    "    long long c3 = __builtin_readcyclecounter();\n    __syncthreads();  // 2 -> next 1\n    long long c4 = __builtin_readcyclecounter();\n    tb[0] += c1 - c0; tb[1] += c2 - c1; tb[2] += c3 - c2; tb[3] += c4 - c3;\n  }\n  if (tmE)\n    for (int i = 0; i < 4; ++i) g_wf_tbuf[(tid == NE ? 8 : 24) + i] = tb[i];\n}")
s += '\nextern "C" int wf_debug_tbuf(long long* host) {\n  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(wf::g_wf_tbuf), 64 * sizeof(long long));\n}\n'
open(p, "w").write(s)
PY
make -C $T/waveformer_amd/csrc -j8 ARCH=gfx950 OUT=$R/variants/var_time.so BUILD=$T/obj > $T/build.log 2>&1 || { grep -i error $T/build.log; exit 1; }
echo built $R/variants/var_time.so
