// wf_api.hip -- error plumbing and small utilities of the C-ABI (include/waveformer_hip.h).
#include "kernels.hpp"

#include <mutex>
#include <unordered_map>

namespace wf {
void set_max_lds(const void* fn, int bytes) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> done;
  std::lock_guard<std::mutex> lock(mu);
  int& cur = done[fn];
  if (bytes > cur) {
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    cur = bytes;
  }
}

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return (int)e;
  }
  return WF_OK;
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ in, uint16_t* __restrict__ out,
                                     int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = f2bf(in[i]);
}

__global__ void split_f32_bf16x2_kernel(const float* __restrict__ in, uint16_t* __restrict__ out,
                                        int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    const float v = in[i];
    const uint16_t hi = f2bf(v);
    out[i] = hi;
    out[n + i] = f2bf(v - bf2f(hi));
  }
}

// Many weights in one launch: table = [n + 1] int64 element offsets (prefix sums), then n
// source pointers, then n destination pointers, all in device memory.  Destination d of
// weight s holds its [2][numel] {hi, lo} planes, as wf_split_f32_to_bf16x2 writes them.
template <bool F16>
__device__ __forceinline__ void split_one(float v, uint16_t& h, uint16_t& l) {
  if (F16) {
    h = f2h(v);
    l = 0;
  } else {
    h = f2bf(v);
    l = f2bf(v - bf2f(h));
  }
}

// A workgroup owns 1024 consecutive elements of the concatenated weights: their first segment
// is found once (binary search, uniform), each thread walks forward from it for its 4
// elements, which move as one float4 load + two 8-B stores when they sit in one segment at a
// 4-aligned offset (every weight of the Python arena: numel % 8 == 0), element by element
// otherwise.  (A per-element binary search over the table ran the launch at ~3 TB/s.)
template <bool F16>
__global__ __launch_bounds__(256) void split_multi_kernel(const int64_t* __restrict__ table,
                                                          int n, int64_t total) {
  const int64_t* pre = table;
  const float* const* src = reinterpret_cast<const float* const*>(table + n + 1);
  uint16_t* const* dst = reinterpret_cast<uint16_t* const*>(table + 2 * n + 1);
  for (int64_t base = (int64_t)blockIdx.x * 1024; base < total; base += (int64_t)gridDim.x * 1024) {
    int lo = 0, hi = n - 1;  // last segment with pre[s] <= base
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pre[mid] <= base) lo = mid; else hi = mid - 1;
    }
    const int64_t i = base + 4 * (int64_t)threadIdx.x;
    if (i >= total) continue;
    int sg = lo;
    while (sg + 1 < n && pre[sg + 1] <= i) ++sg;
    const int64_t j = i - pre[sg], m = pre[sg + 1] - pre[sg];
    if (j + 4 <= m && (j & 3) == 0) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(src[sg] + j);
      uint16_t h[4], l[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) split_one<F16>(v[e], h[e], l[e]);
      *reinterpret_cast<uint2*>(dst[sg] + j) =
          uint2{(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)};
      *reinterpret_cast<uint2*>(dst[sg] + m + j) =
          uint2{(uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16)};
    } else {
      for (int e = 0; e < 4 && i + e < total; ++e) {
        const int64_t ie = i + e;
        while (sg + 1 < n && pre[sg + 1] <= ie) ++sg;
        const int64_t je = ie - pre[sg], me = pre[sg + 1] - pre[sg];
        uint16_t hh, ll;
        split_one<F16>(src[sg][je], hh, ll);
        dst[sg][je] = hh;
        dst[sg][me + je] = ll;
      }
    }
  }
}

__global__ void cast_f16x2_kernel(const float* __restrict__ in, uint16_t* __restrict__ out,
                                  int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    out[i] = f2h(in[i]);
    out[n + i] = 0;
  }
}

// Test support: fill `words` of LDS with a quiet-NaN pattern (volatile: the stores are kept)
__global__ __launch_bounds__(256) void poison_lds_kernel(int words) {
  extern __shared__ uint32_t pl[];
  volatile uint32_t* v = pl;
  for (int i = threadIdx.x; i < words; i += blockDim.x) v[i] = 0x7fc00000u | (uint32_t)(i & 0xffff);
}

}  // namespace wf

extern "C" int wf_abi_version(void) { return WF_ABI_VERSION; }

extern "C" int wf_debug_poison_lds(int64_t blocks, int lds_bytes, void* stream) {
  WF_REQUIRE(blocks >= 1 && blocks <= (1 << 20), "blocks out of range");
  WF_REQUIRE(lds_bytes >= 4 && lds_bytes <= 160 * 1024, "lds_bytes out of range");
  wf::set_max_lds(reinterpret_cast<const void*>(wf::poison_lds_kernel), lds_bytes);
  hipLaunchKernelGGL(wf::poison_lds_kernel, dim3((unsigned)blocks), dim3(256), (size_t)lds_bytes,
                     (hipStream_t)stream, lds_bytes / 4);
  return wf::check_launch("wf_debug_poison_lds");
}

static int split_multi(const int64_t* table_dev, int64_t n, int64_t total, void* stream,
                       bool f16) {
  WF_REQUIRE(n >= 0 && total >= 0, "negative count");
  if (n == 0 || total == 0) return WF_OK;
  WF_REQUIRE_PTR(table_dev);
  int64_t blocks = wf::cdiv(total, 1024);
  if (blocks > 65535) blocks = 65535;
  if (f16)
    hipLaunchKernelGGL(wf::split_multi_kernel<true>, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, table_dev, (int)n, total);
  else
    hipLaunchKernelGGL(wf::split_multi_kernel<false>, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, table_dev, (int)n, total);
  return wf::check_launch("wf_split_f32_to_bf16x2_multi");
}

extern "C" int wf_split_f32_to_bf16x2_multi(const int64_t* table_dev, int64_t n, int64_t total,
                                            void* stream) {
  return split_multi(table_dev, n, total, stream, false);
}

extern "C" int wf_cast_f32_to_f16x2_multi(const int64_t* table_dev, int64_t n, int64_t total,
                                          void* stream) {
  return split_multi(table_dev, n, total, stream, true);
}

extern "C" int wf_cast_f32_to_f16x2(const float* in, uint16_t* out, int64_t n, void* stream) {
  WF_REQUIRE(n >= 0, "n < 0");
  if (n == 0) return WF_OK;
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(out);
  int64_t blocks = wf::cdiv(n, 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(wf::cast_f16x2_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, in, out, n);
  return wf::check_launch("wf_cast_f32_to_f16x2");
}

extern "C" const char* wf_last_error(void) { return wf::g_last_error.c_str(); }

extern "C" int wf_cast_f32_to_bf16(const float* in, uint16_t* out, int64_t n, void* stream) {
  WF_REQUIRE(n >= 0, "n < 0");
  if (n == 0) return WF_OK;
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(out);
  int64_t blocks = wf::cdiv(n, 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(wf::cast_f32_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, in, out, n);
  return wf::check_launch("wf_cast_f32_to_bf16");
}

extern "C" int wf_split_f32_to_bf16x2(const float* in, uint16_t* out, int64_t n, void* stream) {
  WF_REQUIRE(n >= 0, "n < 0");
  if (n == 0) return WF_OK;
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(out);
  int64_t blocks = wf::cdiv(n, 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(wf::split_f32_bf16x2_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, in, out, n);
  return wf::check_launch("wf_split_f32_to_bf16x2");
}

using wf::GemmArgs;
using namespace wf;

// out[m, n] = bias[n] + sum_k act(x[m, k]) * W[n, k] over fp32 rows (act = GELU(erf) or
// identity): the decoder's 1x1x1 convolutions of ProjectionUpsample on the MFMA GEMM family
// (gemm_rows / gemm_kc / gemm_ares, bf16x3 or bf16 operands, fp32 accumulation).
extern "C" int wf_convtranspose2_cl(const float* x, const uint16_t* w_bf16x2, const float* bias,
                                    float* out, int64_t ldo, int64_t B, int64_t Cin, int64_t Cout,
                                    int64_t d, int64_t h, int64_t w, int precision, void* stream) {
  WF_REQUIRE(B >= 1 && d >= 1 && h >= 1 && w >= 1, "empty tensor");
  WF_REQUIRE(Cin >= 8 && Cin % 8 == 0 && Cout >= 4 && Cout % 4 == 0,
             "need Cin a multiple of 8 and Cout a multiple of 4");
  WF_REQUIRE(ldo >= Cout && ldo % 4 == 0, "ldo must be >= Cout and a multiple of 4");
  WF_REQUIRE(valid_prec(precision), "unknown precision");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(w_bf16x2);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0,
             "x / out must be 16-byte aligned");
  WF_REQUIRE(B * d * h * w < ((int64_t)1 << 31) && 8 * Cout <= 4096, "shape too large");
  GemmArgs g{};
  g.prec = precision;
  g.a_src = x;
  g.a_C = (int)Cin;
  g.a_nseg = 1;
  g.a_map = MAP_IDENTITY;
  g.a_ln = LN_NONE;
  g.mB = (int)B;
  g.mD = (int)d;
  g.mH = (int)h;
  g.mW = (int)w;
  g.w = w_bf16x2;
  g.M = B * d * h * w;
  g.N = (int)(8 * Cout);
  g.K = (int)Cin;
  g.epi = EPI_SUBVOXEL;
  g.bias = bias;
  g.out = out;
  g.ldo = ldo;
  if (!try_launch_gemm_rows(g, (hipStream_t)stream, false))
    return fail(WF_E_SHAPE, "wf_convtranspose2_cl: shape not covered by the streaming GEMM");
  return check_launch("wf_convtranspose2_cl");
}

extern "C" int wf_linear_fwd(const float* x, const uint16_t* w_bf16x2, const float* bias,
                             float* out, int64_t M, int64_t K, int64_t N, int gelu_in,
                             int precision, void* stream) {
  WF_REQUIRE(M >= 0 && K >= 8 && K % 8 == 0 && N >= 4 && N % 4 == 0,
             "need K a multiple of 8 and N a multiple of 4");
  WF_REQUIRE(valid_prec(precision), "unknown precision");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(w_bf16x2);
  WF_REQUIRE_PTR(out);
  GemmArgs g{};
  g.prec = precision;
  g.a_src = x;
  g.a_bf16 = 0;
  g.a_C = (int)K;
  g.a_nseg = 1;
  g.a_map = MAP_IDENTITY;
  g.a_ln = LN_NONE;
  g.a_gelu = gelu_in ? 1 : 0;
  g.w = w_bf16x2;
  g.M = M;
  g.N = (int)N;
  g.K = (int)K;
  g.epi = EPI_STORE;
  g.bias = bias;
  g.out = out;
  g.out_bf16 = 0;
  g.ldo = N;
  return launch_gemm(g, (hipStream_t)stream, "wf_linear_fwd");
}
