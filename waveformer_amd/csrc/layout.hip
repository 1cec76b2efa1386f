// layout.hip -- data movement of the decoder's channel-last buffers (config 3 / 5 inference).
//
// The decoder keeps its activations channel-last (channels_last_3d: the channels of one
// position contiguous, positions `ld` floats apart).  Two moves the PyTorch layer left to
// generic copy kernels (strided, 4-byte elements; profiled in one 192^3 config-5 forward,
// tools/copy_trace.py):
//   * torch.cat((out, skip), 1) / torch.cat([up4, up3, dec2], 1): channel slices of one
//     channel-last tensor into another -- wf_copy_cl, one float4 per lane (1.16 ms for the
//     2 x 48 x 192^3 skip copy of decoder1);
//   * ConvTranspose3d(k = s = 2) as a GEMM (positions x Cin) . (Cin x 8 Cout) whose columns
//     are the 8 sub-voxels (monai unetr_block.py:73-80 via blocks.UnetrUpBlock): the GEMM rows
//     scattered into the 2 x 2 x 2 children of each position, + bias -- wf_subvoxel_scatter_cl
//     (1.35 ms as a permuted copy_, plus a separate bias add).
// Both are HBM-bound: 8 bytes of traffic per float moved.
#include "kernels.hpp"

namespace wf {

// n / d for 0 <= n < 2^31 by a multiply-high and a shift (Granlund-Montgomery round-up
// method, multiplier and shift made on the host): a 64-bit division per element made these
// copies VALU-bound (the sub-voxel scatter ran at 1.1 TB/s)
struct FastDiv {
  uint32_t d, m, s;
  explicit FastDiv(uint32_t dv = 1) : d(dv), m(1), s(0) {
    while ((1ull << s) < dv) ++s;
    m = (uint32_t)((((1ull << 32) * ((1ull << s) - dv)) / dv) + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    return (__umulhi(n, m) + n) >> s;
  }
};

__global__ __launch_bounds__(256) void copy_cl_kernel(const float* __restrict__ src, int64_t lds,
                                                      float* __restrict__ dst, int64_t ldd,
                                                      FastDiv c4d, uint32_t total) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const uint32_t p = c4d.div(i);
    const uint32_t c = (i - p * c4d.d) * 4;
    *reinterpret_cast<f32x4*>(dst + (int64_t)p * ldd + c) =
        *reinterpret_cast<const f32x4*>(src + (int64_t)p * lds + c);
  }
}

// g: (B*d*h*w, 8*C) rows, column s*C + c with s = dz*4 + dy*2 + dx (g.view(B,d,h,w,2,2,2,C));
// dst: channel-last (B, C, 2d, 2h, 2w) positions ldd floats apart
__global__ __launch_bounds__(256) void subvoxel_scatter_cl_kernel(
    const float* __restrict__ g, const float* __restrict__ bias, float* __restrict__ dst,
    int64_t ldd, FastDiv c4d, FastDiv wd, FastDiv hd, FastDiv dd, uint32_t total) {
  const uint32_t C = 4 * c4d.d, w = wd.d, h = hd.d, d = dd.d;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    // i = ((row * 8 + s) * C4 + c4): consecutive lanes read consecutive 16 B of a g row
    const uint32_t rs = c4d.div(i);
    const uint32_t c = (i - rs * c4d.d) * 4;
    const uint32_t sv = rs & 7, r0 = rs >> 3;
    const uint32_t r1 = wd.div(r0), x = r0 - r1 * w;
    const uint32_t r2 = hd.div(r1), y = r1 - r2 * h;
    const uint32_t b = dd.div(r2), z = r2 - b * d;
    const uint32_t dz = sv >> 2, dy = (sv >> 1) & 1, dx = sv & 1;
    f32x4 v = *reinterpret_cast<const f32x4*>(g + (int64_t)rs * C + c);
    if (bias) v += *reinterpret_cast<const f32x4*>(bias + c);
    const int64_t pos = (((int64_t)b * (2 * d) + 2 * z + dz) * (2 * h) + 2 * y + dy) * (2 * w) +
                        2 * x + dx;
    *reinterpret_cast<f32x4*>(dst + pos * ldd + c) = v;
  }
}

// UnetOutBlock (monai dynunet_block.py:188-210): 1x1x1 conv, K input channels (channel-last,
// positions ldx floats apart) -> N <= 16 classes written NCDHW, the layout the network returns.
// A workgroup stages 256 positions x K channels (coalesced 16-B loads, row stride K + 4 floats)
// and the (N, K) weights in LDS; lane t then computes position t's N outputs from 16-B LDS
// reads only (weights as broadcast reads: scalar weight loads would share lgkmcnt with the LDS
// reads and serialise them), fp32 FMAs; the N stores are coalesced along positions.
// grid (cdiv(P, 256), B)
constexpr int HEAD_TP = 256;
template <int N>
__global__ __launch_bounds__(256) void conv1x1_head_kernel(
    const float* __restrict__ x, int64_t ldx, const float* __restrict__ wt,
    const float* __restrict__ bias, float* __restrict__ out, int K, int64_t P) {
  extern __shared__ __attribute__((aligned(16))) float tile[];  // [HEAD_TP][K + 4], [N][K]
  const int b = blockIdx.y;
  const int64_t p0 = (int64_t)blockIdx.x * HEAD_TP;
  const int np = (int)min((int64_t)HEAD_TP, P - p0);
  const int K4 = K >> 2, KS = K + 4;
  float* wl = tile + HEAD_TP * KS;
  const float* src = x + ((int64_t)b * P + p0) * ldx;
  // four 16-B loads in flight per lane before their LDS stores (clamped addresses, guarded
  // stores): a load-store pair per iteration left one load in flight and ran latency-bound
  const int tot = np * K4;
  for (int e0 = threadIdx.x; e0 < tot; e0 += 4 * HEAD_TP) {
    f32x4 v[4];
    int off[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = min(e0 + u * HEAD_TP, tot - 1);
      const int r = e / K4, c = 4 * (e - r * K4);
      off[u] = r * KS + c;
      v[u] = *reinterpret_cast<const f32x4*>(src + (int64_t)r * ldx + c);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (e0 + u * HEAD_TP < tot) *reinterpret_cast<f32x4*>(tile + off[u]) = v[u];
  }
  for (int e = threadIdx.x; e < N * K4; e += blockDim.x)
    *reinterpret_cast<f32x4*>(wl + 4 * e) = *reinterpret_cast<const f32x4*>(wt + 4 * e);
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= np) return;
  float acc[N];
#pragma unroll
  for (int n = 0; n < N; ++n) acc[n] = bias ? bias[n] : 0.f;
  const float* xr = tile + t * KS;
  for (int k = 0; k < K; k += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(xr + k);
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(wl + n * K + k);
      acc[n] = fmaf(w.x, v.x, acc[n]);
      acc[n] = fmaf(w.y, v.y, acc[n]);
      acc[n] = fmaf(w.z, v.z, acc[n]);
      acc[n] = fmaf(w.w, v.w, acc[n]);
    }
  }
  float* o = out + (int64_t)b * N * P + p0 + t;
#pragma unroll
  for (int n = 0; n < N; ++n) o[(int64_t)n * P] = acc[n];
}

static unsigned grid_for(int64_t total) {
  int64_t blocks = cdiv(total, 256);
  if (blocks > 65536) blocks = 65536;  // grid-stride beyond: ~256 workgroups per CU
  return (unsigned)(blocks < 1 ? 1 : blocks);
}

// y (M, N) = x (M, K) . w (N, K)^T + bias for K < 8 -- the shapes the MFMA GEMM's K-octet loader
// does not take: the 4-channel stem / head convolutions of the full model in training (UnetResBlock
// conv3 4 -> 48 forward, UnetOutBlock 48 -> 4 input gradient).  One thread per (row, 4 outputs),
// exact fp32 FMAs in k order from the bias; the N / 4 threads of a row write its y row as one
// contiguous run, the x row (<= 32 B) is shared through the cache.
template <int K>
__global__ __launch_bounds__(256) void linear_smallk_kernel(
    const float* __restrict__ x, int64_t ldx, const float* __restrict__ w,
    const float* __restrict__ bias, float* __restrict__ y, int64_t ldy, uint32_t M, int N) {
  extern __shared__ __attribute__((aligned(16))) float wl[];  // [N][K], then bias [N]
  for (int i = threadIdx.x; i < N * K; i += 256) wl[i] = w[i];
  for (int i = threadIdx.x; i < N; i += 256) wl[N * K + i] = bias ? bias[i] : 0.f;
  __syncthreads();
  const uint32_t N4 = (uint32_t)N >> 2;
  const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
  const uint32_t row = idx / N4, j = idx - row * N4;
  if (row >= M) return;
  const float* xr = x + (int64_t)row * ldx;
  float xv[K];
#pragma unroll
  for (int k = 0; k < K; ++k) xv[k] = xr[k];
  float acc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const float* wr = wl + (4 * j + n) * K;
    float a = wl[N * K + 4 * j + n];
#pragma unroll
    for (int k = 0; k < K; ++k) a = fmaf(xv[k], wr[k], a);
    acc[n] = a;
  }
  *reinterpret_cast<f32x4*>(y + (int64_t)row * ldy + 4 * j) = f32x4{acc[0], acc[1], acc[2], acc[3]};
}

}  // namespace wf

using namespace wf;

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

extern "C" int wf_copy_cl(const float* src, int64_t lds, float* dst, int64_t ldd, int64_t P,
                          int64_t C, void* stream) {
  WF_REQUIRE(P >= 0 && C >= 4 && C % 4 == 0, "C must be a positive multiple of 4");
  WF_REQUIRE(lds >= C && ldd >= C && lds % 4 == 0 && ldd % 4 == 0,
             "position strides must be >= C and multiples of 4");
  WF_REQUIRE_PTR(src);
  WF_REQUIRE_PTR(dst);
  WF_REQUIRE(aligned16(src) && aligned16(dst), "src / dst must be 16-byte aligned");
  if (P == 0) return WF_OK;
  const int64_t total = P * (C / 4);
  WF_REQUIRE(total < ((int64_t)1 << 31), "wf_copy_cl: more than 2^31 float4 items");
  hipLaunchKernelGGL(copy_cl_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                     src, lds, dst, ldd, FastDiv((uint32_t)(C / 4)), (uint32_t)total);
  return check_launch("wf_copy_cl");
}

extern "C" int wf_subvoxel_scatter_cl(const float* g, const float* bias, float* dst, int64_t ldd,
                                      int64_t B, int64_t C, int64_t d, int64_t h, int64_t w,
                                      void* stream) {
  WF_REQUIRE(B >= 1 && d >= 1 && h >= 1 && w >= 1, "empty tensor");
  WF_REQUIRE(C >= 4 && C % 4 == 0 && ldd >= C && ldd % 4 == 0,
             "C must be a positive multiple of 4, ldd >= C a multiple of 4");
  WF_REQUIRE_PTR(g);
  WF_REQUIRE_PTR(dst);
  WF_REQUIRE(aligned16(g) && aligned16(dst) && (!bias || aligned16(bias)),
             "g / dst / bias must be 16-byte aligned");
  const int64_t total = B * d * h * w * 8 * (C / 4);
  WF_REQUIRE(total < ((int64_t)1 << 31), "wf_subvoxel_scatter_cl: more than 2^31 float4 items");
  hipLaunchKernelGGL(subvoxel_scatter_cl_kernel, dim3(grid_for(total)), dim3(256), 0,
                     (hipStream_t)stream, g, bias, dst, ldd, FastDiv((uint32_t)(C / 4)),
                     FastDiv((uint32_t)w), FastDiv((uint32_t)h), FastDiv((uint32_t)d),
                     (uint32_t)total);
  return check_launch("wf_subvoxel_scatter_cl");
}

extern "C" int wf_linear_smallk_fwd(const float* x, int64_t ldx, const float* w,
                                    const float* bias, float* y, int64_t ldy, int64_t M,
                                    int64_t K, int64_t N, void* stream) {
  WF_REQUIRE(M >= 0 && K >= 1 && K <= 7 && N >= 4 && N % 4 == 0 && N <= 4096,
             "small-K linear: K in [1, 7], N a multiple of 4 up to 4096");
  WF_REQUIRE(ldx >= K && ldy >= N && ldy % 4 == 0, "ldx >= K, ldy >= N a multiple of 4");
  WF_REQUIRE(M * (N / 4) < ((int64_t)1 << 31), "small-K linear: too many outputs");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(w);
  WF_REQUIRE_PTR(y);
  WF_REQUIRE(aligned16(y), "y must be 16-byte aligned");
  if (M == 0) return WF_OK;
  const size_t lds = (size_t)N * (K + 1) * sizeof(float);
  const dim3 grid((unsigned)cdiv(M * (N / 4), 256));
  hipStream_t s = (hipStream_t)stream;
  switch (K) {
#define WF_SK(k) case k: hipLaunchKernelGGL(linear_smallk_kernel<k>, grid, dim3(256), lds, s, x, ldx, w, bias, y, ldy, (uint32_t)M, (int)N); break;
    WF_SK(1) WF_SK(2) WF_SK(3) WF_SK(4) WF_SK(5) WF_SK(6) WF_SK(7)
#undef WF_SK
  }
  return check_launch("wf_linear_smallk_fwd");
}

extern "C" int wf_conv1x1_head_cl(const float* x, int64_t ldx, const float* weight,
                                  const float* bias, float* out, int64_t B, int64_t K, int64_t N,
                                  int64_t P, void* stream) {
  WF_REQUIRE(B >= 1 && P >= 1, "empty tensor");
  WF_REQUIRE(K >= 4 && K % 4 == 0 && K <= 120 && ldx >= K && ldx % 4 == 0,
             "K must be a multiple of 4 in [4, 120], ldx >= K a multiple of 4");
  WF_REQUIRE(N >= 1 && N <= 16, "N must be in [1, 16]");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(weight);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE(aligned16(x) && aligned16(weight), "x / weight must be 16-byte aligned");
  const size_t lds = ((size_t)HEAD_TP * (K + 4) + N * K) * sizeof(float);
  const dim3 grid((unsigned)cdiv(P, HEAD_TP), (unsigned)B);
  hipStream_t s = (hipStream_t)stream;
  switch (N) {
#define WF_HEAD(n) case n: if (lds > 64 * 1024) set_max_lds(reinterpret_cast<const void*>(conv1x1_head_kernel<n>), (int)lds); hipLaunchKernelGGL(conv1x1_head_kernel<n>, grid, dim3(256), lds, s, x, ldx, weight, bias, out, (int)K, P); break;
    WF_HEAD(1) WF_HEAD(2) WF_HEAD(3) WF_HEAD(4) WF_HEAD(5) WF_HEAD(6) WF_HEAD(7) WF_HEAD(8)
    WF_HEAD(9) WF_HEAD(10) WF_HEAD(11) WF_HEAD(12) WF_HEAD(13) WF_HEAD(14) WF_HEAD(15) WF_HEAD(16)
#undef WF_HEAD
  }
  return check_launch("wf_conv1x1_head_cl");
}
