// instnorm.hip -- InstanceNorm3d (affine=False, biased variance) + LeakyReLU + residual on
// channel-last activations: the norm / act / add glue of MONAI's UnetResBlock and
// UnetBasicBlock (monai/networks/blocks/dynunet_block.py:98-111, :170-185) around the
// decoder's 3x3x3 convolutions (conv3d.hip).
//
//   stats:  per (b, c): mean and rstd = 1 / sqrt(var + eps) over the D*H*W positions of
//           sample b.  Sums and sums of squares accumulate in fp64 (per thread, then per
//           workgroup, then one fp64 atomic per channel and workgroup), so E[x^2] - mean^2
//           loses nothing against PyTorch's fp32 Welford.
//   apply:  out = act((a - mean_a) * rstd_a + r'), r' = (r - mean_r) * rstd_r (norm3 of the
//           1x1 residual), r itself, or 0; act = LeakyReLU(slope) (slope 1 = identity).
// Both are one streaming pass over the tensor (HBM roofline).
#include "kernels.hpp"

namespace wf {

// grid (chunks, B); block 256 = R rows x C4 channel groups (R = 256 / C4)
__global__ __launch_bounds__(256) void instnorm_partial_kernel(
    const float* __restrict__ x, int64_t ldx, int C, int64_t P, int64_t chunk,
    double* __restrict__ acc) {
  extern __shared__ double red[];  // [R][C4][8]
  const int C4 = C >> 2;
  const int R = 256 / C4;
  const int tid = threadIdx.x;
  const int row = tid / C4, g = tid - row * C4;
  const int b = blockIdx.y;
  const int64_t p0 = (int64_t)blockIdx.x * chunk;
  const int64_t p1 = min(P, p0 + chunk);
  double s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
  if (row < R) {
    const float* base = x + ((int64_t)b * P) * ldx + 4 * g;
    for (int64_t p = p0 + row; p < p1; p += R) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(base + p * ldx);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double d = (double)v[j];
        s[j] += d;
        q[j] += d * d;
      }
    }
    double* r = red + ((int64_t)row * C4 + g) * 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r[j] = s[j];
      r[4 + j] = q[j];
    }
  }
  __syncthreads();
  // one thread per (channel, moment): sum the R rows, one atomic
  for (int i = tid; i < C * 2; i += blockDim.x) {
    const int c = i >> 1, mom = i & 1;
    const int gg = c >> 2, j = c & 3;
    double t = 0;
    for (int rr = 0; rr < R; ++rr) t += red[((int64_t)rr * C4 + gg) * 8 + 4 * mom + j];
    atomicAdd(acc + ((int64_t)b * C + c) * 2 + mom, t);
  }
}

__global__ void instnorm_finalize_kernel(const double* __restrict__ acc, float* __restrict__ stats,
                                         int B, int C, int64_t P, float eps) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * C) return;
  const int b = i / C, c = i - b * C;
  const double n = (double)P;
  const double mean = acc[2 * i] / n;
  double var = acc[2 * i + 1] / n - mean * mean;
  if (var < 0) var = 0;
  stats[(int64_t)(b * 2) * C + c] = (float)mean;
  stats[(int64_t)(b * 2 + 1) * C + c] = (float)(1.0 / sqrt(var + (double)eps));
}

// grid (chunks, B): a workgroup streams `chunk` positions of sample b; thread (row, g) owns
// channels 4g..4g+3 (its statistics in registers) and every R-th position (R = 256 / C4), so a
// wave's accesses are whole contiguous position rows and no per-element index division
__global__ __launch_bounds__(256) void norm_act_kernel(
    const float* __restrict__ a, int64_t lda, const float* __restrict__ sa,
    const float* __restrict__ r, int64_t ldr, const float* __restrict__ sr,
    float* __restrict__ out, int64_t ldo, int C, int64_t P, int64_t chunk, float slope) {
  const int C4 = C >> 2;
  const int R = 256 / C4;
  const int row = threadIdx.x / C4, g = threadIdx.x - row * C4;
  if (row >= R) return;
  const int b = blockIdx.y, c = 4 * g;
  const f32x4 ma = *reinterpret_cast<const f32x4*>(sa + (int64_t)(2 * b) * C + c);
  const f32x4 ra = *reinterpret_cast<const f32x4*>(sa + (int64_t)(2 * b + 1) * C + c);
  f32x4 mr = {0.f, 0.f, 0.f, 0.f}, rr = {1.f, 1.f, 1.f, 1.f};
  if (sr) {
    mr = *reinterpret_cast<const f32x4*>(sr + (int64_t)(2 * b) * C + c);
    rr = *reinterpret_cast<const f32x4*>(sr + (int64_t)(2 * b + 1) * C + c);
  }
  const int64_t p0 = (int64_t)blockIdx.x * chunk, p1 = min(P, p0 + chunk);
#pragma unroll 2
  for (int64_t p = p0 + row; p < p1; p += R) {
    const int64_t pos = (int64_t)b * P + p;
    f32x4 v = (*reinterpret_cast<const f32x4*>(a + pos * lda + c) - ma) * ra;
    if (r) v += (*reinterpret_cast<const f32x4*>(r + pos * ldr + c) - mr) * rr;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = v[j] >= 0.f ? v[j] : v[j] * slope;
    *reinterpret_cast<f32x4*>(out + pos * ldo + c) = v;
  }
}

// norm + LeakyReLU (no residual) stored as fp16 (round to nearest even): the input of the next
// WF_PREC_FP16 convolution, which stages exactly these operands (conv3d_k3_kernel<.., XH>)
__global__ __launch_bounds__(256) void norm_act_h_kernel(
    const float* __restrict__ a, int64_t lda, const float* __restrict__ sa,
    uint16_t* __restrict__ out, int64_t ldo, int C, int64_t P, int64_t chunk, float slope) {
  const int C4 = C >> 2;
  const int R = 256 / C4;
  const int row = threadIdx.x / C4, g = threadIdx.x - row * C4;
  if (row >= R) return;
  const int b = blockIdx.y, c = 4 * g;
  const f32x4 ma = *reinterpret_cast<const f32x4*>(sa + (int64_t)(2 * b) * C + c);
  const f32x4 ra = *reinterpret_cast<const f32x4*>(sa + (int64_t)(2 * b + 1) * C + c);
  const int64_t p0 = (int64_t)blockIdx.x * chunk, p1 = min(P, p0 + chunk);
#pragma unroll 2
  for (int64_t p = p0 + row; p < p1; p += R) {
    const int64_t pos = (int64_t)b * P + p;
    f32x4 v = (*reinterpret_cast<const f32x4*>(a + pos * lda + c) - ma) * ra;
    bf16x4 h;
#pragma unroll
    for (int j = 0; j < 4; ++j) h[j] = (short)f2h(v[j] >= 0.f ? v[j] : v[j] * slope);
    *reinterpret_cast<bf16x4*>(out + pos * ldo + c) = h;
  }
}

// (chunks, B) grid of the streaming elementwise kernels: ~4096 workgroups, chunk a multiple of
// the R rows a workgroup covers per step
static void stream_grid(int64_t B, int64_t P, int64_t C, int64_t* chunks, int64_t* chunk) {
  const int64_t R = 256 / (C / 4);
  int64_t n = cdiv(4096, B);
  int64_t ch = cdiv(P, n);
  ch = cdiv(ch, R) * R;
  if (ch < 4 * R) ch = 4 * R;
  *chunk = ch;
  *chunks = cdiv(P, ch);
}

// ---- a residual r = conv1x1(x) with few input channels (UnetResBlock's conv3 + norm3 when
// Cin < 8: encoder1, 4 -> 48), never materialised.  InstanceNorm of a linear map of x is fixed
// by x's per-sample mean and covariance: mean_r = W mean_x + b, var_r = W_c^T Cov_x W_c; the
// host folds r' = (r - mean_r) * rstd_r into per-sample weights W' = rstd_r W, b' = (b -
// mean_r) rstd_r (exact in real arithmetic), and norm_act reads K floats of x per position
// instead of the C-channel residual and its statistics pass.
// moments: acc (B, K + K*K) fp64 += sum_p x_k, sum_p x_k x_l; grid (chunks, B), 256 threads
template <int K>
__global__ __launch_bounds__(256) void moments_kernel(const float* __restrict__ x, int64_t ldx,
                                                      int64_t P, int64_t chunk,
                                                      double* __restrict__ acc) {
  constexpr int NM = K + K * (K + 1) / 2;
  __shared__ double red[4][NM];
  const int b = blockIdx.y;
  const int64_t p0 = (int64_t)blockIdx.x * chunk;
  const int64_t p1 = min(P, p0 + chunk);
  double m[NM];
#pragma unroll
  for (int i = 0; i < NM; ++i) m[i] = 0.0;
  const float* base = x + (int64_t)b * P * ldx;
  for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    double v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = (double)base[p * ldx + k];
    int i = K;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      m[k] += v[k];
#pragma unroll
      for (int l = k; l < K; ++l) m[i++] += v[k] * v[l];
    }
  }
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    double t = m[i];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o, 64);
    m[i] = t;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NM; ++i) red[w][i] = m[i];
  }
  __syncthreads();
  if (threadIdx.x < NM) {
    const int i = threadIdx.x;
    const double t = red[0][i] + red[1][i] + red[2][i] + red[3][i];
    // upper-triangle moment i -> both (k, l) and (l, k) of the K x K block
    if (i < K) {
      atomicAdd(acc + (int64_t)b * (K + K * K) + i, t);
    } else {
      int j = i - K, k = 0;
      while (j >= K - k) {
        j -= K - k;
        ++k;
      }
      const int l = k + j;
      double* q = acc + (int64_t)b * (K + K * K) + K;
      atomicAdd(q + k * K + l, t);
      if (l != k) atomicAdd(q + l * K + k, t);
    }
  }
}

// out = act((a - mean_a) * rstd_a + sum_k wf[b][c][k] x[p][k] + bf[b][c]); the (chunks, B)
// mapping of norm_act_kernel, the folded weights of the thread's 4 channels in registers
template <int K>
__global__ __launch_bounds__(256) void norm_act_lin_kernel(
    const float* __restrict__ a, int64_t lda, const float* __restrict__ sa,
    const float* __restrict__ x, int64_t ldx, const float* __restrict__ wf,
    const float* __restrict__ bf, float* __restrict__ out, int64_t ldo, int C, int64_t P,
    int64_t chunk, float slope, int xvec) {
  const int C4 = C >> 2;
  const int R = 256 / C4;
  const int row = threadIdx.x / C4, g = threadIdx.x - row * C4;
  if (row >= R) return;
  const int b = blockIdx.y, c = 4 * g;
  const f32x4 ma = *reinterpret_cast<const f32x4*>(sa + (int64_t)(2 * b) * C + c);
  const f32x4 ra = *reinterpret_cast<const f32x4*>(sa + (int64_t)(2 * b + 1) * C + c);
  const f32x4 bb = *reinterpret_cast<const f32x4*>(bf + (int64_t)b * C + c) - ma * ra;
  float w[4][K];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < K; ++k) w[j][k] = wf[((int64_t)b * C + c + j) * K + k];
  const bool x4 = K == 4 && xvec;  // one 16-B load of the position's x
  const int64_t p0 = (int64_t)blockIdx.x * chunk, p1 = min(P, p0 + chunk);
#pragma unroll 2
  for (int64_t p = p0 + row; p < p1; p += R) {
    const int64_t pos = (int64_t)b * P + p;
    float xv[K];
    if (x4) {
      const f32x4 t = *reinterpret_cast<const f32x4*>(x + pos * ldx);
#pragma unroll
      for (int k = 0; k < K; ++k) xv[k] = t[k & 3];
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) xv[k] = x[pos * ldx + k];
    }
    f32x4 v = *reinterpret_cast<const f32x4*>(a + pos * lda + c) * ra + bb;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int k = 0; k < K; ++k) v[j] = fmaf(w[j][k], xv[k], v[j]);
      v[j] = v[j] >= 0.f ? v[j] : v[j] * slope;
    }
    *reinterpret_cast<f32x4*>(out + pos * ldo + c) = v;
  }
}

// ---- backward of y = act((a - mean_a) * rstd_a + r'), act = LeakyReLU(slope) (training of
// UnetResBlock / UnetBasicBlock).  dz = dy * (y > 0 ? 1 : slope) -- the sign of y is the sign
// of the pre-activation for slope > 0, as the in-place LeakyReLU's own backward uses it.
// Pass 1: per (b, c) the sums of dz, dz * xhat_a and (normed residual) dz * xhat_r, fp64 per
// workgroup, one fp64 atomic per channel, moment and workgroup.  Pass 2 (elementwise):
//   da = rstd_a * (dz - S0 / P - xhat_a * S1 / P)
//   dr = rstd_r * (dz - S0 / P - xhat_r * S2 / P)   (normed residual)  |  dz  (plain residual)
struct NaBwd {
  const float* dy; int64_t ldd;
  const float* y; int64_t ldy;
  const float* a; int64_t lda;
  const float* sa;           // (B, 2, C) {mean, rstd}
  const float* r; int64_t ldr;
  const float* sr;           // (B, 2, C) or nullptr
  double* acc;               // (B, C, 3)
  float* da; int64_t ldda;
  float* dr; int64_t lddr;   // nullptr: no residual gradient wanted
  int C;
  int64_t P;
  float slope;
};

__global__ __launch_bounds__(256) void norm_act_bwd_reduce_kernel(NaBwd k, int64_t chunk) {
  extern __shared__ double red3[];  // [R][C4][12]
  const int C4 = k.C >> 2;
  const int R = 256 / C4;
  const int tid = threadIdx.x;
  const int row = tid / C4, g = tid - row * C4;
  const int b = blockIdx.y;
  const int64_t p0 = (int64_t)blockIdx.x * chunk;
  const int64_t p1 = min(k.P, p0 + chunk);
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  if (row < R) {
    const int c = 4 * g;
    const f32x4 ma = *reinterpret_cast<const f32x4*>(k.sa + (int64_t)(2 * b) * k.C + c);
    const f32x4 ra = *reinterpret_cast<const f32x4*>(k.sa + (int64_t)(2 * b + 1) * k.C + c);
    f32x4 mr = {0, 0, 0, 0}, rr = {0, 0, 0, 0};
    if (k.sr) {
      mr = *reinterpret_cast<const f32x4*>(k.sr + (int64_t)(2 * b) * k.C + c);
      rr = *reinterpret_cast<const f32x4*>(k.sr + (int64_t)(2 * b + 1) * k.C + c);
    }
    for (int64_t p = p0 + row; p < p1; p += R) {
      const int64_t pos = (int64_t)b * k.P + p;
      const f32x4 dy = *reinterpret_cast<const f32x4*>(k.dy + pos * k.ldd + c);
      const f32x4 y = *reinterpret_cast<const f32x4*>(k.y + pos * k.ldy + c);
      const f32x4 xa = (*reinterpret_cast<const f32x4*>(k.a + pos * k.lda + c) - ma) * ra;
      f32x4 xr = {0, 0, 0, 0};
      if (k.sr) xr = (*reinterpret_cast<const f32x4*>(k.r + pos * k.ldr + c) - mr) * rr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double dz = (double)(y[j] > 0.f ? dy[j] : dy[j] * k.slope);
        s0[j] += dz;
        s1[j] += dz * (double)xa[j];
        s2[j] += dz * (double)xr[j];
      }
    }
    double* rd = red3 + ((int64_t)row * C4 + g) * 12;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      rd[j] = s0[j];
      rd[4 + j] = s1[j];
      rd[8 + j] = s2[j];
    }
  }
  __syncthreads();
  const int nm = k.sr ? 3 : 2;
  for (int i = tid; i < k.C * nm; i += blockDim.x) {
    const int c = i / nm, mom = i - c * nm;
    const int gg = c >> 2, j = c & 3;
    double t = 0;
    for (int rr2 = 0; rr2 < R; ++rr2) t += red3[((int64_t)rr2 * C4 + gg) * 12 + 4 * mom + j];
    atomicAdd(k.acc + ((int64_t)b * k.C + c) * 3 + mom, t);
  }
}

__global__ __launch_bounds__(256) void norm_act_bwd_apply_kernel(NaBwd k, int64_t total) {
  const int C4 = k.C >> 2;
  const double invP = 1.0 / (double)k.P;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pos = i / C4;
    const int c = 4 * (int)(i - pos * C4);
    const int b = (int)(pos / k.P);
    const f32x4 ma = *reinterpret_cast<const f32x4*>(k.sa + (int64_t)(2 * b) * k.C + c);
    const f32x4 ra = *reinterpret_cast<const f32x4*>(k.sa + (int64_t)(2 * b + 1) * k.C + c);
    const f32x4 dy = *reinterpret_cast<const f32x4*>(k.dy + pos * k.ldd + c);
    const f32x4 y = *reinterpret_cast<const f32x4*>(k.y + pos * k.ldy + c);
    const f32x4 xa = (*reinterpret_cast<const f32x4*>(k.a + pos * k.lda + c) - ma) * ra;
    const double* ac = k.acc + ((int64_t)b * k.C + c) * 3;
    f32x4 dz, da, dr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dz[j] = y[j] > 0.f ? dy[j] : dy[j] * k.slope;
      const float m0 = (float)(ac[3 * j] * invP), m1 = (float)(ac[3 * j + 1] * invP);
      da[j] = ra[j] * (dz[j] - m0 - xa[j] * m1);
    }
    *reinterpret_cast<f32x4*>(k.da + pos * k.ldda + c) = da;
    if (k.dr) {
      if (k.sr) {
        const f32x4 mr = *reinterpret_cast<const f32x4*>(k.sr + (int64_t)(2 * b) * k.C + c);
        const f32x4 rr = *reinterpret_cast<const f32x4*>(k.sr + (int64_t)(2 * b + 1) * k.C + c);
        const f32x4 xr = (*reinterpret_cast<const f32x4*>(k.r + pos * k.ldr + c) - mr) * rr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float m0 = (float)(ac[3 * j] * invP), m2 = (float)(ac[3 * j + 2] * invP);
          dr[j] = rr[j] * (dz[j] - m0 - xr[j] * m2);
        }
      } else {
        dr = dz;
      }
      *reinterpret_cast<f32x4*>(k.dr + pos * k.lddr + c) = dr;
    }
  }
}

}  // namespace wf

using namespace wf;

extern "C" int64_t wf_norm_act_bwd_workspace_bytes(int64_t B, int64_t C) {
  return B * C * 3 * (int64_t)sizeof(double);
}

extern "C" int wf_norm_act_bwd_cl(const float* dy, int64_t ldd, const float* y, int64_t ldy,
                                  const float* a, int64_t lda, const float* stats_a,
                                  const float* r, int64_t ldr, const float* stats_r,
                                  float* da, int64_t ldda, float* dr, int64_t lddr, int64_t B,
                                  int64_t C, int64_t P, float slope, void* workspace,
                                  void* stream) {
  WF_REQUIRE(B >= 1 && P >= 1, "empty tensor");
  WF_REQUIRE(C >= 4 && C % 4 == 0 && C <= 1024, "C must be a multiple of 4 in [4, 1024]");
  WF_REQUIRE(ldd >= C && ldy >= C && lda >= C && ldda >= C && ldd % 4 == 0 && ldy % 4 == 0 &&
             lda % 4 == 0 && ldda % 4 == 0 && (!dr || (lddr >= C && lddr % 4 == 0)) &&
             (!stats_r || (r && ldr >= C && ldr % 4 == 0)),
             "every ld must be >= C and a multiple of 4");
  WF_REQUIRE_PTR(dy);
  WF_REQUIRE_PTR(y);
  WF_REQUIRE_PTR(a);
  WF_REQUIRE_PTR(stats_a);
  WF_REQUIRE_PTR(da);
  WF_REQUIRE_PTR(workspace);
  NaBwd k{dy, ldd, y, ldy, a, lda, stats_a, r, ldr, stats_r,
          reinterpret_cast<double*>(workspace), da, ldda, dr, lddr, (int)C, P, slope};
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(k.acc, 0, (size_t)wf_norm_act_bwd_workspace_bytes(B, C), s) != hipSuccess)
    return check_launch("wf_norm_act_bwd_cl (memset)");
  const int C4 = (int)(C / 4);
  const int R = 256 / C4;
  int64_t chunks = cdiv(1024, B);
  int64_t chunk = cdiv(P, chunks);
  if (chunk < 4 * R) chunk = 4 * R;
  chunks = cdiv(P, chunk);
  const size_t lds = (size_t)R * C4 * 12 * sizeof(double);
  hipLaunchKernelGGL(norm_act_bwd_reduce_kernel, dim3((unsigned)chunks, (unsigned)B), dim3(256),
                     lds, s, k, chunk);
  int rc = check_launch("wf_norm_act_bwd_cl (reduce)");
  if (rc) return rc;
  const int64_t total = B * P * C4;
  int64_t blocks = cdiv(total, 256);
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(norm_act_bwd_apply_kernel, dim3((unsigned)blocks), dim3(256), 0, s, k,
                     total);
  return check_launch("wf_norm_act_bwd_cl (apply)");
}

extern "C" int64_t wf_instnorm_workspace_bytes(int64_t B, int64_t C) {
  return B * C * 2 * (int64_t)sizeof(double);
}

// partial sums into a zeroed (B, C, 2) fp64 accumulator (shared with conv3d.hip's split-K path)
int wf::launch_instnorm_partial(const float* x, int64_t ldx, int64_t B, int64_t C, int64_t P,
                            double* acc, hipStream_t s) {
  const int C4 = (int)(C / 4);
  const int R = 256 / C4;
  int64_t chunks = cdiv(1024, B);
  int64_t chunk = cdiv(P, chunks);
  if (chunk < 4 * R) chunk = 4 * R;
  chunks = cdiv(P, chunk);
  const size_t lds = (size_t)R * C4 * 8 * sizeof(double);
  hipLaunchKernelGGL(instnorm_partial_kernel, dim3((unsigned)chunks, (unsigned)B), dim3(256), lds,
                     s, x, ldx, (int)C, P, chunk, acc);
  return check_launch("instnorm partial sums");
}

extern "C" int wf_instnorm_finalize(const double* acc, float* stats, int64_t B, int64_t C,
                                    int64_t P, float eps, void* stream) {
  WF_REQUIRE(B >= 1 && C >= 1 && P >= 1, "empty tensor");
  WF_REQUIRE_PTR(acc);
  WF_REQUIRE_PTR(stats);
  hipLaunchKernelGGL(instnorm_finalize_kernel, dim3((unsigned)cdiv(B * C, 256)), dim3(256), 0,
                     (hipStream_t)stream, acc, stats, (int)B, (int)C, P, eps);
  return check_launch("wf_instnorm_finalize");
}

extern "C" int wf_instnorm_stats_cl(const float* x, int64_t ldx, int64_t B, int64_t C,
                                    int64_t P, float eps, float* stats, void* workspace,
                                    void* stream) {
  WF_REQUIRE(B >= 1 && P >= 1, "empty tensor");
  WF_REQUIRE(C >= 4 && C % 4 == 0 && C <= 1024 && ldx >= C && ldx % 4 == 0,
             "C must be a multiple of 4 in [4, 1024] with ldx >= C, ldx % 4 == 0");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(stats);
  WF_REQUIRE_PTR(workspace);
  hipStream_t s = (hipStream_t)stream;
  double* acc = reinterpret_cast<double*>(workspace);
  if (hipMemsetAsync(acc, 0, (size_t)(B * C * 2) * sizeof(double), s) != hipSuccess)
    return check_launch("wf_instnorm_stats_cl (memset)");
  const int C4 = (int)(C / 4);
  const int R = 256 / C4;
  // ~1024 workgroups over the batch, at least 4 rows per thread
  int64_t chunks = cdiv(1024, B);
  int64_t chunk = cdiv(P, chunks);
  if (chunk < 4 * R) chunk = 4 * R;
  chunks = cdiv(P, chunk);
  const size_t lds = (size_t)R * C4 * 8 * sizeof(double);
  hipLaunchKernelGGL(instnorm_partial_kernel, dim3((unsigned)chunks, (unsigned)B), dim3(256), lds,
                     s, x, ldx, (int)C, P, chunk, acc);
  int rc = check_launch("wf_instnorm_stats_cl");
  if (rc) return rc;
  hipLaunchKernelGGL(instnorm_finalize_kernel, dim3((unsigned)cdiv(B * C, 256)), dim3(256), 0, s,
                     acc, stats, (int)B, (int)C, P, eps);
  return check_launch("wf_instnorm_stats_cl (finalize)");
}

extern "C" int wf_norm_act_cl(const float* a, int64_t lda, const float* stats_a, const float* r,
                              int64_t ldr, const float* stats_r, float* out, int64_t ldo,
                              int64_t B, int64_t C, int64_t P, float slope, void* stream) {
  WF_REQUIRE(B >= 1 && P >= 1, "empty tensor");
  WF_REQUIRE(C >= 4 && C % 4 == 0 && lda >= C && lda % 4 == 0 && ldo >= C && ldo % 4 == 0 &&
             (!r || (ldr >= C && ldr % 4 == 0)),
             "C must be a multiple of 4 and every ld >= C, a multiple of 4");
  WF_REQUIRE_PTR(a);
  WF_REQUIRE_PTR(stats_a);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE(C <= 1024, "C must be <= 1024");
  int64_t chunks, chunk;
  stream_grid(B, P, C, &chunks, &chunk);
  hipLaunchKernelGGL(norm_act_kernel, dim3((unsigned)chunks, (unsigned)B), dim3(256), 0,
                     (hipStream_t)stream, a, lda, stats_a, r, ldr, stats_r, out, ldo, (int)C, P,
                     chunk, slope);
  return check_launch("wf_norm_act_cl");
}

extern "C" int wf_moments_cl(const float* x, int64_t ldx, int64_t B, int64_t K, int64_t P,
                             double* acc, void* stream) {
  WF_REQUIRE(B >= 1 && P >= 1, "empty tensor");
  WF_REQUIRE(K >= 1 && K <= 7 && ldx >= K, "K must be in [1, 7] with ldx >= K");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(acc);
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(acc, 0, (size_t)(B * (K + K * K)) * sizeof(double), s) != hipSuccess)
    return check_launch("wf_moments_cl (memset)");
  int64_t chunks = cdiv(2048, B);
  int64_t chunk = cdiv(P, chunks);
  if (chunk < 1024) chunk = 1024;
  chunks = cdiv(P, chunk);
  const dim3 grid((unsigned)chunks, (unsigned)B);
  switch (K) {
#define WF_MOM(k) case k: hipLaunchKernelGGL(moments_kernel<k>, grid, dim3(256), 0, s, x, ldx, P, chunk, acc); break;
    WF_MOM(1) WF_MOM(2) WF_MOM(3) WF_MOM(4) WF_MOM(5) WF_MOM(6) WF_MOM(7)
#undef WF_MOM
  }
  return check_launch("wf_moments_cl");
}

extern "C" int wf_norm_act_lin_cl(const float* a, int64_t lda, const float* stats_a,
                                  const float* x, int64_t ldx, int64_t K, const float* wfold,
                                  const float* bfold, float* out, int64_t ldo, int64_t B,
                                  int64_t C, int64_t P, float slope, void* stream) {
  WF_REQUIRE(B >= 1 && P >= 1, "empty tensor");
  WF_REQUIRE(C >= 4 && C % 4 == 0 && lda >= C && lda % 4 == 0 && ldo >= C && ldo % 4 == 0,
             "C must be a multiple of 4 and every ld >= C, a multiple of 4");
  WF_REQUIRE(K >= 1 && K <= 7 && ldx >= K, "K must be in [1, 7] with ldx >= K");
  WF_REQUIRE_PTR(a);
  WF_REQUIRE_PTR(stats_a);
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(wfold);
  WF_REQUIRE_PTR(bfold);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE(C <= 1024, "C must be <= 1024");
  int64_t chunks, chunk;
  stream_grid(B, P, C, &chunks, &chunk);
  const dim3 grid((unsigned)chunks, (unsigned)B);
  const int xvec = (ldx % 4 == 0) && (((uintptr_t)x & 15) == 0);
  hipStream_t s = (hipStream_t)stream;
  switch (K) {
#define WF_NAL(k) case k: hipLaunchKernelGGL(norm_act_lin_kernel<k>, grid, dim3(256), 0, s, a, lda, stats_a, x, ldx, wfold, bfold, out, ldo, (int)C, P, chunk, slope, xvec); break;
    WF_NAL(1) WF_NAL(2) WF_NAL(3) WF_NAL(4) WF_NAL(5) WF_NAL(6) WF_NAL(7)
#undef WF_NAL
  }
  return check_launch("wf_norm_act_lin_cl");
}

extern "C" int wf_norm_act_h_cl(const float* a, int64_t lda, const float* stats_a, uint16_t* out,
                                int64_t ldo, int64_t B, int64_t C, int64_t P, float slope,
                                void* stream) {
  WF_REQUIRE(B >= 1 && P >= 1, "empty tensor");
  WF_REQUIRE(C >= 4 && C % 4 == 0 && C <= 1024 && lda >= C && lda % 4 == 0 && ldo >= C &&
             ldo % 4 == 0, "C must be a multiple of 4 in [4, 1024], every ld >= C, % 4 == 0");
  WF_REQUIRE_PTR(a);
  WF_REQUIRE_PTR(stats_a);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE(((uintptr_t)out & 7) == 0, "out must be 8-byte aligned");
  int64_t chunks, chunk;
  stream_grid(B, P, C, &chunks, &chunk);
  hipLaunchKernelGGL(norm_act_h_kernel, dim3((unsigned)chunks, (unsigned)B), dim3(256), 0,
                     (hipStream_t)stream, a, lda, stats_a, out, ldo, (int)C, P, chunk, slope);
  return check_launch("wf_norm_act_h_cl");
}
