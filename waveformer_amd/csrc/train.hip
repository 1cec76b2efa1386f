// train.hip -- backward kernels of the encoder hot path (config 4: fwd + bwd DiceCE, DDP).
//
// The forward kernels fuse aggressively (norm1 into the DWT, norm2 into the FFN loader, h2 kept
// on chip).  Training re-enters at the module boundaries the reference's autograd sees:
//   Haar DWT (wave_helper.py:350)  adjoint = inverse butterfly (orthonormal filters)
//   Haar IDWT (idwt_upsample.py:160) adjoint = analysis of the output gradient
//   windowed attention (attention.py:83-104): recompute S from the saved qkv and the per-row
//     log-sum-exp of the forward, dV = P^T dO, dS = P (dP - rowsum(dO o O)), dQ/dK, and the
//     relative-position bias gradient summed over windows, then scattered into the table
//   trilinear fuse (wave_helper.py:500): per-axis adjoint of the interpolation
//   LayerNorm (+ GELU) rows, depthwise 3^3 conv (dgrad = conv with the flipped kernel, wgrad
//     = per-channel correlation), PatchMerging gather (Q3 duplicates accumulate), PatchEmbed
//     patch gather, NCDHW -> channel-last transpose (proj_out)
// The dense GEMM gradients (dX = dY W, dW = dY^T X) are plain library GEMMs (hipBLASLt via
// torch.mm on the caller's side).  Everything here is fp32 VALU arithmetic: exact enough for
// the fp32 reference's training and free of the split-bf16 bookkeeping.
#include "kernels.hpp"

namespace wf {

// ------------------------------------------------------------------------------------------
// column sums: partial sums of row chunks, then one reduction block per column chunk
// ------------------------------------------------------------------------------------------
constexpr int kColsumMaxParts = 1024;

int64_t colsum_parts(int64_t R) {
  int64_t p = cdiv(R, 256);
  return p > kColsumMaxParts ? kColsumMaxParts : (p < 1 ? 1 : p);
}

// block (part p, column chunk): rows [p*rpp, (p+1)*rpp); 256 threads = 64 columns x 4 phases
__global__ __launch_bounds__(256) void colsum_part_kernel(const float* __restrict__ in,
                                                          int64_t R, int64_t N, int64_t rpp,
                                                          const float* __restrict__ rscale,
                                                          int64_t rows_per_scale,
                                                          float* __restrict__ part) {
  __shared__ float red[4][64];
  const int tc = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.y * 64 + tc;
  const int64_t r0 = blockIdx.x * rpp, r1 = min(R, r0 + rpp);
  float acc = 0.f;
  if (c < N) {
    for (int64_t r = r0 + ph; r < r1; r += 4) {
      const float v = in[r * N + c];
      acc += rscale ? v * rscale[r / rows_per_scale] : v;
    }
  }
  red[ph][tc] = acc;
  __syncthreads();
  if (ph == 0 && c < N)
    part[(int64_t)blockIdx.x * N + c] = (red[0][tc] + red[1][tc]) + (red[2][tc] + red[3][tc]);
}

// one wave per column: lane l sums parts l, l + 64, ... in order, then a fixed xor tree over
// the lanes (deterministic; the one-thread-per-column form ran a 1024-long dependent chain,
// ~100 us per call, 47 calls per config-4 step)
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part,
                                                           int64_t P, int64_t N,
                                                           float* __restrict__ out) {
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= N) return;
  float acc = 0.f;
  for (int64_t p = lane; p < P; p += 64) acc += part[p * N + c];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) out[c] = acc;
}

int launch_colsum(const float* in, int64_t R, int64_t N, const float* rscale,
                  int64_t rows_per_scale, float* part, float* out, hipStream_t s) {
  if (N <= 0) return WF_OK;
  const int64_t P = colsum_parts(R);
  if (R <= 0) return hipMemsetAsync(out, 0, N * sizeof(float), s) == hipSuccess
                         ? WF_OK : check_launch("colsum memset");
  const int64_t rpp = cdiv(R, P);
  hipLaunchKernelGGL(colsum_part_kernel, dim3((unsigned)P, (unsigned)cdiv(N, 64)), dim3(256), 0,
                     s, in, R, N, rpp, rscale, rows_per_scale > 0 ? rows_per_scale : R, part);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((unsigned)cdiv(N, 4)), dim3(256), 0, s, part,
                     P, N, out);
  return check_launch("colsum");
}

// ------------------------------------------------------------------------------------------
// LayerNorm (+ GELU) rows: one wave per row, J = ceil(N / 64) values per lane in registers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float gelu_exact(float z) {
  return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_grad(float z) {
  // d/dz [z Phi(z)] = Phi(z) + z phi(z)
  return 0.5f * (1.f + erff(z * 0.70710678118654752f)) +
         z * 0.39894228040143268f * expf(-0.5f * z * z);
}

template <int J>
__device__ __forceinline__ void row_stats(const float (&v)[J], int N, int lane, float& mean,
                                          float& rstd, float eps) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j) s += (lane + 64 * j < N) ? v[j] : 0.f;
  mean = wave_sum(s) / (float)N;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const float d = v[j] - mean;
    q += (lane + 64 * j < N) ? d * d : 0.f;
  }
  rstd = rsqrtf(wave_sum(q) / (float)N + eps);  // biased variance, as nn.LayerNorm
}

template <int J>
__global__ __launch_bounds__(256) void ln_act_fwd_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ b, float eps,
                                                         int gelu, float* __restrict__ y,
                                                         int64_t M, int N) {
  const int lane = threadIdx.x & 63;
  const int64_t wv = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wv; r < M; r += nw) {
    const float* xr = x + r * N;
    float v[J];
#pragma unroll
    for (int j = 0; j < J; ++j) v[j] = (lane + 64 * j < N) ? xr[lane + 64 * j] : 0.f;
    float mean, rstd;
    row_stats<J>(v, N, lane, mean, rstd, eps);
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int c = lane + 64 * j;
      if (c >= N) continue;
      float z = (v[j] - mean) * rstd;
      if (w) z = z * w[c] + b[c];
      y[r * N + c] = gelu ? gelu_exact(z) : z;
    }
  }
}

// dx = [dadd +] LN_bwd(dz), dz = dy (* GELU'(z) when gelu), z = LN(x) (affine when w != NULL).
// Per-block partial sums of dgamma = sum dz * xhat and dbeta = sum dz go to
// part[blockIdx.x][0 .. N) and part[blockIdx.x][N .. 2N).
template <int J>
__global__ __launch_bounds__(256) void ln_act_bwd_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ b, float eps,
                                                         int gelu, const float* __restrict__ dy,
                                                         const float* __restrict__ dadd,
                                                         float* __restrict__ dx,
                                                         float* __restrict__ part, int64_t M,
                                                         int N) {
  __shared__ float red[4][2][J * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t wv = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  float gw[J], gb[J];
#pragma unroll
  for (int j = 0; j < J; ++j) gw[j] = gb[j] = 0.f;
  for (int64_t r = wv; r < M; r += nw) {
    float v[J], d[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int c = lane + 64 * j;
      v[j] = c < N ? x[r * N + c] : 0.f;
      d[j] = c < N ? dy[r * N + c] : 0.f;
    }
    float mean, rstd;
    row_stats<J>(v, N, lane, mean, rstd, eps);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int c = lane + 64 * j;
      const bool ok = c < N;
      const float xh = (v[j] - mean) * rstd;
      const float wc = (w && ok) ? w[c] : 1.f;
      float dz = d[j];
      if (gelu) {
        const float z = w ? xh * wc + (ok ? b[c] : 0.f) : xh;
        dz *= gelu_grad(z);
      }
      dz = ok ? dz : 0.f;
      gw[j] += dz * xh;
      gb[j] += dz;
      const float dxh = dz * wc;
      s1 += dxh;
      s2 += dxh * xh;
      v[j] = xh;
      d[j] = dxh;
    }
    s1 = wave_sum(s1) / (float)N;
    s2 = wave_sum(s2) / (float)N;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int c = lane + 64 * j;
      if (c >= N) continue;
      float g = rstd * (d[j] - s1 - v[j] * s2);
      if (dadd) g += dadd[r * N + c];
      dx[r * N + c] = g;
    }
  }
  if (!part) return;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    red[wid][0][lane + 64 * j] = gw[j];
    red[wid][1][lane + 64 * j] = gb[j];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * N; i += blockDim.x) {
    const int k = i / N, c = i % N;
    part[(int64_t)blockIdx.x * 2 * N + i] =
        (red[0][k][c] + red[1][k][c]) + (red[2][k][c] + red[3][k][c]);
  }
}

int64_t ln_parts(int64_t M) {
  int64_t g = cdiv(M, 16);  // >= 4 rows per wave
  return g > 1024 ? 1024 : (g < 1 ? 1 : g);
}

#define WF_LN_DISPATCH(N, MACRO) \
  if (N <= 64) { MACRO(1) }      \
  else if (N <= 128) { MACRO(2) } \
  else if (N <= 192) { MACRO(3) } \
  else if (N <= 256) { MACRO(4) } \
  else if (N <= 384) { MACRO(6) } \
  else if (N <= 512) { MACRO(8) } \
  else if (N <= 768) { MACRO(12) } \
  else if (N <= 1024) { MACRO(16) } \
  else { MACRO(24) }

// ------------------------------------------------------------------------------------------
// Haar adjoints.  Band k = (kd << 2) | (kh << 1) | kw  ('a' = 0, 'd' = 1; ptwt key order).
// Analysis: band_k = sum_{i,j,l} x[2z+i][2y+j][2x+l] s(kd,i) s(kh,j) s(kw,l) / (2 sqrt 2),
// s(0, .) = 1, s(1, i) = (i ? -1 : 1).  The matrix is orthogonal and symmetric up to the
// index roles, so synthesis (= the analysis adjoint) uses the same signs.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void haar8(float (&v)[8]) {
  // v indexed by (i<<2)|(j<<1)|l on input, by k on output (same butterfly both ways)
  const float r = 0.35355339059327373f;  // 1 / (2 sqrt 2)
#pragma unroll
  for (int bit = 1; bit < 8; bit <<= 1) {
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      if (a & bit) continue;
      const float p = v[a], q = v[a | bit];
      v[a] = p + q;
      v[a | bit] = p - q;
    }
  }
#pragma unroll
  for (int a = 0; a < 8; ++a) v[a] *= r;
}

struct BandPtrs {
  const float* p[8];
  int64_t s[8][5];  // (b, z, y, x, c) element strides
};

// dx (B, D, H, W, C) channel-last = synthesis of 8 band gradients (NULL band = 0)
__global__ __launch_bounds__(256) void dwt_bwd_cl_kernel(BandPtrs bp, float* __restrict__ dx,
                                                         int B, int C, int d, int h, int w) {
  const int64_t n = (int64_t)B * d * h * w * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    int64_t t = i / C;
    const int x = (int)(t % w);
    t /= w;
    const int y = (int)(t % h);
    t /= h;
    const int z = (int)(t % d);
    const int b = (int)(t / d);
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float* p = bp.p[k];
      v[k] = p ? p[b * bp.s[k][0] + z * bp.s[k][1] + y * bp.s[k][2] + x * bp.s[k][3] +
                   c * bp.s[k][4]]
               : 0.f;
    }
    haar8(v);
    const int64_t H2 = 2 * h, W2 = 2 * w;
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      const int64_t zz = 2 * z + (a >> 2), yy = 2 * y + ((a >> 1) & 1), xx = 2 * x + (a & 1);
      dx[((((int64_t)b * 2 * d + zz) * H2 + yy) * W2 + xx) * C + c] = v[a];
    }
  }
}

// one analysis level of an NCDHW gradient: in (B, C, 2d, 2h, 2w) at in + b*in_bs + c*in_cs
// -> band 0 into ll (NCDHW contiguous (B, C, d, h, w)), bands 1..7 into det[k-1] at
// b*s0 + c*s1 + z*s2 + y*s3 + x*s4
struct DetOut {
  float* p[7];
  int64_t s[5];
};
__global__ __launch_bounds__(256) void haar_analysis_ncdhw_kernel(
    const float* __restrict__ in, int64_t in_bs, int64_t in_cs, float* __restrict__ ll,
    DetOut det, int B, int C, int d, int h, int w) {
  const int64_t n = (int64_t)B * C * d * h * w;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % w);
    int64_t t = i / w;
    const int y = (int)(t % h);
    t /= h;
    const int z = (int)(t % d);
    t /= d;
    const int c = (int)(t % C);
    const int b = (int)(t / C);
    const float* src = in + b * in_bs + c * in_cs;
    const int64_t W2 = 2 * w, HW2 = (int64_t)2 * h * W2;
    float v[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      const int64_t zz = 2 * z + (a >> 2), yy = 2 * y + ((a >> 1) & 1), xx = 2 * x + (a & 1);
      v[a] = src[zz * HW2 + yy * W2 + xx];
    }
    haar8(v);
    ll[i] = v[0];
    const int64_t o = b * det.s[0] + c * det.s[1] + z * det.s[2] + y * det.s[3] + x * det.s[4];
#pragma unroll
    for (int k = 1; k < 8; ++k) det.p[k - 1][o] = v[k];
  }
}

// ------------------------------------------------------------------------------------------
// window attention backward (fp32 VALU), deterministic: no atomics, every sum in a fixed order.
// One workgroup = (64-key block kb, head, window group g); it walks the windows g, g + G, ...
// in order, and per window the 64-query blocks:  S = scale q k^T + bias,
// P = exp2(S log2e - lse2), dP = dO v^T, dS = P (dP - D), D = rowsum(dO o O);
// dV = P^T dO, dK = scale dS^T q (registers, written once per window to the raster row);
// dQ (unscaled) of this key block -> dq_part[kb][window-major row] (each element written by
// exactly one workgroup); dBias -> db_part[g][h][q][key], owned by this workgroup and summed
// over its windows in order.  attn_dq_reduce / attn_db_reduce then add the key-block / group
// partials in index order.  qkv / O / dO / lse are window-major; dqkv rows are RASTER rows of
// the token (the inverse of window_partition), so the qkv weight gradient pairs them with the
// un-permuted (normed) raster.
// ------------------------------------------------------------------------------------------
constexpr int kAB = 64;

struct AttnBwdArgs {
  const float* qkv;   // (Bw*N, 3C) window-major
  const float* o;     // (Bw*N, C) attention output (pre-proj)
  const float* dout;  // (Bw*N, C) gradient of o
  const float* bias;  // (heads, N, N)
  const float* lse;   // (Bw, heads, N) log2-domain row log-sum-exp of the forward
  float* dqkv;        // (B*D1*H1*W1, 3C) raster rows: dK / dV columns written here
  float* dq_part;     // (nkb, Bw*N, C) window-major, unscaled
  float* db_part;     // (G, heads, N, N)
  int64_t Bw;
  int N, heads, C, ws, nD, nH, nW;  // windows per axis
  int G;
  float scale, scale_log2;
};

__device__ __forceinline__ int64_t raster_row_of(int64_t bw, int t, int ws, int nD, int nH,
                                                 int nW) {
  int64_t r = bw;
  const int ww = (int)(r % nW);
  r /= nW;
  const int wh = (int)(r % nH);
  r /= nH;
  const int wd = (int)(r % nD);
  const int64_t b = r / nD;
  const int tx = t % ws, ty = (t / ws) % ws, tz = t / (ws * ws);
  const int64_t D1 = (int64_t)nD * ws, H1 = (int64_t)nH * ws, W1 = (int64_t)nW * ws;
  return ((b * D1 + wd * ws + tz) * H1 + wh * ws + ty) * W1 + ww * ws + tx;
}

template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_kernel(AttnBwdArgs a) {
  constexpr int HP = HD + 1;
  constexpr int DPT = HD / 4;  // head-dim values per thread in the 64 x HD phases
  __shared__ float Ks[kAB][HP], Vs[kAB][HP], Qs[kAB][HP], dOs[kAB][HP];
  __shared__ float Ps[kAB][kAB + 1], dSs[kAB][kAB + 1];
  __shared__ float Ls[kAB], Dq[kAB];
  const int tid = threadIdx.x;
  const int kb = blockIdx.x, h = blockIdx.y, g = blockIdx.z;
  const int N = a.N, C = a.C, ld = 3 * C;
  const int k0 = kb * kAB;
  // phase-2 ownership: key/query row pr = tid / 4, head-dim chunk d0
  const int pr = tid >> 2, d0 = (tid & 3) * DPT;
  // S-tile ownership: queries ti*4 .. +3, keys tj*4 .. +3
  const int ti = tid >> 4, tj = tid & 15;
  float* dq_base = a.dq_part + (int64_t)kb * a.Bw * N * C;

  for (int64_t bw = g; bw < a.Bw; bw += a.G) {
    const bool first = bw == g;
    const int64_t row0 = bw * N;
    __syncthreads();  // the previous window is done with Ks / Vs
    // this block's keys / values
    for (int i = tid; i < kAB * HD; i += 256) {
      const int r = i / HD, dd = i % HD;
      const int key = k0 + r;
      float kv = 0.f, vv = 0.f;
      if (key < N) {
        const float* p = a.qkv + (row0 + key) * ld + h * HD + dd;
        kv = p[C];
        vv = p[2 * C];
      }
      Ks[r][dd] = kv;
      Vs[r][dd] = vv;
    }
    float dk[DPT], dv[DPT];
#pragma unroll
    for (int e = 0; e < DPT; ++e) dk[e] = dv[e] = 0.f;

    for (int q0 = 0; q0 < N; q0 += kAB) {
      __syncthreads();  // previous iteration done with Qs / dOs / Ps / dSs
      for (int i = tid; i < kAB * HD; i += 256) {
        const int r = i / HD, dd = i % HD;
        const int q = q0 + r;
        float qv = 0.f, gv = 0.f;
        if (q < N) {
          qv = a.qkv[(row0 + q) * ld + h * HD + dd];
          gv = a.dout[(row0 + q) * C + h * HD + dd];
        }
        Qs[r][dd] = qv;
        dOs[r][dd] = gv;
      }
      {  // D = rowsum(dO o O): 4 lanes per query
        const int q = q0 + pr;
        float s = 0.f;
        if (q < N) {
          const float* op = a.o + (row0 + q) * C + h * HD + d0;
          const float* gp = a.dout + (row0 + q) * C + h * HD + d0;
#pragma unroll
          for (int e = 0; e < DPT; ++e) s += op[e] * gp[e];
        }
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        if ((tid & 3) == 0) {
          Dq[pr] = s;
          Ls[pr] = q < N ? a.lse[(bw * a.heads + h) * N + q] : 0.f;
        }
      }
      __syncthreads();
      // S, dP microtiles
      float s[4][4], dp[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) s[i][j] = dp[i][j] = 0.f;
#pragma unroll
      for (int dd = 0; dd < HD; ++dd) {
        float qv[4], gv[4], kv[4], vv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          qv[i] = Qs[ti * 4 + i][dd];
          gv[i] = dOs[ti * 4 + i][dd];
          kv[i] = Ks[tj * 4 + i][dd];
          vv[i] = Vs[tj * 4 + i][dd];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            s[i][j] = fmaf(qv[i], kv[j], s[i][j]);
            dp[i][j] = fmaf(gv[i], vv[j], dp[i][j]);
          }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ql = ti * 4 + i, q = q0 + ql;
        const bool qok = q < N;
        const float* brow = a.bias + ((int64_t)h * N + (qok ? q : 0)) * N;
        float* dbrow = a.db_part + (((int64_t)g * a.heads + h) * N + (qok ? q : 0)) * N;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int kl = tj * 4 + j, key = k0 + kl;
          const bool ok = qok && key < N;
          float p = 0.f, ds = 0.f;
          if (ok) {
            p = exp2f(s[i][j] * a.scale_log2 + brow[key] * 1.4426950408889634f - Ls[ql]);
            ds = p * (dp[i][j] - Dq[ql]);
            // this thread owns db_part[g][h][q][key]: the windows of group g add in order
            dbrow[key] = first ? ds : dbrow[key] + ds;
          }
          Ps[ql][kl] = p;
          dSs[ql][kl] = ds;
        }
      }
      __syncthreads();
      // dV, dK for key pr; this key block's dQ for query pr
      {
        const int kl = pr;
        for (int ql = 0; ql < kAB; ++ql) {
          const float p = Ps[ql][kl], ds = dSs[ql][kl];
#pragma unroll
          for (int e = 0; e < DPT; ++e) {
            dv[e] = fmaf(p, dOs[ql][d0 + e], dv[e]);
            dk[e] = fmaf(ds, Qs[ql][d0 + e], dk[e]);
          }
        }
        const int ql = pr, q = q0 + ql;
        if (q < N) {
          float dq[DPT];
#pragma unroll
          for (int e = 0; e < DPT; ++e) dq[e] = 0.f;
          for (int k = 0; k < kAB; ++k) {
            const float ds = dSs[ql][k];
#pragma unroll
            for (int e = 0; e < DPT; ++e) dq[e] = fmaf(ds, Ks[k][d0 + e], dq[e]);
          }
          float* dst = dq_base + (row0 + q) * C + h * HD + d0;
#pragma unroll
          for (int e = 0; e < DPT; ++e) dst[e] = dq[e];
        }
      }
    }
    const int key = k0 + pr;
    if (key < N) {
      float* dst = a.dqkv + raster_row_of(bw, key, a.ws, a.nD, a.nH, a.nW) * ld + h * HD + d0;
#pragma unroll
      for (int e = 0; e < DPT; ++e) {
        dst[C + e] = dk[e] * a.scale;
        dst[2 * C + e] = dv[e];
      }
    }
  }
}

// dQ of window-major row wr = scale * sum_kb dq_part[kb][wr] (kb ascending) -> the q columns of
// the token's raster row; one thread per (row, 4 channels)
__global__ __launch_bounds__(256) void attn_dq_reduce_kernel(const float* __restrict__ part,
                                                             float* __restrict__ dqkv,
                                                             int64_t rows, int C, int nkb,
                                                             float scale, int ws, int nD, int nH,
                                                             int nW) {
  const int C4 = C >> 2;
  const int64_t total = rows * C4;
  const int N = ws * ws * ws;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t wr = i / C4;
    const int c = 4 * (int)(i - wr * C4);
    f32x4 s = *reinterpret_cast<const f32x4*>(part + wr * C + c);
    for (int k = 1; k < nkb; ++k)
      s += *reinterpret_cast<const f32x4*>(part + ((int64_t)k * rows + wr) * C + c);
    const int64_t bw = wr / N;
    const int t = (int)(wr - bw * N);
    *reinterpret_cast<f32x4*>(dqkv + raster_row_of(bw, t, ws, nD, nH, nW) * 3 * C + c) =
        s * scale;
  }
}

// dbias[e] = sum_g db_part[g][e] (g ascending), e over heads * N * N
__global__ __launch_bounds__(256) void attn_db_reduce_kernel(const float* __restrict__ part,
                                                             float* __restrict__ dbias,
                                                             int64_t n, int G) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float s = part[i];
    for (int g = 1; g < G; ++g) s += part[(int64_t)g * n + i];
    dbias[i] = s;
  }
}

// dtable[r][h] = sum over the (i, j) with index[i][j] == r, in ascending flat order, of
// dbias[h][i][j] -- the adjoint of the gather at attention.py:94-97 without atomics: `perm`
// lists the flat positions grouped by table row (a stable sort of the index), `offsets` (T + 1)
// delimits each row's group
// (one wave per (row, head): lane l sums group entries l, l + 64, ... in order, then a fixed
// xor tree -- deterministic, and 64 gathers in flight per row instead of one dependent chain)
__global__ __launch_bounds__(256) void rel_pos_bias_bwd_kernel(const float* __restrict__ dbias,
                                                               const int64_t* __restrict__ perm,
                                                               const int64_t* __restrict__ offsets,
                                                               float* __restrict__ dtable,
                                                               int64_t NN, int heads, int64_t T) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= T * heads) return;
  const int64_t r = i / heads;
  const int h = (int)(i - r * heads);
  const float* db = dbias + (int64_t)h * NN;
  float s = 0.f;
  for (int64_t k = offsets[r] + lane; k < offsets[r + 1]; k += 64) s += db[perm[k]];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) dtable[i] = s;
}

// ------------------------------------------------------------------------------------------
// trilinear (align_corners=False) adjoint along one axis: in (outer, Lout, inner) ->
// out (outer, Lin, inner), out[o][i][n] = sum_p w(p -> i) in[o][p][n] (gather form)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void lin_src(int p, int in, int out, int& i0, int& i1, float& l0,
                                        float& l1) {
  const float scale = (float)in / (float)out;
  float s = __fmul_rn(scale, (float)p + 0.5f) - 0.5f;
  s = s < 0.f ? 0.f : s;
  i0 = min((int)floorf(s), in - 1);
  l1 = fminf(fmaxf(s - (float)i0, 0.f), 1.f);
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l0 = 1.f - l1;
}

// align_corners=True: src = p * (in - 1) / (out - 1) (PyTorch's area_pixel_compute_scale)
__device__ __forceinline__ void lin_src_ac(int p, int in, int out, int& i0, int& i1, float& l0,
                                           float& l1) {
  const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  const float s = scale * (float)p;
  i0 = min((int)s, in - 1);
  l1 = fminf(fmaxf(s - (float)i0, 0.f), 1.f);
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l0 = 1.f - l1;
}

template <bool AC>
__global__ __launch_bounds__(256) void interp_adjoint_kernel(
    const float* __restrict__ in, float* __restrict__ out, int64_t outer, int Lout, int Lin,
    int64_t inner, const float* __restrict__ oscale, int64_t outer_per_scale) {
  const int64_t n = outer * Lin * inner;
  const float r = AC ? (Lin > 1 ? (float)(Lout - 1) / (float)(Lin - 1) : (float)Lout)
                     : (float)Lout / (float)Lin;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = idx % inner;
    int64_t t = idx / inner;
    const int i = (int)(t % Lin);
    const int64_t o = t / Lin;
    int pmin = (int)floorf(((float)i - 0.5f) * r - 0.5f) - 2;
    int pmax = (int)ceilf(((float)i + 1.5f) * r - 0.5f) + 2;
    pmin = pmin < 0 ? 0 : pmin;
    pmax = pmax > Lout - 1 ? Lout - 1 : pmax;
    const float* src = in + o * Lout * inner + e;
    float acc = 0.f;
    for (int p = pmin; p <= pmax; ++p) {
      int i0, i1;
      float l0, l1;
      if (AC) lin_src_ac(p, Lin, Lout, i0, i1, l0, l1);
      else lin_src(p, Lin, Lout, i0, i1, l0, l1);
      float wgt = (i0 == i ? l0 : 0.f) + (i1 == i ? l1 : 0.f);
      if (wgt != 0.f) acc = fmaf(wgt, src[(int64_t)p * inner], acc);
    }
    if (oscale) acc *= oscale[o / outer_per_scale];
    out[idx] = acc;
  }
}

// ------------------------------------------------------------------------------------------
// depthwise 3^3 conv, channel-last, zero padding 1: out = conv(in, w[c][27]) (+ bias);
// flip != 0 uses w[c][26 - k] (the input-gradient of the forward conv)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dwconv_cl_kernel(const float* __restrict__ in,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ bias,
                                                        int flip, float* __restrict__ out,
                                                        int B, int C, int D, int H, int W) {
  const int C4 = C / 4;
  const int64_t n = (int64_t)B * D * H * W * C4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    int64_t t = i / C4;
    const int x = (int)(t % W);
    t /= W;
    const int y = (int)(t % H);
    t /= H;
    const int z = (int)(t % D);
    const int b = (int)(t / D);
    f32x4 acc = bias ? *reinterpret_cast<const f32x4*>(bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < 27; ++k) {
      const int zz = z + k / 9 - 1, yy = y + (k / 3) % 3 - 1, xx = x + k % 3 - 1;
      if (zz < 0 || zz >= D || yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
      const f32x4 v = *reinterpret_cast<const f32x4*>(
          in + ((((int64_t)b * D + zz) * H + yy) * W + xx) * C + c);
      const int kk = flip ? 26 - k : k;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = fmaf(w[(c + e) * 27 + kk], v[e], acc[e]);
    }
    *reinterpret_cast<f32x4*>(out + i * 4) = acc;
  }
}

// dw[c][k] = sum_pos dy[pos][c] * x[pos + off_k][c]; block = (position chunk, 64 channel
// groups of 4); 4 position phases per block; partials (parts, C*27) in [c][k] order
__global__ __launch_bounds__(256) void dwconv_wgrad_kernel(const float* __restrict__ dy,
                                                           const float* __restrict__ x,
                                                           float* __restrict__ part, int B,
                                                           int C, int D, int H, int W,
                                                           int64_t ppb) {
  __shared__ float red[64][4 * 27 + 1];
  const int g = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = (blockIdx.y * 64 + g) * 4;
  const bool cok = c < C;
  const int64_t P = (int64_t)B * D * H * W;
  const int64_t p0 = blockIdx.x * ppb, p1 = min(P, p0 + ppb);
  f32x4 acc[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (cok) {
    for (int64_t p = p0 + ph; p < p1; p += 4) {
      const int xq = (int)(p % W);
      int64_t t = p / W;
      const int yq = (int)(t % H);
      t /= H;
      const int zq = (int)(t % D);
      const int64_t b = t / D;
      const f32x4 g4 = *reinterpret_cast<const f32x4*>(dy + p * C + c);
#pragma unroll
      for (int k = 0; k < 27; ++k) {
        const int zz = zq + k / 9 - 1, yy = yq + (k / 3) % 3 - 1, xx = xq + k % 3 - 1;
        if (zz < 0 || zz >= D || yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
        const f32x4 v = *reinterpret_cast<const f32x4*>(
            x + (((b * D + zz) * H + yy) * W + xx) * C + c);
        acc[k] += g4 * v;
      }
    }
  }
  // phases 1..3 hand their sums to phase 0 one at a time through one LDS slab
  for (int q = 1; q < 4; ++q) {
    if (ph == q) {
#pragma unroll
      for (int k = 0; k < 27; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[g][e * 27 + k] = acc[k][e];
    }
    __syncthreads();
    if (ph == 0) {
#pragma unroll
      for (int k = 0; k < 27; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[k][e] += red[g][e * 27 + k];
    }
    __syncthreads();
  }
  if (ph == 0 && cok) {
    float* dst = part + (int64_t)blockIdx.x * C * 27 + (int64_t)c * 27;
#pragma unroll
    for (int k = 0; k < 27; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[e * 27 + k] = acc[k][e];
  }
}

// ------------------------------------------------------------------------------------------
// PatchMerging gather / scatter (code: nibble s = (d<<2|h<<1|w) offset of slot s)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void merge_gather_kernel(const float* __restrict__ x,
                                                           uint32_t code, float* __restrict__ m,
                                                           int B, int C, int D, int H, int W) {
  const int d = D / 2, h = H / 2, w = W / 2;
  const int64_t n = (int64_t)B * d * h * w * 8 * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    int64_t t = i / C;
    const int s = (int)(t % 8);
    t /= 8;
    const int xo = (int)(t % w);
    t /= w;
    const int yo = (int)(t % h);
    t /= h;
    const int zo = (int)(t % d);
    const int64_t b = t / d;
    const int off = (code >> (4 * s)) & 7;
    const int64_t zz = 2 * zo + (off >> 2), yy = 2 * yo + ((off >> 1) & 1), xx = 2 * xo + (off & 1);
    m[i] = x[(((b * D + zz) * H + yy) * W + xx) * C + c];
  }
}

__global__ __launch_bounds__(256) void merge_scatter_kernel(const float* __restrict__ dm,
                                                            uint32_t code,
                                                            float* __restrict__ dx, int B,
                                                            int C, int D, int H, int W) {
  const int d = D / 2, h = H / 2, w = W / 2;
  const int64_t n = (int64_t)B * D * H * W * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    int64_t t = i / C;
    const int x = (int)(t % W);
    t /= W;
    const int y = (int)(t % H);
    t /= H;
    const int z = (int)(t % D);
    const int64_t b = t / D;
    const int par = ((z & 1) << 2) | ((y & 1) << 1) | (x & 1);
    const int64_t mrow = (((b * d + z / 2) * h + y / 2) * w + x / 2) * 8 * C;
    float acc = 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if ((int)((code >> (4 * s)) & 7) == par) acc += dm[mrow + s * C + c];
    dx[i] = acc;
  }
}

// ------------------------------------------------------------------------------------------
// PatchEmbed patches: x NCDHW (B, Cin, 2D, 2H, 2W) <-> rows (B*D*H*W, Cin*8), column
// ci*8 + kz*4 + ky*2 + kx (the flattened Conv3d weight order).  dir 0: gather, 1: scatter.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void patchify_kernel(float* __restrict__ x,
                                                       float* __restrict__ rows, int dir,
                                                       int B, int Cin, int D, int H, int W) {
  const int K = Cin * 8;
  const int64_t n = (int64_t)B * D * H * W * K;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int col = (int)(i % K);
    int64_t t = i / K;
    const int xo = (int)(t % W);
    t /= W;
    const int yo = (int)(t % H);
    t /= H;
    const int zo = (int)(t % D);
    const int64_t b = t / D;
    const int ci = col / 8, kz = (col >> 2) & 1, ky = (col >> 1) & 1, kx = col & 1;
    const int64_t xi = (((b * Cin + ci) * 2 * D + 2 * zo + kz) * 2 * H + 2 * yo + ky) * 2 * W +
                       2 * xo + kx;
    if (dir == 0)
      rows[i] = x[xi];
    else
      x[xi] = rows[i];
  }
}

// ------------------------------------------------------------------------------------------
// (B, C, S) -> (B, S, C) transpose through a 32 x 33 LDS tile
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void transpose_cs_kernel(const float* __restrict__ in,
                                                           float* __restrict__ out, int C,
                                                           int64_t S) {
  __shared__ float tile[32][33];
  const int64_t b = blockIdx.z;
  const int64_t s0 = (int64_t)blockIdx.x * 32;
  const int c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const float* src = in + b * C * S;
  float* dst = out + b * C * S;
  for (int r = ty; r < 32; r += 8) {
    const int c = c0 + r;
    const int64_t s = s0 + tx;
    tile[r][tx] = (c < C && s < S) ? src[(int64_t)c * S + s] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int64_t s = s0 + r;
    const int c = c0 + tx;
    if (c < C && s < S) dst[s * C + c] = tile[tx][r];
  }
}

#define WF_HIP(call)                                                                \
  do {                                                                              \
    hipError_t e_ = (call);                                                         \
    if (e_ != hipSuccess) return ::wf::fail((int)e_, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

static unsigned grid_for(int64_t n, int64_t cap = 16384) {
  int64_t g = cdiv(n, 256);
  if (g > cap) g = cap;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace wf

using namespace wf;

// ==========================================================================================
// C-ABI
// ==========================================================================================
extern "C" int64_t wf_colsum_parts(int64_t R) { return colsum_parts(R); }

extern "C" int wf_colsum(const float* in, int64_t R, int64_t N, const float* row_scale,
                         int64_t rows_per_scale, float* partials, float* out, void* stream) {
  WF_REQUIRE(R >= 0 && N >= 0, "negative size");
  WF_REQUIRE_PTR(out);
  if (R > 0) {
    WF_REQUIRE_PTR(in);
    WF_REQUIRE_PTR(partials);
  }
  return launch_colsum(in, R, N, row_scale, rows_per_scale, partials, out,
                       (hipStream_t)stream);
}

extern "C" int wf_ln_act_fwd(const float* x, const float* w, const float* b, float eps, int gelu,
                             float* y, int64_t M, int64_t N, void* stream) {
  WF_REQUIRE(M >= 0 && N >= 1 && N <= 1536, "row width must be in [1, 1536]");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(y);
  if (w) WF_REQUIRE_PTR(b);
  if (M == 0) return WF_OK;
  const unsigned g = grid_for(M * 64, 8192);
  hipStream_t s = (hipStream_t)stream;
#define WF_M(J) hipLaunchKernelGGL(ln_act_fwd_kernel<J>, dim3(g), dim3(256), 0, s, x, w, b, eps, gelu, y, M, (int)N);
  WF_LN_DISPATCH(N, WF_M)
#undef WF_M
  return check_launch("wf_ln_act_fwd");
}

extern "C" int wf_ln_act_bwd(const float* x, const float* w, const float* b, float eps, int gelu,
                             const float* dy, const float* dadd, float* dx, float* partials,
                             float* dw, float* db, int64_t M, int64_t N, void* stream) {
  WF_REQUIRE(M >= 0 && N >= 1 && N <= 1536, "row width must be in [1, 1536]");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(dy);
  WF_REQUIRE_PTR(dx);
  if (w) {
    WF_REQUIRE_PTR(b);
    WF_REQUIRE_PTR(partials);
    WF_REQUIRE_PTR(dw);
    WF_REQUIRE_PTR(db);
  }
  hipStream_t s = (hipStream_t)stream;
  const int64_t G = ln_parts(M);
  float* part = w ? partials : nullptr;
  if (M > 0) {
#define WF_M(J) hipLaunchKernelGGL(ln_act_bwd_kernel<J>, dim3((unsigned)G), dim3(256), 0, s, x, w, b, eps, gelu, dy, dadd, dx, part, M, (int)N);
    WF_LN_DISPATCH(N, WF_M)
#undef WF_M
    int rc = check_launch("wf_ln_act_bwd");
    if (rc) return rc;
  }
  if (!w) return WF_OK;
  if (M == 0) {
    WF_HIP(hipMemsetAsync(dw, 0, N * sizeof(float), s));
    WF_HIP(hipMemsetAsync(db, 0, N * sizeof(float), s));
    return check_launch("wf_ln_act_bwd");
  }
  // partials (G, 2N) -> column sums: dw = cols [0, N), db = cols [N, 2N)
  float* tmp = partials + G * 2 * N;  // the caller sizes partials for both (wf_ln_bwd_ws)
  int rc = launch_colsum(partials, G, 2 * N, nullptr, 0, tmp, tmp + colsum_parts(G) * 2 * N, s);
  if (rc) return rc;
  WF_HIP(hipMemcpyAsync(dw, tmp + colsum_parts(G) * 2 * N, N * sizeof(float), hipMemcpyDeviceToDevice,
                 s));
  WF_HIP(hipMemcpyAsync(db, tmp + colsum_parts(G) * 2 * N + N, N * sizeof(float),
                 hipMemcpyDeviceToDevice, s));
  return check_launch("wf_ln_act_bwd(reduce)");
}

extern "C" int64_t wf_ln_bwd_workspace_floats(int64_t M, int64_t N) {
  const int64_t G = ln_parts(M);
  return G * 2 * N + colsum_parts(G) * 2 * N + 2 * N;
}

extern "C" int wf_dwt3d_haar_bwd(const float* const* dband, const int64_t* strides, float* dx,
                                 int64_t B, int64_t C, int64_t D, int64_t H, int64_t W,
                                 void* stream) {
  WF_REQUIRE(B >= 1 && C >= 1 && D % 2 == 0 && H % 2 == 0 && W % 2 == 0 && D >= 2 && H >= 2 &&
                 W >= 2, "even positive sizes required");
  WF_REQUIRE_PTR(dx);
  WF_REQUIRE_PTR(dband);
  WF_REQUIRE_PTR(strides);
  BandPtrs bp;
  for (int k = 0; k < 8; ++k) {
    bp.p[k] = dband[k];
    for (int j = 0; j < 5; ++j) bp.s[k][j] = strides[5 * k + j];
  }
  const int64_t n = B * (D / 2) * (H / 2) * (W / 2) * C;
  hipLaunchKernelGGL(dwt_bwd_cl_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, bp,
                     dx, (int)B, (int)C, (int)(D / 2), (int)(H / 2), (int)(W / 2));
  return check_launch("wf_dwt3d_haar_bwd");
}

extern "C" int wf_haar_analysis_ncdhw(const float* in, int64_t in_bstride, int64_t in_cstride,
                                      float* ll, float* const* det, const int64_t* det_strides,
                                      int64_t B, int64_t C, int64_t d, int64_t h, int64_t w,
                                      void* stream) {
  WF_REQUIRE(B >= 1 && C >= 1 && d >= 1 && h >= 1 && w >= 1, "empty volume");
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(ll);
  WF_REQUIRE_PTR(det);
  WF_REQUIRE_PTR(det_strides);
  DetOut o;
  for (int k = 0; k < 7; ++k) {
    WF_REQUIRE_PTR(det[k]);
    o.p[k] = det[k];
  }
  for (int j = 0; j < 5; ++j) o.s[j] = det_strides[j];
  const int64_t n = B * C * d * h * w;
  hipLaunchKernelGGL(haar_analysis_ncdhw_kernel, dim3(grid_for(n)), dim3(256), 0,
                     (hipStream_t)stream, in, in_bstride, in_cstride, ll, o, (int)B, (int)C,
                     (int)d, (int)h, (int)w);
  return check_launch("wf_haar_analysis_ncdhw");
}

namespace {
// window groups of the attention backward: enough (key block, head, group) workgroups to
// cover the CUs, each group walking ceil(Bw / G) windows
int64_t attn_bwd_groups(int64_t Bw, int64_t N, int64_t heads) {
  const int64_t nkb = cdiv(N, kAB);
  int64_t G = cdiv(1024, nkb * heads);
  G = std::min<int64_t>(std::max<int64_t>(G, 1), Bw);
  return cdiv(Bw, cdiv(Bw, G));  // balance: every group gets the same window count (+-1)
}
inline int64_t align256(int64_t b) { return (b + 255) & ~(int64_t)255; }
}  // namespace

extern "C" int64_t wf_window_attention_bwd_workspace_bytes(int64_t B, int64_t C, int64_t D1,
                                                           int64_t H1, int64_t W1, int64_t ws,
                                                           int64_t heads) {
  if (ws < 1 || heads < 1 || D1 % ws || H1 % ws || W1 % ws) return -1;
  const int64_t N = ws * ws * ws;
  const int64_t Bw = B * (D1 / ws) * (H1 / ws) * (W1 / ws);
  const int64_t rows = B * D1 * H1 * W1;
  const int64_t G = attn_bwd_groups(Bw, N, heads);
  return align256(cdiv(N, kAB) * rows * C * 4) + align256(G * heads * N * N * 4);
}

extern "C" int wf_window_attention_bwd_core(const float* qkv, const float* o, const float* dout,
                                            const float* bias, const float* lse, float* dqkv,
                                            float* dbias, void* workspace, int64_t B, int64_t C,
                                            int64_t D1, int64_t H1, int64_t W1, int64_t ws,
                                            int64_t heads, float scale, void* stream) {
  WF_REQUIRE(ws >= 1 && D1 % ws == 0 && H1 % ws == 0 && W1 % ws == 0,
             "the raster must tile into ws^3 windows");
  WF_REQUIRE(heads >= 1 && C % heads == 0 && C % 4 == 0,
             "dim must be divisible by num_heads and by 4");
  WF_REQUIRE_PTR(qkv);
  WF_REQUIRE_PTR(o);
  WF_REQUIRE_PTR(dout);
  WF_REQUIRE_PTR(bias);
  WF_REQUIRE_PTR(lse);
  WF_REQUIRE_PTR(dqkv);
  WF_REQUIRE_PTR(dbias);
  WF_REQUIRE_PTR(workspace);
  const int64_t N = ws * ws * ws;
  const int64_t Bw = B * (D1 / ws) * (H1 / ws) * (W1 / ws);
  const int64_t rows = B * D1 * H1 * W1;
  const int64_t nkb = cdiv(N, kAB);
  const int64_t G = attn_bwd_groups(Bw, N, heads);
  WF_REQUIRE(G <= 65535 && nkb <= 65535, "too many windows per call");
  const int hd = (int)(C / heads);
  WF_REQUIRE(hd == 16 || hd == 32 || hd == 48 || hd == 64,
             "attention backward: head_dim must be 16, 32, 48 or 64");
  hipStream_t s = (hipStream_t)stream;
  AttnBwdArgs a;
  a.qkv = qkv;
  a.o = o;
  a.dout = dout;
  a.bias = bias;
  a.lse = lse;
  a.dqkv = dqkv;
  a.dq_part = static_cast<float*>(workspace);
  a.db_part = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                       align256(nkb * rows * C * 4));
  a.Bw = Bw;
  a.N = (int)N;
  a.heads = (int)heads;
  a.C = (int)C;
  a.ws = (int)ws;
  a.nD = (int)(D1 / ws);
  a.nH = (int)(H1 / ws);
  a.nW = (int)(W1 / ws);
  a.G = (int)G;
  a.scale = scale;
  a.scale_log2 = scale * 1.4426950408889634f;
  dim3 grid((unsigned)nkb, (unsigned)heads, (unsigned)G);
  switch (hd) {
    case 16: hipLaunchKernelGGL(attn_bwd_kernel<16>, grid, dim3(256), 0, s, a); break;
    case 32: hipLaunchKernelGGL(attn_bwd_kernel<32>, grid, dim3(256), 0, s, a); break;
    case 48: hipLaunchKernelGGL(attn_bwd_kernel<48>, grid, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL(attn_bwd_kernel<64>, grid, dim3(256), 0, s, a); break;
  }
  int rc = check_launch("wf_window_attention_bwd_core");
  if (rc) return rc;
  const int64_t tq = rows * (C / 4);
  hipLaunchKernelGGL(attn_dq_reduce_kernel, dim3((unsigned)std::min<int64_t>(cdiv(tq, 256), 8192)),
                     dim3(256), 0, s, a.dq_part, dqkv, rows, (int)C, (int)nkb, scale, (int)ws,
                     a.nD, a.nH, a.nW);
  rc = check_launch("wf_window_attention_bwd_core (dQ reduce)");
  if (rc) return rc;
  const int64_t nb = heads * N * N;
  hipLaunchKernelGGL(attn_db_reduce_kernel, dim3((unsigned)std::min<int64_t>(cdiv(nb, 256), 8192)),
                     dim3(256), 0, s, a.db_part, dbias, nb, (int)G);
  return check_launch("wf_window_attention_bwd_core (dBias reduce)");
}

extern "C" int wf_rel_pos_bias_bwd(const float* dbias, const int64_t* perm,
                                   const int64_t* offsets, float* dtable, int64_t N, int64_t heads,
                                   int64_t table_rows, void* stream) {
  WF_REQUIRE_PTR(dbias);
  WF_REQUIRE_PTR(perm);
  WF_REQUIRE_PTR(offsets);
  WF_REQUIRE_PTR(dtable);
  WF_REQUIRE(heads >= 1 && table_rows >= 1, "empty table");
  const int64_t n = table_rows * heads;
  hipLaunchKernelGGL(rel_pos_bias_bwd_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0,
                     (hipStream_t)stream, dbias, perm, offsets, dtable, N * N, (int)heads,
                     table_rows);
  return check_launch("wf_rel_pos_bias_bwd");
}

extern "C" int wf_interp_adjoint_axis(const float* in, float* out, int64_t outer, int64_t Lout,
                                      int64_t Lin, int64_t inner, const float* outer_scale,
                                      int64_t outer_per_scale, void* stream) {
  WF_REQUIRE(outer >= 1 && Lout >= 1 && Lin >= 1 && inner >= 1, "empty interpolation axis");
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(out);
  const int64_t n = outer * Lin * inner;
  hipLaunchKernelGGL(interp_adjoint_kernel<false>, dim3(grid_for(n)), dim3(256), 0,
                     (hipStream_t)stream, in, out, outer, (int)Lout, (int)Lin, inner, outer_scale,
                     outer_per_scale > 0 ? outer_per_scale : outer);
  return check_launch("wf_interp_adjoint_axis");
}

extern "C" int wf_interp_adjoint_axis_ac(const float* in, float* out, int64_t outer,
                                         int64_t Lout, int64_t Lin, int64_t inner,
                                         void* stream) {
  WF_REQUIRE(outer >= 1 && Lout >= 1 && Lin >= 1 && inner >= 1, "empty interpolation axis");
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(out);
  const int64_t n = outer * Lin * inner;
  hipLaunchKernelGGL(interp_adjoint_kernel<true>, dim3(grid_for(n)), dim3(256), 0,
                     (hipStream_t)stream, in, out, outer, (int)Lout, (int)Lin, inner, nullptr,
                     outer);
  return check_launch("wf_interp_adjoint_axis_ac");
}

extern "C" int wf_dwconv3d_cl(const float* in, const float* w, const float* bias, int flip,
                              float* out, int64_t B, int64_t C, int64_t D, int64_t H, int64_t W,
                              void* stream) {
  WF_REQUIRE(C % 4 == 0 && C >= 4, "channels must be a multiple of 4");
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(w);
  WF_REQUIRE_PTR(out);
  // 32-channel groups: the z-streaming LDS-tiled kernel of CCF_FFN (ffn.hip), forward or
  // flipped (the input gradient: 1.0x the forward's time instead of the per-output 27-load
  // kernel below, 4.1 ms per 64^3 x 192 launch at B = 4)
  if (C % 32 == 0)
    return launch_dwconv3d(in, w, bias, out, nullptr, (int)B, (int)C, (int)D, (int)H, (int)W,
                           PREC_SPLIT, (hipStream_t)stream, nullptr, nullptr, nullptr, nullptr,
                           flip);
  const int64_t n = B * D * H * W * (C / 4);
  hipLaunchKernelGGL(dwconv_cl_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, in, w,
                     bias, flip, out, (int)B, (int)C, (int)D, (int)H, (int)W);
  return check_launch("wf_dwconv3d_cl");
}

extern "C" int wf_dwconv3d_stats_cl(const float* in, const float* w, const float* bias,
                                    float* out, double* stats_acc, int64_t B, int64_t C,
                                    int64_t D, int64_t H, int64_t W, void* stream) {
  WF_REQUIRE(C % 32 == 0 && C >= 32, "channels must be a multiple of 32");
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(w);
  WF_REQUIRE_PTR(bias);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE_PTR(stats_acc);
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(stats_acc, 0, (size_t)(B * C * 2) * sizeof(double), s) != hipSuccess)
    return check_launch("wf_dwconv3d_stats_cl (memset)");
  return launch_dwconv3d(in, w, bias, out, nullptr, (int)B, (int)C, (int)D, (int)H, (int)W,
                         PREC_SPLIT, s, stats_acc);
}

namespace wf {
// ------------------------------------------------------------------------------------------
// depthwise 3^3 weight gradient, z-streaming: dw[c][k] = sum_p dy[p][c] x[p + off_k][c]
// A workgroup = (32 channels, one 8 x 16 tile of a z segment), 256 threads = 16 columns x 16
// channel pairs (the tiling of dwconv3d_kernel, ffn.hip).  The haloed x plane q (10 x 18
// positions x 32 channels) is staged in LDS once (double buffered, next plane in flight); it
// meets the output gradients of planes q + 1 (kz = 0), q (kz = 1) and q - 1 (kz = 2), which
// ride in registers (three rolling sets of the thread's 8 rows).  Each thread accumulates the
// 27 taps of its channel pair over its positions; the 16 columns are then combined in a fixed
// order (two xor steps inside the wave, the 4 waves through LDS) and each workgroup writes one
// partial (27 x 32 floats); a column-sum kernel adds the partials in order.  Replaces the
// per-position kernel below (27 global 16-B loads per position: 5.2 ms per 64^3 x 192 call).
constexpr int DWG_CH = 32, DWG_TX = 16, DWG_TY = 8, DWG_PY = DWG_TY + 2, DWG_PX = DWG_TX + 2;
constexpr int DWG_NV = DWG_CH / 4;                                 // f32x4 per position
constexpr int DWG_NLD = (DWG_PY * DWG_PX * DWG_NV + 255) / 256;

struct DwgArgs {
  const float* dy;
  const float* x;
  float* part;  // (tiles, C * 27): tile-major, [c][k] inside
  int B, C, D, H, W, ZS;
};

__global__ __launch_bounds__(256) void dwconv_wgrad_z_kernel(DwgArgs a) {
  __shared__ __attribute__((aligned(16))) float pl[2][DWG_PY * DWG_PX * DWG_CH];
  const int C = a.C, D = a.D, H = a.H, W = a.W;
  const int ncc = C / DWG_CH, ntx = (W + DWG_TX - 1) / DWG_TX, nty = (H + DWG_TY - 1) / DWG_TY;
  const int nzs = (D + a.ZS - 1) / a.ZS;
  int t = blockIdx.x;
  const int cc = t % ncc;
  t /= ncc;
  const int tile = t;  // partial index (spatial tile incl. z segment and sample)
  const int xt = t % ntx;
  t /= ntx;
  const int yt = t % nty;
  t /= nty;
  const int zt = t % nzs;
  const int b = t / nzs;
  const int x0 = xt * DWG_TX, y0 = yt * DWG_TY, z0 = zt * a.ZS, z1 = min(z0 + a.ZS, D);
  const int c0 = cc * DWG_CH;
  const int tid = threadIdx.x;
  const int cp = tid % (DWG_CH / 2), xi = tid / (DWG_CH / 2);
  const int xo = x0 + xi;
  const int64_t sb = (int64_t)b * D * H * W;
  const float* xs = a.x + sb * C + c0;
  const float* gs = a.dy + sb * C + c0 + 2 * cp;

  f32x4 stg[DWG_NLD];
  auto fetch = [&](int p) {
    const bool pz = p >= 0 && p < D;
    const int pc = min(max(p, 0), D - 1);
#pragma unroll
    for (int j = 0; j < DWG_NLD; ++j) {
      const int i = min(j * 256 + tid, DWG_PY * DWG_PX * DWG_NV - 1);
      const int pos = i / DWG_NV, v = i - pos * DWG_NV;
      const int yy = y0 - 1 + pos / DWG_PX, xx = x0 - 1 + pos % DWG_PX;
      const bool ok = pz && yy >= 0 && yy < H && xx >= 0 && xx < W;
      const int yc = min(max(yy, 0), H - 1), xc = min(max(xx, 0), W - 1);
      const f32x4 u = *reinterpret_cast<const f32x4*>(
          xs + (((int64_t)pc * H + yc) * W + xc) * C + 4 * v);
      stg[j] = ok ? u : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int j = 0; j < DWG_NLD; ++j) {
      const int i = j * 256 + tid;
      if (i < DWG_PY * DWG_PX * DWG_NV) *reinterpret_cast<f32x4*>(pl[buf] + (size_t)i * 4) = stg[j];
    }
  };
  // the output gradient rows of plane z (zero outside the segment / volume)
  auto gload = [&](int z, f32x2 (&g)[DWG_TY]) {
    const bool zv = z >= z0 && z < z1 && xo < W;
    const int zc = min(max(z, 0), D - 1), xc = min(xo, W - 1);
#pragma unroll
    for (int o = 0; o < DWG_TY; ++o) {
      const int yo = y0 + o;
      const f32x2 u = *reinterpret_cast<const f32x2*>(
          gs + (((int64_t)zc * H + min(yo, H - 1)) * W + xc) * C);
      g[o] = (zv && yo < H) ? u : f32x2{0.f, 0.f};
    }
  };

  f32x2 acc[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) acc[k] = f32x2{0.f, 0.f};
  // plane q meets dy of q + 1 (gC, kz = 0), q (gB, kz = 1), q - 1 (gA, kz = 2)
  f32x2 gA[DWG_TY], gB[DWG_TY], gC[DWG_TY], gN[DWG_TY];
  gload(z0 - 2, gA);  // zeros
  gload(z0 - 1, gB);  // zeros
  gload(z0, gC);
  fetch(z0 - 1);
  commit(0);
  __syncthreads();
  int buf = 0;
  for (int q = z0 - 1; q <= z1; ++q) {
    fetch(q + 1);     // next x plane in flight
    gload(q + 2, gN); // and the dy rows the next plane needs
    const float* P = pl[buf] + xi * DWG_CH + 2 * cp;
#pragma unroll
    for (int r = 0; r < DWG_PY; ++r) {
      const f32x2 v0 = *reinterpret_cast<const f32x2*>(P + (r * DWG_PX + 0) * DWG_CH);
      const f32x2 v1 = *reinterpret_cast<const f32x2*>(P + (r * DWG_PX + 1) * DWG_CH);
      const f32x2 v2 = *reinterpret_cast<const f32x2*>(P + (r * DWG_PX + 2) * DWG_CH);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int o = r - ky;  // output row fed by input row r through tap ky
        if (o < 0 || o >= DWG_TY) continue;
        acc[ky * 3 + 0] += gC[o] * v0;
        acc[ky * 3 + 1] += gC[o] * v1;
        acc[ky * 3 + 2] += gC[o] * v2;
        acc[9 + ky * 3 + 0] += gB[o] * v0;
        acc[9 + ky * 3 + 1] += gB[o] * v1;
        acc[9 + ky * 3 + 2] += gB[o] * v2;
        acc[18 + ky * 3 + 0] += gA[o] * v0;
        acc[18 + ky * 3 + 1] += gA[o] * v1;
        acc[18 + ky * 3 + 2] += gA[o] * v2;
      }
    }
#pragma unroll
    for (int o = 0; o < DWG_TY; ++o) {
      gA[o] = gB[o];
      gB[o] = gC[o];
      gC[o] = gN[o];
    }
    commit(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // the 16 columns of a channel pair: lanes cp, cp + 16, cp + 32, cp + 48 of each wave (two
  // xor steps), then the 4 waves in order through LDS
#pragma unroll
  for (int k = 0; k < 27; ++k) {
    acc[k].x += __shfl_xor(acc[k].x, 16, 64);
    acc[k].y += __shfl_xor(acc[k].y, 16, 64);
    acc[k].x += __shfl_xor(acc[k].x, 32, 64);
    acc[k].y += __shfl_xor(acc[k].y, 32, 64);
  }
  float* red = pl[0];  // [4 waves][27][32 channels]
  const int wv = tid >> 6, lane = tid & 63;
  if (lane < 16) {
#pragma unroll
    for (int k = 0; k < 27; ++k) {
      red[(wv * 27 + k) * DWG_CH + 2 * lane] = acc[k].x;
      red[(wv * 27 + k) * DWG_CH + 2 * lane + 1] = acc[k].y;
    }
  }
  __syncthreads();
  float* dst = a.part + (int64_t)tile * C * 27;
  for (int i = tid; i < 27 * DWG_CH; i += 256) {
    const int k = i / DWG_CH, c = i - k * DWG_CH;
    const float v = (red[(0 * 27 + k) * DWG_CH + c] + red[(1 * 27 + k) * DWG_CH + c]) +
                    (red[(2 * 27 + k) * DWG_CH + c] + red[(3 * 27 + k) * DWG_CH + c]);
    dst[(c0 + c) * 27 + k] = v;
  }
}

// z segment length of the z-streaming weight gradient: ~2048 workgroups
int dwg_zs(int64_t B, int64_t C, int64_t D, int64_t H, int64_t W) {
  const int64_t base = B * (C / DWG_CH) * cdiv(H, DWG_TY) * cdiv(W, DWG_TX);
  int ZS = (int)D;
  while (ZS > 4 && base * cdiv(D, ZS) < 2048) ZS = (ZS + 1) / 2;
  return ZS;
}
int64_t dwg_tiles(int64_t B, int64_t D, int64_t H, int64_t W, int ZS) {
  return B * cdiv(D, ZS) * cdiv(H, DWG_TY) * cdiv(W, DWG_TX);
}
}  // namespace wf

static int64_t wf_dwconv_wgrad_parts(int64_t positions) {
  int64_t p = cdiv(positions, 512);
  return p > 512 ? 512 : (p < 1 ? 1 : p);
}

extern "C" int wf_dwconv3d_wgrad(const float* dy, const float* x, float* partials, float* dw,
                                 int64_t B, int64_t C, int64_t D, int64_t H, int64_t W,
                                 void* stream) {
  WF_REQUIRE(C % 4 == 0 && C >= 4, "channels must be a multiple of 4");
  WF_REQUIRE_PTR(dy);
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(partials);
  WF_REQUIRE_PTR(dw);
  hipStream_t s = (hipStream_t)stream;
  if (C % DWG_CH == 0 && B * D * H * W * C < ((int64_t)1 << 40)) {
    DwgArgs g{dy, x, partials, (int)B, (int)C, (int)D, (int)H, (int)W, dwg_zs(B, C, D, H, W)};
    const int64_t tiles = dwg_tiles(B, D, H, W, g.ZS);
    WF_REQUIRE(tiles * (C / DWG_CH) < ((int64_t)1 << 31), "too many tiles");
    hipLaunchKernelGGL(dwconv_wgrad_z_kernel, dim3((unsigned)(tiles * (C / DWG_CH))), dim3(256),
                       0, s, g);
    int rc = check_launch("wf_dwconv3d_wgrad");
    if (rc) return rc;
    float* tmp = partials + tiles * C * 27;
    return launch_colsum(partials, tiles, C * 27, nullptr, 0, tmp, dw, s);
  }
  const int64_t P = B * D * H * W;
  const int64_t parts = wf_dwconv_wgrad_parts(P);
  const int64_t ppb = cdiv(P, parts);
  hipLaunchKernelGGL(dwconv_wgrad_kernel, dim3((unsigned)parts, (unsigned)cdiv(C / 4, 64)),
                     dim3(256), 0, s, dy, x, partials, (int)B, (int)C, (int)D, (int)H, (int)W,
                     ppb);
  int rc = check_launch("wf_dwconv3d_wgrad");
  if (rc) return rc;
  float* tmp = partials + parts * C * 27;  // caller sizes partials (wf_dwconv_wgrad_ws_floats)
  return launch_colsum(partials, parts, C * 27, nullptr, 0, tmp, dw, s);
}

extern "C" int64_t wf_dwconv_wgrad_ws_floats(int64_t B, int64_t C, int64_t D, int64_t H,
                                             int64_t W) {
  int64_t parts = wf_dwconv_wgrad_parts(B * D * H * W);
  if (C % DWG_CH == 0) parts = std::max(parts, dwg_tiles(B, D, H, W, dwg_zs(B, C, D, H, W)));
  return parts * C * 27 + colsum_parts(parts) * C * 27;
}

static uint32_t merge_code(int v2) { return v2 ? 0x76543210u : 0x71251240u; }

extern "C" int wf_patch_merging_gather(const float* x, int v2, float* merged, int64_t B,
                                       int64_t C, int64_t D, int64_t H, int64_t W,
                                       void* stream) {
  WF_REQUIRE(D % 2 == 0 && H % 2 == 0 && W % 2 == 0, "even sizes required");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(merged);
  const int64_t n = B * D * H * W * C;
  hipLaunchKernelGGL(merge_gather_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x,
                     merge_code(v2), merged, (int)B, (int)C, (int)D, (int)H, (int)W);
  return check_launch("wf_patch_merging_gather");
}

extern "C" int wf_patch_merging_scatter(const float* dmerged, int v2, float* dx, int64_t B,
                                        int64_t C, int64_t D, int64_t H, int64_t W,
                                        void* stream) {
  WF_REQUIRE(D % 2 == 0 && H % 2 == 0 && W % 2 == 0, "even sizes required");
  WF_REQUIRE_PTR(dmerged);
  WF_REQUIRE_PTR(dx);
  const int64_t n = B * D * H * W * C;
  hipLaunchKernelGGL(merge_scatter_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                     dmerged, merge_code(v2), dx, (int)B, (int)C, (int)D, (int)H, (int)W);
  return check_launch("wf_patch_merging_scatter");
}

extern "C" int wf_patchify(float* x, float* rows, int dir, int64_t B, int64_t Cin, int64_t D,
                           int64_t H, int64_t W, void* stream) {
  WF_REQUIRE(dir == 0 || dir == 1, "dir must be 0 (gather) or 1 (scatter)");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(rows);
  const int64_t n = B * D * H * W * Cin * 8;
  hipLaunchKernelGGL(patchify_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, rows,
                     dir, (int)B, (int)Cin, (int)D, (int)H, (int)W);
  return check_launch("wf_patchify");
}

extern "C" int wf_transpose_cs(const float* in, float* out, int64_t B, int64_t C, int64_t S,
                               void* stream) {
  WF_REQUIRE(B >= 1 && B <= 65535 && C >= 1, "bad batch / channels");
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(out);
  dim3 grid((unsigned)cdiv(S, 32), (unsigned)cdiv(C, 32), (unsigned)B);
  hipLaunchKernelGGL(transpose_cs_kernel, grid, dim3(256), 0, (hipStream_t)stream, in, out,
                     (int)C, S);
  return check_launch("wf_transpose_cs");
}
