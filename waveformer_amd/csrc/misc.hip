// misc.hip -- PatchEmbed (a10), the multi-scale fuse (a6) and the stage output projection
// (a10, quirk Q5).  All three are HBM-streaming row kernels over channel-last data.
#include <math.h>

#include <algorithm>

#include "kernels.hpp"
#include "rowgroup.hpp"

namespace wf {

// ---------------------------------------------------------------------------------------
// PatchEmbed, one output position per lane, weights as wave-uniform (scalar-cache) operands:
// the Conv3d(k = 2, s = 2) of the encoder stem (Cin 4 or 1 -> Cout 48; patchembedding.py:
// 188-214) is a (32 or 8) x 48 product per position.  A lane loads its 2x2x2 x Cin inputs
// straight from the NCDHW volume (float2 per (ci, dz, dy) row pair: the wave's 64 consecutive
// x positions read 512 contiguous bytes per load), keeps them in VGPRs, and runs the 48 output
// channels as 48 independent FMA chains whose weights w[c][k] are uniform across the wave --
// the compiler fetches them with s_load into SGPR operands -- in exact fp32 (the reference's
// arithmetic; no MFMA rounding).  HBM-streaming: the input once, the channel-last output once.
// (The row-staged kernels below ran their FMAs on packed pairs; with packed-FP32 instructions
// off (Makefile) their VALU work doubled: 182 -> 377 us per B = 8 launch.)
// ---------------------------------------------------------------------------------------
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void patch_embed_lane_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ out, int D, int H, int W, int64_t total) {
  constexpr int K = CIN * 8;
  constexpr int RS = COUT + 4;  // LDS row stride (floats): 8-lane store groups conflict-free
  __shared__ __attribute__((aligned(16))) float tile[4][64 * RS];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t p0 = (int64_t)blockIdx.x * 256 + wv * 64;     // first position of this wave
  // (b, z, y, x) raster position, decoded in 32 bits (the host keeps total below 2^31)
  const uint32_t p = (uint32_t)min(p0 + lane, total - 1);
  const int xo = (int)(p % (uint32_t)W);
  uint32_t t = p / (uint32_t)W;
  const int yo = (int)(t % (uint32_t)H);
  t /= (uint32_t)H;
  const int zo = (int)(t % (uint32_t)D);
  const int64_t b = t / (uint32_t)D;
  const int W2 = 2 * W, H2 = 2 * H, D2 = 2 * D;
  float v[K];
#pragma unroll
  for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        const float2 u = *reinterpret_cast<const float2*>(
            x + (((b * CIN + ci) * D2 + 2 * zo + dz) * H2 + 2 * yo + dy) * W2 + 2 * xo);
        v[ci * 8 + dz * 4 + dy * 2] = u.x;
        v[ci * 8 + dz * 4 + dy * 2 + 1] = u.y;
      }
  float* row = &tile[wv][lane * RS];
  // 4 channels per iteration, K split in halves of at most 16 weights per channel: 64 weight
  // SGPRs in flight (the whole 48 x 32 set would spill the scalar file)
  constexpr int KH = K > 16 ? 16 : K;
#pragma unroll 1
  for (int c4 = 0; c4 < COUT / 4; ++c4) {
    float a[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) a[e] = bias ? bias[4 * c4 + e] : 0.f;
#pragma unroll 1
    for (int k0 = 0; k0 < K; k0 += KH) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float* wc = w + (4 * c4 + e) * K + k0;
#pragma unroll
        for (int k = 0; k < KH; ++k) a[e] = fmaf(v[k0 + k], wc[k], a[e]);
      }
    }
    *reinterpret_cast<f32x4*>(row + 4 * c4) = f32x4{a[0], a[1], a[2], a[3]};
  }
  // the wave's 64 positions x COUT channels are one contiguous run of the channel-last output:
  // write it back with every store instruction covering 1 KB (the per-lane rows would leave
  // each instruction 64 scattered 16-B pieces)
  const int nval = (int)min<int64_t>(64, total - p0) * COUT / 4;  // f32x4 of this wave
  float* o = out + p0 * COUT;
#pragma unroll
  for (int j = 0; j < COUT / 4; ++j) {
    const int e = j * 64 + lane;  // f32x4 index in the run
    if (e < nval) {
      const int pos = e / (COUT / 4), c = (e - pos * (COUT / 4)) * 4;
      *reinterpret_cast<f32x4*>(o + 4 * (int64_t)e) =
          *reinterpret_cast<const f32x4*>(&tile[wv][pos * RS + c]);
    }
  }
}

// ---------------------------------------------------------------------------------------
// PatchEmbed + the first Block's norm1 + Haar LL (round 5; inference, when the stage's first
// Block drops its detail bands): the lane kernel above with a workgroup = the 2 x 2 output rows
// (z + dz, y + dy) of one (z, y) pair, wave 2 dz + dy, lane = x (W <= 64, even).  Each lane
// keeps its position's COUT outputs in registers, so norm1's two-pass moments cost no
// exchange; after one barrier the LL of every 2 x 2 x 2 cube is formed from the LDS rows in the
// Haar butterfly order of dwt3d_haar_fwd_kernel (x, then y, then z).  The stage-1 activation is
// written as before; the LL (B, D/2, H/2, W/2, COUT) replaces that Block's LL-only DWT launch,
// which re-read the whole 402 MB activation (B = 8).
// ---------------------------------------------------------------------------------------
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void patch_embed_ll_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ out, const float* __restrict__ ln_w, const float* __restrict__ ln_b,
    float ln_eps, float* __restrict__ ll, int D, int H, int W) {
  constexpr int K = CIN * 8;
  constexpr int RS = COUT + 4;
  constexpr int C4 = COUT / 4;
  __shared__ __attribute__((aligned(16))) float tile[4][64 * RS];
  __shared__ float2 mst[4][64];  // {mean, rstd} of each position
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int hp = H >> 1, dp = D >> 1;
  int64_t t = blockIdx.x;
  const int yp = (int)(t % hp);
  t /= hp;
  const int zp = (int)(t % dp);
  const int64_t b = t / dp;
  const int zo = 2 * zp + (wv >> 1), yo = 2 * yp + (wv & 1);
  const int xo = min(lane, W - 1);
  const int W2 = 2 * W, H2 = 2 * H, D2 = 2 * D;
  float v[K];
#pragma unroll
  for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        const float2 u = *reinterpret_cast<const float2*>(
            x + (((b * CIN + ci) * D2 + 2 * zo + dz) * H2 + 2 * yo + dy) * W2 + 2 * xo);
        v[ci * 8 + dz * 4 + dy * 2] = u.x;
        v[ci * 8 + dz * 4 + dy * 2 + 1] = u.y;
      }
  float* row = &tile[wv][lane * RS];
  constexpr int KH = K > 16 ? 16 : K;
  float o[COUT];
#pragma unroll
  for (int c4 = 0; c4 < C4; ++c4) {
    float a[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) a[e] = bias ? bias[4 * c4 + e] : 0.f;
#pragma unroll
    for (int k0 = 0; k0 < K; k0 += KH) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float* wc = w + (4 * c4 + e) * K + k0;
#pragma unroll
        for (int k = 0; k < KH; ++k) a[e] = fmaf(v[k0 + k], wc[k], a[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) o[4 * c4 + e] = a[e];
    *reinterpret_cast<f32x4*>(row + 4 * c4) = f32x4{a[0], a[1], a[2], a[3]};
  }
  // norm1's moments of this position (two-pass, as row_stats)
  {
    float sm = 0.f;
#pragma unroll
    for (int c4 = 0; c4 < C4; ++c4)
      sm += (o[4 * c4] + o[4 * c4 + 1]) + (o[4 * c4 + 2] + o[4 * c4 + 3]);
    const float mean = sm / (float)COUT;
    float q = 0.f;
#pragma unroll
    for (int c4 = 0; c4 < C4; ++c4) {
      const float d0 = o[4 * c4] - mean, d1 = o[4 * c4 + 1] - mean, d2 = o[4 * c4 + 2] - mean,
                  d3 = o[4 * c4 + 3] - mean;
      q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
    }
    mst[wv][lane] = float2{mean, rsqrtf(q / (float)COUT + ln_eps)};
  }
  // the activation row (W positions x COUT, contiguous channel-last) with 1 KB stores
  {
    const int64_t p0 = ((b * D + zo) * H + yo) * W;
    float* dst = out + p0 * COUT;
    const int nval = W * C4;
#pragma unroll
    for (int j = 0; j < C4; ++j) {
      const int e = j * 64 + lane;
      if (e < nval) {
        const int pos = e / C4, c = (e - pos * C4) * 4;
        *reinterpret_cast<f32x4*>(dst + 4 * (int64_t)e) =
            *reinterpret_cast<const f32x4*>(&tile[wv][pos * RS + c]);
      }
    }
  }
  __syncthreads();
  // LL of the W/2 cubes x C4 channel quads: n = 4 dz + 2 dy + dx, butterflies x, y, z
  const int wp = W >> 1;
  const int64_t lbase = ((b * dp + zp) * hp + yp) * (int64_t)wp;
  for (int it = threadIdx.x; it < wp * C4; it += 256) {
    const int lx = it / C4, q4 = it - lx * C4;
    const f32x4 gw = *reinterpret_cast<const f32x4*>(ln_w + 4 * q4);
    const f32x4 gb = *reinterpret_cast<const f32x4*>(ln_b + 4 * q4);
    f32x4 c[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int wn = ((n >> 2) << 1) | ((n >> 1) & 1), ln = 2 * lx + (n & 1);
      const float2 ms = mst[wn][ln];
      const f32x4 val = *reinterpret_cast<const f32x4*>(&tile[wn][ln * RS + 4 * q4]);
      c[n] = (val - ms.x) * ms.y * gw + gb;
    }
    const f32x4 s01 = c[0] + c[1], s23 = c[2] + c[3], s45 = c[4] + c[5], s67 = c[6] + c[7];
    const f32x4 r = ((s01 + s23) + (s45 + s67)) * 0.35355339059327373f;
    *reinterpret_cast<f32x4*>(ll + (lbase + lx) * COUT + 4 * q4) = r;
  }
}

// The same kernel with the 4 -> 48 convolution on the matrix cores (Cin = 4: K = 32, one
// v_mfma_f32_16x16x32_bf16 K step): lane (l15, g4) of position tile pt holds input channel
// ci = g4's 2 x 2 x 2 patch of output position x = 16 pt + l15 (four float2 loads, the same bytes
// per thread as above), split to bf16 hi / lo (bf16x3: hi*hi + hi*lo + lo*hi, fp32-faithful
// products, as every GEMM of the path); the weight fragments (output channel 16 rt + l15, k
// octet g4) are split once per thread.  The FMA form ran 1536 fp32 FMAs per position -- ~80 us
// of the 191 us launch at B = 8 in VALU issue alone (profiles/r6/r6pe_*).  The products land
// as 4 consecutive channels of one position per lane, are written (+ bias) into the same LDS row
// tile, and each lane then reads its own position's row back for norm1's moments; stores, LN
// and LL are the FMA kernel's.
__global__ __launch_bounds__(256) void patch_embed_ll_mfma_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ out, const float* __restrict__ ln_w, const float* __restrict__ ln_b,
    float ln_eps, float* __restrict__ ll, int D, int H, int W) {
  constexpr int CIN = 4, COUT = 48, K = 32;
  constexpr int RS = COUT + 4;
  constexpr int C4 = COUT / 4;
  constexpr int RT = COUT / 16;  // output-channel tiles
  __shared__ __attribute__((aligned(16))) float tile[4][64 * RS];
  __shared__ float2 mst[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l15 = lane & 15, g4 = lane >> 4;
  const int hp = H >> 1, dp = D >> 1;
  int64_t t = blockIdx.x;
  const int yp = (int)(t % hp);
  t /= hp;
  const int zp = (int)(t % dp);
  const int64_t b = t / dp;
  const int zo = 2 * zp + (wv >> 1), yo = 2 * yp + (wv & 1);
  const int W2 = 2 * W, H2 = 2 * H, D2 = 2 * D;
  // patches first (the loads in flight while the weights are split)
  float v[4][8];
  const float* xb = x + ((b * CIN + g4) * D2 + 2 * zo) * (int64_t)H2 * W2 + (int64_t)(2 * yo) * W2;
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    const int xo = min(16 * pt + l15, W - 1);
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        const float2 u = *reinterpret_cast<const float2*>(xb + ((int64_t)dz * H2 + dy) * W2 + 2 * xo);
        v[pt][dz * 4 + dy * 2] = u.x;
        v[pt][dz * 4 + dy * 2 + 1] = u.y;
      }
  }
  bf16x8 wh[RT], wl[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(w + (16 * rt + l15) * K + 8 * g4);
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(w + (16 * rt + l15) * K + 8 * g4 + 4);
    const float wf[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    split8<PREC_SPLIT>(wf, wh[rt], wl[rt]);
  }
  f32x4 bq[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
    bq[rt] = bias ? *reinterpret_cast<const f32x4*>(bias + 16 * rt + 4 * g4) : f32x4{0.f, 0.f, 0.f, 0.f};
  float* tw = tile[wv];
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    bf16x8 ph, pl;
    split8<PREC_SPLIT>(v[pt], ph, pl);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      acc = mma32<PREC_SPLIT>(wh[rt], pl, acc);
      acc = mma32<PREC_SPLIT>(wl[rt], ph, acc);
      acc = mma32<PREC_SPLIT>(wh[rt], ph, acc);
      *reinterpret_cast<f32x4*>(tw + (16 * pt + l15) * RS + 16 * rt + 4 * g4) = acc + bq[rt];
    }
  }
  __syncthreads();  // the wave's row tile complete (other lanes' products)
  // norm1's moments of this lane's position (two-pass, as row_stats)
  {
    const float* row = tw + lane * RS;
    f32x4 o[C4];
#pragma unroll
    for (int c4 = 0; c4 < C4; ++c4) o[c4] = *reinterpret_cast<const f32x4*>(row + 4 * c4);
    float sm = 0.f;
#pragma unroll
    for (int c4 = 0; c4 < C4; ++c4) sm += (o[c4].x + o[c4].y) + (o[c4].z + o[c4].w);
    const float mean = sm / (float)COUT;
    float q = 0.f;
#pragma unroll
    for (int c4 = 0; c4 < C4; ++c4) {
      const f32x4 d = o[c4] - mean;
      q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
    mst[wv][lane] = float2{mean, rsqrtf(q / (float)COUT + ln_eps)};
  }
  // the activation row (W positions x COUT, contiguous channel-last) with 1 KB stores
  {
    const int64_t p0 = ((b * D + zo) * H + yo) * W;
    float* dst = out + p0 * COUT;
    const int nval = W * C4;
#pragma unroll
    for (int j = 0; j < C4; ++j) {
      const int e = j * 64 + lane;
      if (e < nval) {
        const int pos = e / C4, c = (e - pos * C4) * 4;
        *reinterpret_cast<f32x4*>(dst + 4 * (int64_t)e) = *reinterpret_cast<const f32x4*>(&tw[pos * RS + c]);
      }
    }
  }
  __syncthreads();
  const int wp = W >> 1;
  const int64_t lbase = ((b * dp + zp) * hp + yp) * (int64_t)wp;
  for (int it = threadIdx.x; it < wp * C4; it += 256) {
    const int lx = it / C4, q4 = it - lx * C4;
    const f32x4 gw = *reinterpret_cast<const f32x4*>(ln_w + 4 * q4);
    const f32x4 gb = *reinterpret_cast<const f32x4*>(ln_b + 4 * q4);
    f32x4 c[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int wn = ((n >> 2) << 1) | ((n >> 1) & 1), ln = 2 * lx + (n & 1);
      const float2 ms = mst[wn][ln];
      const f32x4 val = *reinterpret_cast<const f32x4*>(&tile[wn][ln * RS + 4 * q4]);
      c[n] = (val - ms.x) * ms.y * gw + gb;
    }
    const f32x4 s01 = c[0] + c[1], s23 = c[2] + c[3], s45 = c[4] + c[5], s67 = c[6] + c[7];
    const f32x4 r = ((s01 + s23) + (s45 + s67)) * 0.35355339059327373f;
    *reinterpret_cast<f32x4*>(ll + (lbase + lx) * COUT + 4 * q4) = r;
  }
}

// v2: no LDS row tile.  norm1's moments of a position are reduced over the four lanes that hold
// its 48 channels (xor 16 / 32), the activation is stored straight from the MFMA layout (per
// store instruction 16 positions x 64 B; the three channel tiles complete each 192-B row), and
// only the x-pair sums of the normalised values cross waves, through 24 KB of LDS (was 55 KB:
// two workgroups per CU, now the waves' registers bound it).  The LL sums in the butterfly
// order of the kernel above: ((s01 + s23) + (s45 + s67)) with s = the x pairs of the four rows.
__global__ __launch_bounds__(256) void patch_embed_ll_mfma2_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ out, const float* __restrict__ ln_w, const float* __restrict__ ln_b,
    float ln_eps, float* __restrict__ ll, int D, int H, int W) {
  constexpr int CIN = 4, COUT = 48, K = 32, RT = COUT / 16;
  __shared__ __attribute__((aligned(16))) float pairs[4][32 * COUT];  // [row][x pair][channel]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l15 = lane & 15, g4 = lane >> 4;
  const int hp = H >> 1, dp = D >> 1;
  int64_t t = blockIdx.x;
  const int yp = (int)(t % hp);
  t /= hp;
  const int zp = (int)(t % dp);
  const int64_t b = t / dp;
  const int zo = 2 * zp + (wv >> 1), yo = 2 * yp + (wv & 1);
  const int W2 = 2 * W, H2 = 2 * H, D2 = 2 * D;
  float v[4][8];
  const float* xb = x + ((b * CIN + g4) * D2 + 2 * zo) * (int64_t)H2 * W2 + (int64_t)(2 * yo) * W2;
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    const int xo = min(16 * pt + l15, W - 1);
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        const float2 u = *reinterpret_cast<const float2*>(xb + ((int64_t)dz * H2 + dy) * W2 + 2 * xo);
        v[pt][dz * 4 + dy * 2] = u.x;
        v[pt][dz * 4 + dy * 2 + 1] = u.y;
      }
  }
  bf16x8 wh[RT], wl[RT];
  f32x4 bq[RT], gw[RT], gb[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(w + (16 * rt + l15) * K + 8 * g4);
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(w + (16 * rt + l15) * K + 8 * g4 + 4);
    const float wf[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    split8<PREC_SPLIT>(wf, wh[rt], wl[rt]);
    const int c = 16 * rt + 4 * g4;
    bq[rt] = bias ? *reinterpret_cast<const f32x4*>(bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    gw[rt] = *reinterpret_cast<const f32x4*>(ln_w + c);
    gb[rt] = *reinterpret_cast<const f32x4*>(ln_b + c);
  }
  const int64_t p0 = ((b * D + zo) * H + yo) * W;
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    bf16x8 ph, pl;
    split8<PREC_SPLIT>(v[pt], ph, pl);
    f32x4 acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
      a = mma32<PREC_SPLIT>(wh[rt], pl, a);
      a = mma32<PREC_SPLIT>(wl[rt], ph, a);
      a = mma32<PREC_SPLIT>(wh[rt], ph, a);
      acc[rt] = a + bq[rt];
    }
    const int xo = 16 * pt + l15;
    if (xo < W) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        *reinterpret_cast<f32x4*>(out + (p0 + xo) * COUT + 16 * rt + 4 * g4) = acc[rt];
    }
    // moments over the position's 48 channels: 12 in this lane, the rest in lanes +-16, +-32
    float sm = 0.f;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) sm += (acc[rt].x + acc[rt].y) + (acc[rt].z + acc[rt].w);
    sm += __shfl_xor(sm, 16, 64);
    sm += __shfl_xor(sm, 32, 64);
    const float mean = sm * (1.f / COUT);
    float q = 0.f;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const f32x4 d = acc[rt] - mean;
      q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float rstd = rsqrtf(q * (1.f / COUT) + ln_eps);
    // normalised, then the x pair (lanes l15, l15 ^ 1): s = c[2 lx] + c[2 lx + 1]
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const f32x4 n = (acc[rt] - mean) * rstd * gw[rt] + gb[rt];
      f32x4 o;
      o.x = __shfl_xor(n.x, 1, 64);
      o.y = __shfl_xor(n.y, 1, 64);
      o.z = __shfl_xor(n.z, 1, 64);
      o.w = __shfl_xor(n.w, 1, 64);
      if (!(l15 & 1)) {
        const int lx = 8 * pt + (l15 >> 1);
        *reinterpret_cast<f32x4*>(&pairs[wv][lx * COUT + 16 * rt + 4 * g4]) = n + o;
      }
    }
  }
  __syncthreads();
  const int wp = W >> 1;
  constexpr int C4 = COUT / 4;
  const int64_t lbase = ((b * dp + zp) * hp + yp) * (int64_t)wp;
  for (int it = threadIdx.x; it < wp * C4; it += 256) {
    const int lx = it / C4, q4 = it - lx * C4;
    const int o = lx * COUT + 4 * q4;
    const f32x4 s01 = *reinterpret_cast<const f32x4*>(&pairs[0][o]);
    const f32x4 s23 = *reinterpret_cast<const f32x4*>(&pairs[1][o]);
    const f32x4 s45 = *reinterpret_cast<const f32x4*>(&pairs[2][o]);
    const f32x4 s67 = *reinterpret_cast<const f32x4*>(&pairs[3][o]);
    *reinterpret_cast<f32x4*>(ll + (lbase + lx) * COUT + 4 * q4) =
        ((s01 + s23) + (s45 + s67)) * 0.35355339059327373f;
  }
}

// ---------------------------------------------------------------------------------------
// PatchEmbed, streaming variant (Cin = 4, Cout % 4 == 0, W % 2 == 0: the encoder's 4 -> 48
// stem): a persistent workgroup walks groups of R output rows; the next group's 2x2 input
// rows are loaded into registers (8 float4 per thread at R = 4) while the current group is
// computed out of LDS, then written to the other LDS buffer -- the input stream never waits
// on a barrier-separated load phase (the one-shot kernel above: 282 us at B = 8, 2.4 TB/s).
// ---------------------------------------------------------------------------------------
// XI = ceil(W / XG) output positions per thread and row, unrolled: with the outputs leaving
// through range-checked buffer stores (out-of-range x / idle lanes get an offset past the
// descriptor), every lane issues the same R * XI stores per group, so the wait for the next
// group's fetch can leave them in flight (vmcnt(R * XI)) instead of draining every store
// (vmcnt(0)) as the exec-masked store loop forced.  The output must stay below 2^31 bytes.
template <int R, int XI>
__global__ __launch_bounds__(256) void patch_embed_stream_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ out, int Cout, int D, int H, int W, int64_t ngroups) {
  constexpr int CIN = 4, NK = CIN * 8;
  extern __shared__ __attribute__((aligned(16))) float slab[];  // [2][R][Cin][dz][dy][2W]
  const int W2 = 2 * W, H2 = 2 * H, D2 = 2 * D;
  const int rowf = CIN * 4 * W2;            // floats per output row
  const int per = rowf >> 2;                // float4 per output row
  const int gper = R * per;                 // float4 per group
  const int NLD = (gper + 255) / 256;       // <= 8 at W = 64, R = 4 (host-checked)
  const int nyb = H / R;                    // H % R == 0 (host-checked)
  const int tid = threadIdx.x;
  float* buf0 = slab;
  float* buf1 = slab + R * rowf;

  // thread = (4-channel group, x group): weights as channel pairs, pair FMAs (as above)
  const int C4 = Cout >> 2;
  const int XG = blockDim.x / C4;
  const int cq = tid % C4, xg = tid / C4;
  const bool act = xg < XG;
  const int c0 = 4 * (act ? cq : 0);
  f32x2 wa[NK], wb[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    wa[k] = f32x2{w[(int64_t)(c0 + 0) * NK + k], w[(int64_t)(c0 + 1) * NK + k]};
    wb[k] = f32x2{w[(int64_t)(c0 + 2) * NK + k], w[(int64_t)(c0 + 3) * NK + k]};
  }
  const f32x2 ba = bias ? f32x2{bias[c0], bias[c0 + 1]} : f32x2{0.f, 0.f};
  const f32x2 bb = bias ? f32x2{bias[c0 + 2], bias[c0 + 3]} : f32x2{0.f, 0.f};

  f32x4 stg[8];
  auto fetch = [&](int64_t grp) {
    const int y0 = (int)(grp % nyb) * R;
    const int64_t r = grp / nyb;
    const int z = (int)(r % D), b = (int)(r / D);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = min(j * 256 + tid, gper - 1);
      const int rr = i / per, jj = i - rr * per;
      const int x4 = jj % (W2 >> 2), t = jj / (W2 >> 2);
      const int dy = t & 1, dz = (t >> 1) & 1, ci = t >> 2;
      if (j < NLD)
        stg[j] = reinterpret_cast<const f32x4*>(
            x + ((((int64_t)b * CIN + ci) * D2 + 2 * z + dz) * H2 + 2 * (y0 + rr) + dy) * W2)[x4];
    }
  };
  auto commit = [&](float* dst) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = j * 256 + tid;
      if (j < NLD && i < gper) reinterpret_cast<f32x4*>(dst)[i] = stg[j];
    }
  };
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
      out, 0, (int)((int64_t)ngroups * R * W * Cout * 4), 0x00020000);
  auto compute = [&](const float* src, int64_t grp) {
    const int y0 = (int)(grp % nyb) * R;
    const int r = (int)(grp / nyb);
    const int z = r % D, b = r / D;
#pragma unroll 1
    for (int rr = 0; rr < R; ++rr) {
      const float* sl = src + rr * rowf;
      const int orow = ((b * D + z) * H + y0 + rr) * W;
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int xo = xg + i * XG;
        const bool ok = act && xo < W;
        const int xc = ok ? xo : 0;
        f32x2 a0 = ba, a1 = bb;
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float2 v = *reinterpret_cast<const float2*>(sl + (ci * 4 + q) * W2 + 2 * xc);
            const int k = ci * 8 + 2 * q;
            a0 = wa[k] * v.x + a0;
            a1 = wb[k] * v.x + a1;
            a0 = wa[k + 1] * v.y + a0;
            a1 = wb[k + 1] * v.y + a1;
          }
        const int off = ok ? ((orow + xo) * Cout + c0) * 4 : 0x7fffffff;
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4, f32x4{a0.x, a0.y, a1.x, a1.y}), orsrc, off, 0, 0);
      }
    }
  };

  int64_t g = blockIdx.x;
  if (g >= ngroups) return;
  fetch(g);
  commit(buf0);
  __syncthreads();
  int cur = 0;
  for (; g < ngroups; g += gridDim.x) {
    const int64_t gn = g + gridDim.x;
    if (gn < ngroups) fetch(gn);        // next group's input in flight during this compute
    compute(cur ? buf1 : buf0, g);
    if (gn < ngroups) commit(cur ? buf0 : buf1);
    __syncthreads();                    // next buffer written, current buffer free
    cur ^= 1;
  }
}

// ---------------------------------------------------------------------------------------
// PatchEmbed: Conv3d(Cin, Cout, k=2, s=2) on NCDHW input -> channel-last output.
// monai/networks/blocks/patchembedding.py:214 via network_models/waveformer.py:281,286.
// Workgroup = R output rows (b, z, y0 .. y0 + R - 1): the 2x2 input rows of every input
// channel are staged in LDS (coalesced along x); outputs are written channel-last.
// ---------------------------------------------------------------------------------------
// Thread = (output channel co, x group xg): the Cin*8 weights of co sit in registers and the
// thread walks x = xg, xg + XG, ...; the slab reads are wave-wide broadcasts (a wave covers at
// most two x positions) and the stores are contiguous channel-last rows.
template <int CIN>
__global__ __launch_bounds__(256) void patch_embed_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ out, int Cin_rt,
                                                          int Cout, int D, int H, int W, int R) {
  extern __shared__ __attribute__((aligned(16))) float slab[];  // [R][Cin][dz][dy][2W]
  const int Cin = CIN > 0 ? CIN : Cin_rt;
  const int W2 = 2 * W, H2 = 2 * H, D2 = 2 * D;
  const int nyb = (H + R - 1) / R;
  int r = blockIdx.x;
  const int y0 = (r % nyb) * R;
  r /= nyb;
  const int z = r % D;
  const int b = r / D;
  const int nr = min(R, H - y0);  // output rows of this workgroup
  const int tid = threadIdx.x;
  const int rowf = Cin * 4 * W2;   // slab floats per output row
  // stage the 2x2 input rows of every input channel for the nr output rows (float4 when the
  // row allows it): R rows per workgroup keep R times the bytes in flight per load phase
  if ((W2 & 3) == 0) {
    const int per = rowf >> 2;
    for (int i = tid; i < nr * per; i += blockDim.x) {
      const int rr = i / per, j = i - rr * per;
      const int x4 = j % (W2 >> 2);
      const int t = j / (W2 >> 2);
      const int dy = t & 1, dz = (t >> 1) & 1, ci = t >> 2;
      reinterpret_cast<f32x4*>(slab)[i] = reinterpret_cast<const f32x4*>(
          x + ((((int64_t)b * Cin + ci) * D2 + 2 * z + dz) * H2 + 2 * (y0 + rr) + dy) * W2)[x4];
    }
  } else {
    for (int i = tid; i < nr * rowf; i += blockDim.x) {
      const int rr = i / rowf, j = i - rr * rowf;
      const int xx = j % W2;
      const int t = j / W2;
      const int dy = t & 1, dz = (t >> 1) & 1, ci = t >> 2;
      slab[i] = x[((((int64_t)b * Cin + ci) * D2 + 2 * z + dz) * H2 + 2 * (y0 + rr) + dy) * W2 + xx];
    }
  }
  if (CIN > 0 && (Cout & 3) == 0) {
    // thread = (4-channel group, x group): the 4 x 8 CIN weights in registers as channel
    // pairs, f32x2 pair FMAs over two channel pairs per slab value -- per output 4 LDS reads
    // instead of 16 (each pair FMA is two v_fma_f32: no packed FP32 in this build, DESIGN.md
    // 6.1) -- and one 16-byte store
    constexpr int NK = CIN > 0 ? CIN * 8 : 1;
    const int C4 = Cout >> 2;
    const int XG = blockDim.x / C4;
    const int cq = tid % C4, xg = tid / C4;
    const bool act = xg < XG;
    const int c0 = 4 * (act ? cq : 0);
    f32x2 wa[NK], wb[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      wa[k] = f32x2{w[(int64_t)(c0 + 0) * NK + k], w[(int64_t)(c0 + 1) * NK + k]};
      wb[k] = f32x2{w[(int64_t)(c0 + 2) * NK + k], w[(int64_t)(c0 + 3) * NK + k]};
    }
    const f32x2 ba = bias ? f32x2{bias[c0], bias[c0 + 1]} : f32x2{0.f, 0.f};
    const f32x2 bb = bias ? f32x2{bias[c0 + 2], bias[c0 + 3]} : f32x2{0.f, 0.f};
    __syncthreads();
    if (!act) return;
    for (int rr = 0; rr < nr; ++rr) {
      const float* sl = slab + rr * rowf;
      float* orow = out + (((int64_t)b * D + z) * H + y0 + rr) * W * (int64_t)Cout;
      for (int xo = xg; xo < W; xo += XG) {
        f32x2 a0 = ba, a1 = bb;
#pragma unroll
        for (int ci = 0; ci < NK / 8; ++ci)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float2 v = *reinterpret_cast<const float2*>(sl + (ci * 4 + q) * W2 + 2 * xo);
            const int k = ci * 8 + 2 * q;
            a0 = wa[k] * v.x + a0;
            a1 = wb[k] * v.x + a1;
            a0 = wa[k + 1] * v.y + a0;
            a1 = wb[k + 1] * v.y + a1;
          }
        *reinterpret_cast<f32x4*>(orow + (int64_t)xo * Cout + c0) = f32x4{a0.x, a0.y, a1.x, a1.y};
      }
    }
    return;
  }
  const int XG = blockDim.x / Cout;
  const int co = tid % Cout, xg = tid / Cout;
  const bool act = xg < XG;
  const int cw = act ? co : 0;
  // weight (co, ci, dz, dy, dx) at w[(co * Cin + ci) * 8 + (dz * 4 + dy * 2 + dx)]
  constexpr int NW = CIN > 0 ? CIN * 8 : 1;
  float wr[NW];
  if (CIN > 0) {
#pragma unroll
    for (int k = 0; k < NW; ++k) wr[k] = w[(int64_t)cw * NW + k];
  }
  const float bv = bias ? bias[cw] : 0.f;
  __syncthreads();
  if (!act) return;
  for (int rr = 0; rr < nr; ++rr) {
    const float* sl = slab + rr * rowf;
    float* orow = out + (((int64_t)b * D + z) * H + y0 + rr) * W * (int64_t)Cout;
    for (int xo = xg; xo < W; xo += XG) {
      float acc = bv;
      if (CIN > 0) {
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // q = dz * 2 + dy; the dx pair is adjacent in the slab
            const float2 v = *reinterpret_cast<const float2*>(sl + (ci * 4 + q) * W2 + 2 * xo);
            acc += wr[ci * 8 + 2 * q] * v.x + wr[ci * 8 + 2 * q + 1] * v.y;
          }
      } else {
        for (int ci = 0; ci < Cin; ++ci)
          for (int q = 0; q < 4; ++q) {
            const float2 v = *reinterpret_cast<const float2*>(sl + (ci * 4 + q) * W2 + 2 * xo);
            acc += w[((int64_t)co * Cin + ci) * 8 + 2 * q] * v.x +
                   w[((int64_t)co * Cin + ci) * 8 + 2 * q + 1] * v.y;
          }
      }
      orow[(int64_t)xo * Cout + co] = acc;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Multi-scale fuse: out = shortcut + sum_s trilinear(src_s -> (D,H,W)), plus LN stats.
// Index/weight math is PyTorch's upsample_trilinear3d with align_corners=False and an
// explicit output size: scale = in/out, src = max(scale*(o+0.5)-0.5, 0), i0 = floor(src),
// i1 = i0 + (i0 < in-1), l1 = src - i0; identity when in == out.  The 8 corners are combined
// depth-outermost like ATen's CPU Interpolate<3> recursion.
// ---------------------------------------------------------------------------------------
struct MsfuseArgs {
  const float* src[4];
  int sd[4], sh[4], sw[4];
  int nsrc;
  const float* shortcut;
  const float* branch_scale;
  float* out;
  float* stats;
  float eps;
  int B, C, D, H, W;
  int dbg;  // timing experiments only (builds with MSF_DBG=1): phases skipped
};

#ifndef MSF_DBG
#define MSF_DBG 0
#endif

__device__ __forceinline__ void lin_index(int o, int in, int out, int& i0, int& i1, float& l0,
                                          float& l1) {
  if (in == out) {
    i0 = i1 = o;
    l0 = 1.f;
    l1 = 0.f;
    return;
  }
  const float scale = (float)in / (float)out;
  float s = __fmul_rn(scale, (float)o + 0.5f) - 0.5f;
  s = s < 0.f ? 0.f : s;
  i0 = min((int)floorf(s), in - 1);
  l1 = fminf(fmaxf(s - (float)i0, 0.f), 1.f);
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l0 = 1.f - l1;
}

template <int G, int V>
__global__ __launch_bounds__(256) void msfuse_kernel(MsfuseArgs a) {
  const int C = a.C, C4 = C >> 2;
  const int64_t P = (int64_t)a.D * a.H * a.W;
  const int64_t total = (int64_t)a.B * P;
  const int lane = threadIdx.x & 63, gl = lane & (G - 1);
  const int gpb = blockDim.x / G;
  bool live[V];
#pragma unroll
  for (int j = 0; j < V; ++j) live[j] = gl + j * G < C4;
  for (int64_t g = (int64_t)blockIdx.x * gpb + threadIdx.x / G; g < total;
       g += (int64_t)gridDim.x * gpb) {
    const int b = (int)(g / P);
    int64_t p = g - (int64_t)b * P;
    const int x = (int)(p % a.W);
    p /= a.W;
    const int y = (int)(p % a.H);
    const int z = (int)(p / a.H);
    f32x4 acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = f32x4{0, 0, 0, 0};
    for (int s = 0; s < a.nsrc; ++s) {
      const int sd = a.sd[s], sh = a.sh[s], sw = a.sw[s];
      int z0, z1, y0, y1, x0, x1;
      float wz0, wz1, wy0, wy1, wx0, wx1;
      lin_index(z, sd, a.D, z0, z1, wz0, wz1);
      lin_index(y, sh, a.H, y0, y1, wy0, wy1);
      lin_index(x, sw, a.W, x0, x1, wx0, wx1);
      const f32x4* base = reinterpret_cast<const f32x4*>(a.src[s] + (int64_t)b * sd * sh * sw * C);
      auto at = [&](int zz, int yy, int xx, int c4) {
        return base[(((int64_t)zz * sh + yy) * sw + xx) * C4 + c4];
      };
#pragma unroll
      for (int j = 0; j < V; ++j) {
        if (!live[j]) continue;
        const int c4 = gl + j * G;
        const f32x4 t00 = at(z0, y0, x0, c4) * wx0 + at(z0, y0, x1, c4) * wx1;
        const f32x4 t01 = at(z0, y1, x0, c4) * wx0 + at(z0, y1, x1, c4) * wx1;
        const f32x4 t10 = at(z1, y0, x0, c4) * wx0 + at(z1, y0, x1, c4) * wx1;
        const f32x4 t11 = at(z1, y1, x0, c4) * wx0 + at(z1, y1, x1, c4) * wx1;
        const f32x4 t0 = t00 * wy0 + t01 * wy1;
        const f32x4 t1 = t10 * wy0 + t11 * wy1;
        acc[j] += t0 * wz0 + t1 * wz1;
      }
    }
    if (a.branch_scale) {
      const float bs = a.branch_scale[b];
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] *= bs;
    }
    const f32x4* sc = reinterpret_cast<const f32x4*>(a.shortcut + g * C);
    f32x4* dst = reinterpret_cast<f32x4*>(a.out + g * C);
    f32x4 v[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      v[j] = live[j] ? sc[gl + j * G] + acc[j] : f32x4{0, 0, 0, 0};
      if (live[j]) dst[gl + j * G] = v[j];
    }
    if (a.stats) {
      float mean, rstd;
      row_stats<G, V>(v, live, (float)C, a.eps, mean, rstd);
      if (gl == 0) {
        a.stats[2 * g] = mean;
        a.stats[2 * g + 1] = rstd;
      }
    }
  }
}

// Row variant: workgroup = one output row (b, z, y).  For each source the depth/height
// interpolation is done once per source x position -- R_s[xs] = wz0 (wy0 r00 + wy1 r01) +
// wz1 (wy0 r10 + wy1 r11) over the 4 contributing source rows, staged in LDS -- and each output
// then needs 2 LDS reads per source (x interpolation last; ATen interpolates x first, so the
// fp32 rounding differs in the last bits).  Global traffic: the 4 source rows per source (L2)
// plus one read of the shortcut row and one write of the output row.
// COAL (round 6): the shortcut row is read and the output row written by contiguous 1-KB
// instructions (lane = f32x4 index of the row) through an LDS image of the row, instead of
// each instruction touching 16 positions' 64-B pieces (the compute mapping: G lanes per position)
template <int G, int V, bool COAL = false>
__global__ __launch_bounds__(256) void msfuse_row_kernel(MsfuseArgs a) {
  extern __shared__ __attribute__((aligned(16))) float R[];  // sum_s sw[s] * C [+ W * C: COAL]
  const int C = a.C, C4 = C >> 2;
  // XCD-contiguous row order: the hardware deals consecutive workgroups round-robin over the
  // 8 XCDs, which put neighbouring output rows -- which read the same 4 source rows per
  // source -- on different XCDs, each fetching them into its own L2 (PMC: 1.25x the
  // algorithmic bytes at stage 1).  Each XCD takes a contiguous run of rows instead.
  const int nb = gridDim.x, xcd = blockIdx.x & 7, q8 = nb >> 3, r8 = nb & 7;
  int r = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
  const int y = r % a.H;
  r /= a.H;
  const int z = r % a.D;
  const int b = r / a.D;
  const int tid = threadIdx.x;
  // the shortcut row of this thread's first output position, issued before the source
  // staging so its latency overlaps it (a group owns one position when W <= 256 / G)
  const int lane0 = tid & 63, gl0 = lane0 & (G - 1);
  const int64_t rowbase0 = (((int64_t)b * a.D + z) * a.H + y) * a.W;
  const int xf = tid / G;
  f32x4 scp[V];
  constexpr int NK = COAL ? 4 : 1;  // COAL: W * C4 <= 1024 f32x4 per row (host-checked)
  f32x4 scv[NK];
  const int nrow4 = a.W * C4;
  if (COAL) {
    const f32x4* sr = reinterpret_cast<const f32x4*>(a.shortcut + rowbase0 * C);
#pragma unroll
    for (int k = 0; k < NK; ++k) scv[k] = sr[min(tid + 256 * k, nrow4 - 1)];
  } else if (xf < a.W) {
    const f32x4* sc0 = reinterpret_cast<const f32x4*>(a.shortcut + (rowbase0 + xf) * C);
#pragma unroll
    for (int j = 0; j < V; ++j) scp[j] = sc0[min(gl0 + j * G, C4 - 1)];
  }
  int roff[4];
  int ro = 0;
#if MSF_DBG
  const int nsrc_stage = (a.dbg & 2) ? 0 : a.nsrc;
  for (int s = 0; s < a.nsrc; ++s) roff[s] = 0;
  for (int s = 0; s < nsrc_stage; ++s) {
#else
  for (int s = 0; s < a.nsrc; ++s) {
#endif
    roff[s] = ro;
    const int sd = a.sd[s], sh = a.sh[s], sw = a.sw[s];
    int z0, z1, y0, y1;
    float wz0, wz1, wy0, wy1;
    lin_index(z, sd, a.D, z0, z1, wz0, wz1);
    lin_index(y, sh, a.H, y0, y1, wy0, wy1);
    const f32x4* base = reinterpret_cast<const f32x4*>(a.src[s] + (int64_t)b * sd * sh * sw * C);
    const f32x4* r00 = base + ((int64_t)z0 * sh + y0) * sw * C4;
    const f32x4* r01 = base + ((int64_t)z0 * sh + y1) * sw * C4;
    const f32x4* r10 = base + ((int64_t)z1 * sh + y0) * sw * C4;
    const f32x4* r11 = base + ((int64_t)z1 * sh + y1) * sw * C4;
    for (int i = tid; i < sw * C4; i += blockDim.x) {
      const f32x4 t0 = r00[i] * wy0 + r01[i] * wy1;
      const f32x4 t1 = r10[i] * wy0 + r11[i] * wy1;
      reinterpret_cast<f32x4*>(R + ro)[i] = t0 * wz0 + t1 * wz1;
    }
    ro += sw * C;
  }
  f32x4* T = reinterpret_cast<f32x4*>(R + ro);  // COAL: the row image [W][C4]
  if (COAL) {
#pragma unroll
    for (int k = 0; k < NK; ++k)
      if (tid + 256 * k < nrow4) T[tid + 256 * k] = scv[k];
  }
  __syncthreads();
  const int lane = tid & 63, gl = lane & (G - 1);
  const int gpb = blockDim.x / G;
  bool live[V];
#pragma unroll
  for (int j = 0; j < V; ++j) live[j] = gl + j * G < C4;
  const float bs = a.branch_scale ? a.branch_scale[b] : 1.f;
  const int64_t rowbase = (((int64_t)b * a.D + z) * a.H + y) * a.W;
  for (int x = tid / G; x < a.W; x += gpb) {
    f32x4 acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = f32x4{0, 0, 0, 0};
    for (int s = 0; s < a.nsrc; ++s) {
      int x0, x1;
      float wx0, wx1;
      lin_index(x, a.sw[s], a.W, x0, x1, wx0, wx1);
      const f32x4* R0 = reinterpret_cast<const f32x4*>(R + roff[s]) + x0 * C4;
      const f32x4* R1 = reinterpret_cast<const f32x4*>(R + roff[s]) + x1 * C4;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int c4 = min(gl + j * G, C4 - 1);
        acc[j] += R0[c4] * wx0 + R1[c4] * wx1;
      }
    }
    const f32x4* sc = reinterpret_cast<const f32x4*>(a.shortcut + (rowbase + x) * C);
    f32x4* dst = reinterpret_cast<f32x4*>(a.out + (rowbase + x) * C);
    f32x4 v[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c4 = min(gl + j * G, C4 - 1);
      if (COAL) {
        const f32x4 o = T[x * C4 + c4] + acc[j] * bs;
        v[j] = live[j] ? o : f32x4{0, 0, 0, 0};
        if (live[j]) T[x * C4 + c4] = o;
        continue;
      }
      const f32x4 o = (x == xf ? scp[j] : sc[c4]) + acc[j] * bs;
      v[j] = live[j] ? o : f32x4{0, 0, 0, 0};
#if MSF_DBG
      if (live[j] && (!(a.dbg & 1) || o.x == 1234.5f)) dst[c4] = o;
#else
      if (live[j]) dst[c4] = o;
#endif
    }
    if (a.stats) {
      float mean, rstd;
      row_stats<G, V>(v, live, (float)C, a.eps, mean, rstd);
      if (gl == 0) {
        a.stats[2 * (rowbase + x)] = mean;
        a.stats[2 * (rowbase + x) + 1] = rstd;
      }
    }
  }
  if (COAL) {
    __syncthreads();
    f32x4* orow = reinterpret_cast<f32x4*>(a.out + rowbase * C);
#pragma unroll
    for (int k = 0; k < NK; ++k)
      if (tid + 256 * k < nrow4) orow[tid + 256 * k] = T[tid + 256 * k];
  }
}

// ---------------------------------------------------------------------------------------
// proj_out: channel-last (B, S, C) -> [non-affine LayerNorm] -> NCDHW (B, C, S).
// Tile = TP positions of one batch; row groups normalise into an LDS [C][TP+1] image, then
// lanes run along positions so every NCDHW row segment is written contiguously.
// ---------------------------------------------------------------------------------------
template <int G, int V>
__global__ __launch_bounds__(256) void proj_out_kernel(const float* __restrict__ x,
                                                       float* __restrict__ out, int normalize,
                                                       float eps, int B, int C, int64_t S,
                                                       int TP) {
  extern __shared__ __attribute__((aligned(16))) float T[];  // [C][TP+1]
  const int C4 = C >> 2;
  const int64_t ntile = (S + TP - 1) / TP;
  const int b = (int)(blockIdx.x / ntile);
  const int64_t s0 = (blockIdx.x % ntile) * TP;
  const int np = (int)min((int64_t)TP, S - s0);
  const int lane = threadIdx.x & 63, gl = lane & (G - 1);
  const int gpb = blockDim.x / G;
  bool live[V];
#pragma unroll
  for (int j = 0; j < V; ++j) live[j] = gl + j * G < C4;
  for (int p = threadIdx.x / G; p < TP; p += gpb) {
    const bool pv = p < np;  // uniform per group; padded groups still join the shuffles
    const f32x4* row = reinterpret_cast<const f32x4*>(x + ((int64_t)b * S + s0 + (pv ? p : 0)) * C);
    f32x4 v[V];
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = live[j] ? row[gl + j * G] : f32x4{0, 0, 0, 0};
    if (normalize) {
      float mean, rstd;
      row_stats<G, V>(v, live, (float)C, eps, mean, rstd);
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] = (v[j] - mean) * rstd;
    }
    if (pv) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        if (!live[j]) continue;
        const int c = 4 * (gl + j * G);
        T[(c + 0) * (TP + 1) + p] = v[j].x;
        T[(c + 1) * (TP + 1) + p] = v[j].y;
        T[(c + 2) * (TP + 1) + p] = v[j].z;
        T[(c + 3) * (TP + 1) + p] = v[j].w;
      }
    }
  }
  __syncthreads();
  float* ob = out + (int64_t)b * C * S + s0;
  if (TP == 64) {
    // lane = position, wave = channel stride: no per-element index division (the generic loop
    // below divides by np for every element; the VALU pass showed the kernel 77 % issue-busy)
    const int p = threadIdx.x & 63;
    if (p < np)
      for (int c = threadIdx.x >> 6; c < C; c += blockDim.x >> 6)
        ob[(int64_t)c * S + p] = T[c * (TP + 1) + p];
    return;
  }
  for (int i = threadIdx.x; i < C * np; i += blockDim.x) {
    const int c = i / np, p = i - c * np;
    ob[(int64_t)c * S + p] = T[c * (TP + 1) + p];
  }
}

// proj_out for a channel-last consumer: (M, C) -> non-affine LayerNorm -> (M, C).  The same
// row groups, row_stats and (v - mean) * rstd as proj_out_kernel, so the values are bitwise
// those of the NCDHW write; the full model's UnetResBlocks read this layout directly instead
// of transposing proj_out's NCDHW result back (one read + one write per stage output).
template <int G, int V>
__global__ __launch_bounds__(256) void proj_out_cl_kernel(const float* __restrict__ x,
                                                          float* __restrict__ out, float eps,
                                                          int64_t M, int C) {
  const int C4 = C >> 2;
  const int gl = threadIdx.x & (G - 1);
  const int64_t m = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G;
  if (m >= M) return;  // uniform per group: the group's shuffles see only live rows
  bool live[V];
#pragma unroll
  for (int j = 0; j < V; ++j) live[j] = gl + j * G < C4;
  const f32x4* row = reinterpret_cast<const f32x4*>(x + m * C);
  f32x4* dst = reinterpret_cast<f32x4*>(out + m * C);
  f32x4 v[V];
#pragma unroll
  for (int j = 0; j < V; ++j) v[j] = live[j] ? row[gl + j * G] : f32x4{0, 0, 0, 0};
  float mean, rstd;
  row_stats<G, V>(v, live, (float)C, eps, mean, rstd);
#pragma unroll
  for (int j = 0; j < V; ++j)
    if (live[j]) dst[gl + j * G] = (v[j] - mean) * rstd;
}

}  // namespace wf

using namespace wf;

extern "C" int wf_patch_embed_ll_fwd(const float* x, const float* w, const float* bias,
                                     float* out, const float* ln_w, const float* ln_b,
                                     float ln_eps, float* ll, int64_t B, int64_t Cin,
                                     int64_t Cout, int64_t D, int64_t H, int64_t W, void* stream) {
  WF_REQUIRE(B >= 1 && D >= 2 && H >= 2 && W >= 2, "empty tensor");
  WF_REQUIRE(Cout == 48 && (Cin == 4 || Cin == 1),
             "PatchEmbed + LL: Cin 4 or 1, Cout 48 (the encoder stem)");
  WF_REQUIRE(D % 2 == 0 && H % 2 == 0 && W % 2 == 0 && W <= 64,
             "PatchEmbed + LL: even output sizes, W <= 64");
  WF_REQUIRE(B * D * H * W * Cout < ((int64_t)1 << 31), "tensor too large");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(w);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE_PTR(ln_w);
  WF_REQUIRE_PTR(ln_b);
  WF_REQUIRE_PTR(ll);
  const unsigned blocks = (unsigned)(B * (D / 2) * (H / 2));
  // (WF_PE_LL_VALU=1: the fp32-FMA kernel, A/B)
  static const bool valu = getenv("WF_PE_LL_VALU") != nullptr;
  static const bool v1 = getenv("WF_PE_LL_V1") != nullptr;  // A/B: the LDS row-tile version
  if (Cin == 4 && !valu && !v1)
    hipLaunchKernelGGL(patch_embed_ll_mfma2_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       x, w, bias, out, ln_w, ln_b, ln_eps, ll, (int)D, (int)H, (int)W);
  else if (Cin == 4 && !valu)
    hipLaunchKernelGGL(patch_embed_ll_mfma_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       x, w, bias, out, ln_w, ln_b, ln_eps, ll, (int)D, (int)H, (int)W);
  else if (Cin == 4)
    hipLaunchKernelGGL((patch_embed_ll_kernel<4, 48>), dim3(blocks), dim3(256), 0,
                       (hipStream_t)stream, x, w, bias, out, ln_w, ln_b, ln_eps, ll, (int)D,
                       (int)H, (int)W);
  else
    hipLaunchKernelGGL((patch_embed_ll_kernel<1, 48>), dim3(blocks), dim3(256), 0,
                       (hipStream_t)stream, x, w, bias, out, ln_w, ln_b, ln_eps, ll, (int)D,
                       (int)H, (int)W);
  return check_launch("wf_patch_embed_ll_fwd");
}

extern "C" int wf_patch_embed_fwd(const float* x, const float* w, const float* bias, float* out,
                                  int64_t B, int64_t Cin, int64_t Cout, int64_t D, int64_t H,
                                  int64_t W, void* stream) {
  WF_REQUIRE(B >= 1 && Cin >= 1 && Cout >= 1 && D >= 1 && H >= 1 && W >= 1, "empty tensor");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(w);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE(Cout <= 256, "PatchEmbed: at most 256 output channels");
  const size_t row_lds = (size_t)Cin * 8 * W * sizeof(float);
  WF_REQUIRE(row_lds <= 64 * 1024, "PatchEmbed row tile exceeds 64 KB of LDS");
  static const bool one_shot = getenv("WF_PE_ONESHOT") != nullptr;  // A/B: the kernel below
  static const bool rowstream = getenv("WF_PE_ROWSTREAM") != nullptr;  // A/B: the row stream
  if (!one_shot && !rowstream && Cout == 48 && (Cin == 4 || Cin == 1) &&
      B * D * H * W < ((int64_t)1 << 31)) {
    const int64_t total = B * D * H * W;
    const unsigned blocks = (unsigned)cdiv(total, 256);
    if (Cin == 4)
      hipLaunchKernelGGL((patch_embed_lane_kernel<4, 48>), dim3(blocks), dim3(256), 0,
                         (hipStream_t)stream, x, w, bias, out, (int)D, (int)H, (int)W, total);
    else
      hipLaunchKernelGGL((patch_embed_lane_kernel<1, 48>), dim3(blocks), dim3(256), 0,
                         (hipStream_t)stream, x, w, bias, out, (int)D, (int)H, (int)W, total);
    return check_launch("wf_patch_embed_fwd");
  }
  if (!one_shot && Cin == 4 && Cout % 4 == 0 && Cout <= 256 && H % 4 == 0 &&
      4 * (int64_t)Cin * 8 * W / 4 <= 8 * 256) {
    constexpr int R = 4;
    const int64_t ngroups = B * D * (H / R);
    const size_t lds = 2 * R * row_lds;
    const int64_t blocks = std::min<int64_t>(ngroups, 256 * 2);  // 2 persistent per CU (LDS)
    const int xg = 256 / (int)(Cout / 4);
    const int64_t xi = cdiv(W, xg);
    void (*k)(const float*, const float*, const float*, float*, int, int, int, int, int64_t) =
        xi == 1 ? patch_embed_stream_kernel<R, 1> : xi == 2 ? patch_embed_stream_kernel<R, 2>
      : xi == 3 ? patch_embed_stream_kernel<R, 3> : xi == 4 ? patch_embed_stream_kernel<R, 4>
      : xi == 5 ? patch_embed_stream_kernel<R, 5> : xi == 6 ? patch_embed_stream_kernel<R, 6>
                : nullptr;
    if (k && B * D * H * W * Cout * 4 < ((int64_t)1 << 31) - 16) {
      if (lds > 64 * 1024)
        set_max_lds(reinterpret_cast<const void*>(k), (int)lds);
      hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, x, w,
                         bias, out, (int)Cout, (int)D, (int)H, (int)W, ngroups);
      return check_launch("wf_patch_embed_fwd");
    }
  }
  // rows per workgroup: up to 4 within 32 KB of LDS, while the grid keeps >= 2048 workgroups
  static const int rmax = getenv("WF_PE_ROWS") ? atoi(getenv("WF_PE_ROWS")) : 4;
  int R = 1;
  while (R * 2 <= rmax && R * 2 <= H && row_lds * R * 2 <= 32 * 1024 &&
         B * D * cdiv(H, R * 2) >= 2048)
    R *= 2;
  const size_t lds = row_lds * R;
  const dim3 grid((unsigned)(B * D * cdiv(H, R))), block(256);
  hipStream_t s = (hipStream_t)stream;
  const int ci = (int)Cin, co = (int)Cout, d = (int)D, h = (int)H, ww = (int)W;
  switch (Cin) {
    case 1: hipLaunchKernelGGL(patch_embed_kernel<1>, grid, block, lds, s, x, w, bias, out, ci, co, d, h, ww, R); break;
    case 2: hipLaunchKernelGGL(patch_embed_kernel<2>, grid, block, lds, s, x, w, bias, out, ci, co, d, h, ww, R); break;
    case 3: hipLaunchKernelGGL(patch_embed_kernel<3>, grid, block, lds, s, x, w, bias, out, ci, co, d, h, ww, R); break;
    case 4: hipLaunchKernelGGL(patch_embed_kernel<4>, grid, block, lds, s, x, w, bias, out, ci, co, d, h, ww, R); break;
    default: hipLaunchKernelGGL(patch_embed_kernel<0>, grid, block, lds, s, x, w, bias, out, ci, co, d, h, ww, R); break;
  }
  return check_launch("wf_patch_embed_fwd");
}

extern "C" int wf_msfuse_fwd(const float* const* src, const int64_t* src_dhw, int nsrc,
                             const float* shortcut, const float* branch_scale, float* out,
                             float* stats, float ln_eps,
                             int64_t B, int64_t C, int64_t D, int64_t H, int64_t W,
                             void* stream) {
  WF_REQUIRE(nsrc >= 0 && nsrc <= 4, "at most 4 sources");
  WF_REQUIRE(B >= 1 && C >= 4 && C % 4 == 0, "C must be a positive multiple of 4");
  WF_REQUIRE_PTR(shortcut);
  WF_REQUIRE_PTR(out);
  MsfuseArgs a{};
  for (int s = 0; s < nsrc; ++s) {
    WF_REQUIRE_PTR(src[s]);
    a.src[s] = src[s];
    a.sd[s] = (int)src_dhw[3 * s];
    a.sh[s] = (int)src_dhw[3 * s + 1];
    a.sw[s] = (int)src_dhw[3 * s + 2];
    WF_REQUIRE(a.sd[s] >= 1 && a.sh[s] >= 1 && a.sw[s] >= 1, "empty source");
  }
  a.nsrc = nsrc;
  a.shortcut = shortcut;
  a.branch_scale = branch_scale;
  a.out = out;
  a.stats = stats;
  a.eps = ln_eps;
  a.B = (int)B;
  a.C = (int)C;
  a.D = (int)D;
  a.H = (int)H;
  a.W = (int)W;
  a.dbg = MSF_DBG && getenv("MSF_DBG") ? atoi(getenv("MSF_DBG")) : 0;
  const int64_t total = B * D * H * W;
  int64_t rlds = 0;
  for (int s = 0; s < nsrc; ++s) rlds += (int64_t)a.sw[s] * C * 4;
  return dispatch_gv(C / 4, [&](auto G_, auto V_) -> int {
    constexpr int G = decltype(G_)::value, V = decltype(V_)::value;
    // COAL for 4-lane groups only: stage 1 (C = 48) 231-233 -> 215-218 us; at C = 96 and
    // wider it measured 2-5 % slower (profiles/r6/r6ab_msfuse_coal_ab.txt)
    static const bool coal = !getenv("WF_MSF_COAL") || getenv("WF_MSF_COAL")[0] != '0';
    if (G <= 4 && coal && W * (C / 4) <= 1024 && W <= 256 / G && rlds + W * C * 4 <= 64 * 1024 &&
        B * D * H < ((int64_t)1 << 31)) {
      hipLaunchKernelGGL((msfuse_row_kernel<G, V, true>), dim3((unsigned)(B * D * H)), dim3(256),
                         (size_t)(rlds + W * C * 4), (hipStream_t)stream, a);
      return check_launch("wf_msfuse_fwd");
    }
    if (rlds <= 64 * 1024 && B * D * H < ((int64_t)1 << 31)) {
      hipLaunchKernelGGL((msfuse_row_kernel<G, V>), dim3((unsigned)(B * D * H)), dim3(256),
                         (size_t)rlds, (hipStream_t)stream, a);
      return check_launch("wf_msfuse_fwd");
    }
    int64_t blocks = cdiv(total, 256 / G);
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL((msfuse_kernel<G, V>), dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, a);
    return check_launch("wf_msfuse_fwd");
  });
}

extern "C" int wf_proj_out_fwd(const float* x, float* out, int normalize, float eps, int64_t B,
                               int64_t C, int64_t S, void* stream) {
  WF_REQUIRE(B >= 1 && S >= 1 && C >= 4 && C % 4 == 0, "C must be a positive multiple of 4");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(out);
  // LDS [C][TP+1] within 64 KB; TP + 1 odd, so the channel rows a group's lanes write (4 apart)
  // spread over the banks (C = 384 gave TP + 1 = 32 and C = 192 64: every lane of a group on
  // one bank, 29 / 16 conflict cycles per LDS instruction in profiles/r6/r6j_streaming_sq.txt)
  int64_t TP = (64 * 1024 / 4) / C - 1;
  if (TP > 64) TP = 64;
  if (TP < 1) TP = 1;
  if (TP > S) TP = S;
  if (TP > 1 && (TP + 1) % 2 == 0) --TP;
  const size_t lds = (size_t)C * (TP + 1) * sizeof(float);
  const int64_t blocks = B * cdiv(S, TP);
  return dispatch_gv(C / 4, [&](auto G_, auto V_) -> int {
    constexpr int G = decltype(G_)::value, V = decltype(V_)::value;
    hipLaunchKernelGGL((proj_out_kernel<G, V>), dim3((unsigned)blocks), dim3(256), lds,
                       (hipStream_t)stream, x, out, normalize, eps, (int)B, (int)C, S, (int)TP);
    return check_launch("wf_proj_out_fwd");
  });
}

extern "C" int wf_proj_out_cl_fwd(const float* x, float* out, float eps, int64_t M, int64_t C,
                                  void* stream) {
  WF_REQUIRE(M >= 1 && C >= 4 && C % 4 == 0, "C must be a positive multiple of 4");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(out);
  return dispatch_gv(C / 4, [&](auto G_, auto V_) -> int {
    constexpr int G = decltype(G_)::value, V = decltype(V_)::value;
    const int64_t blocks = cdiv(M, 256 / G);
    WF_REQUIRE(blocks < ((int64_t)1 << 31), "too many rows");
    hipLaunchKernelGGL((proj_out_cl_kernel<G, V>), dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, x, out, eps, M, (int)C);
    return check_launch("wf_proj_out_cl_fwd");
  });
}
