// dwt.hip -- 3D Haar analysis (a1) and multi-level synthesis (a11) for gfx950.
//
// Reference arithmetic: ptwt 0.1.9 wavedec3 / waverec3 with wavelet 'db1', mode 'zero'
// (call sites network_models/wave_helper.py:350 and network_models/idwt_upsample.py:160).
// For even sizes the 'zero' padding is empty and one level is, per axis,
//   analysis  a = (x[2n] + x[2n+1]) / sqrt2,  d = (x[2n] - x[2n+1]) / sqrt2
//   synthesis x[2n] = (a + d) / sqrt2,        x[2n+1] = (a - d) / sqrt2
// (pywt dec_lo/dec_hi/rec_lo/rec_hi of 'haar').  ptwt applies the 3D outer-product filter
// in one conv, i.e. each coefficient is (signed sum of 8 voxels) * (1/sqrt2)^3; the kernels
// below do the same: 3 butterfly stages without scaling, then one multiply by 2^-1.5.
//
// HBM roofline: both kernels are pure streaming (8 fp32 in -> 8 fp32 out per 2x2x2 cube).
#include "rowgroup.hpp"

namespace wf {

constexpr float kHaar3 = 0.35355339059327373f;  // (1/sqrt 2)^3

// Forward: one row group per OUTPUT position; lanes over channels.
// x (B,D,H,W,C) channel-last -> bands (8,B,D/2,H/2,W/2,C); band k bits (bd,bh,bw) = k>>2,k>>1,k.
// NB = 8: all bands; NB = 1: the LL band alone (the detail butterflies are dead code then;
// band 0's sums are formed in the same order, so LL is bitwise the 8-band kernel's)
template <int G, int V, bool LN, int NB = 8>
__global__ __launch_bounds__(256) void dwt3d_haar_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ ln_w, const float* __restrict__ ln_b,
    float ln_eps, float* __restrict__ bands, int B, int C, int D, int H, int W) {
  const int C4 = C >> 2;
  const int d = D >> 1, h = H >> 1, w = W >> 1;
  // output positions in 32 bits (the host's element bound keeps them below 2^28): the
  // position decode is three 32-bit divisions instead of the software 64-bit ones
  const uint32_t P = (uint32_t)d * h * w;         // output positions per batch
  const uint32_t total = (uint32_t)B * P;
  const int lane = threadIdx.x & 63;
  const int gl = lane & (G - 1);
  const int groups_per_block = blockDim.x / G;
  const uint32_t gid0 = blockIdx.x * (uint32_t)groups_per_block + threadIdx.x / G;
  const uint32_t gstride = gridDim.x * (uint32_t)groups_per_block;
  const int64_t band_stride = (int64_t)total * C;  // elements per band

  bool live[V];
  f32x4 gw[V], gb[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c4 = gl + j * G;
    live[j] = c4 < C4;
    if (LN) {
      gw[j] = live[j] ? reinterpret_cast<const f32x4*>(ln_w)[c4] : f32x4{0, 0, 0, 0};
      gb[j] = live[j] ? reinterpret_cast<const f32x4*>(ln_b)[c4] : f32x4{0, 0, 0, 0};
    }
  }

  for (uint32_t g = gid0; g < total; g += gstride) {
    const int b = (int)(g / P);
    uint32_t p = g - (uint32_t)b * P;
    const int ox = (int)(p % (uint32_t)w);
    p /= (uint32_t)w;
    const int oy = (int)(p % (uint32_t)h);
    const int oz = (int)(p / (uint32_t)h);

    f32x4 v[8][V];
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int iz = 2 * oz + (n >> 2), iy = 2 * oy + ((n >> 1) & 1), ix = 2 * ox + (n & 1);
      const f32x4* row = reinterpret_cast<const f32x4*>(
          x + ((((int64_t)b * D + iz) * H + iy) * W + ix) * C);
#pragma unroll
      for (int j = 0; j < V; ++j) v[n][j] = live[j] ? row[gl + j * G] : f32x4{0, 0, 0, 0};
    }
    if (LN) {
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        float mean, rstd;
        row_stats<G, V>(v[n], live, (float)C, ln_eps, mean, rstd);
#pragma unroll
        for (int j = 0; j < V; ++j) v[n][j] = (v[n][j] - mean) * rstd * gw[j] + gb[j];
      }
    }
    // butterflies along x (n bit0), y (bit1), z (bit2); slot index becomes the band index
#pragma unroll
    for (int bit = 1; bit < 8; bit <<= 1) {
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        if (!(n & bit)) {
#pragma unroll
          for (int j = 0; j < V; ++j) {
            f32x4 s0 = v[n][j], s1 = v[n | bit][j];
            v[n][j] = s0 + s1;
            v[n | bit][j] = s0 - s1;
          }
        }
      }
    }
    const int64_t obase = (int64_t)g * C;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      f32x4* dst = reinterpret_cast<f32x4*>(bands + k * band_stride + obase);
#pragma unroll
      for (int j = 0; j < V; ++j)
        if (live[j]) dst[gl + j * G] = v[k][j] * kHaar3;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Inverse: multi-level, fused.  One workgroup = one row (b, z1, y1, all x1) of the FINEST
// detail grid and a block of CB channels.  Phase 1 (lanes over channels, matching the
// channel-last detail bands of the forward kernel): every (c, x1) item rebuilds the level-
// (L-1) LL value by walking the coarser levels, then the 8 outputs of its 2x2x2 cube into
// LDS.  Phase 2 (lanes over x): rows of 2*w1 contiguous floats go to the NCDHW output.
// ---------------------------------------------------------------------------------------
constexpr int kMaxLevels = 4;
struct IdwtArgs {
  const float* ll;
  int64_t ll_bstride, ll_cs, ll_ps;  // LL element (b, c, p) at b*ll_bstride + c*ll_cs + p*ll_ps
  const float* det[kMaxLevels * 7];
  int64_t ds[kMaxLevels * 4];  // per level: batch, channel, z, (y*W_l+x) strides
  float* out;
  int64_t out_bstride;
  int64_t ldo;   // channel-last output (CL kernel): floats between positions, channels contiguous
  int levels, B, C, d, h, w, CB;
  const float* skip;             // cl4 kernel: concat skip rows (channel-last) or NULL
  int64_t skip_bstride, skip_ld;
};

__device__ __forceinline__ float idwt_coef(const IdwtArgs& a, int l, int k, int b, int c,
                                           int z, int y, int x) {
  const int64_t Wl = (int64_t)a.w << l;
  const int64_t off = b * a.ds[4 * l] + c * a.ds[4 * l + 1] + z * a.ds[4 * l + 2] +
                      ((int64_t)y * Wl + x) * a.ds[4 * l + 3];
  return a.det[l * 7 + k][off];
}

// CL: write a channel-last output (the decoder's concat buffer kept channels_last_3d) -- the
// LDS image is then [2][2][2*w1][CB+1] (channels innermost, padded) and phase 2 writes each
// position's CB channels contiguously
template <bool CL>
__global__ __launch_bounds__(256) void idwt3d_haar_kernel(IdwtArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_out[];  // [CB][2][2][2*w1]
  const int L = a.levels;
  const int w1 = a.w << (L - 1), h1 = a.h << (L - 1), d1 = a.d << (L - 1);
  const int Wo = 2 * w1, Ho = 2 * h1, Do = 2 * d1;
  int row = blockIdx.x;                 // over B * d1 * h1
  const int y1 = row % h1;
  row /= h1;
  const int z1 = row % d1;
  const int b = row / d1;
  const int c0 = blockIdx.y * a.CB;
  const int CB = min(a.CB, a.C - c0);

  for (int item = threadIdx.x; item < CB * w1; item += blockDim.x) {
    const int cl = item % CB, x1 = item / CB;
    const int c = c0 + cl;
    // coarsest LL (NCDHW, contiguous spatial)
    const int zc = z1 >> (L - 1), yc = y1 >> (L - 1), xc = x1 >> (L - 1);
    float ll = a.ll[b * a.ll_bstride + (int64_t)c * a.ll_cs +
                    (((int64_t)zc * a.h + yc) * a.w + xc) * a.ll_ps];
    // levels 0..L-2 produce the LL of the next level at the ancestor of (z1,y1,x1)
    for (int l = 0; l < L - 1; ++l) {
      const int sh = L - 1 - l;             // ancestor at level l is (z1,y1,x1) >> sh
      const int zl = z1 >> sh, yl = y1 >> sh, xl = x1 >> sh;
      const int sz = (z1 >> (sh - 1)) & 1, sy = (y1 >> (sh - 1)) & 1, sx = (x1 >> (sh - 1)) & 1;
      float acc = ll;
#pragma unroll
      for (int k = 1; k < 8; ++k) {
        const int bd = (k >> 2) & 1, bh = (k >> 1) & 1, bw = k & 1;
        const int neg = (bd & sz) ^ (bh & sy) ^ (bw & sx);
        const float cv = idwt_coef(a, l, k - 1, b, c, zl, yl, xl);
        acc += neg ? -cv : cv;
      }
      ll = acc * kHaar3;
    }
    // finest level: all 8 outputs of the cube via inverse butterflies
    float v[8];
    v[0] = ll;
#pragma unroll
    for (int k = 1; k < 8; ++k) v[k] = idwt_coef(a, L - 1, k - 1, b, c, z1, y1, x1);
#pragma unroll
    for (int bit = 1; bit < 8; bit <<= 1) {
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        if (!(n & bit)) {
          const float s0 = v[n], s1 = v[n | bit];
          v[n] = s0 + s1;
          v[n | bit] = s0 - s1;
        }
      }
    }
    // slot n now holds sub-position (sz,sy,sx) = (n>>2, n>>1 & 1, n & 1)
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int sz = n >> 2, sy = (n >> 1) & 1, sx = n & 1;
      if (CL)
        lds_out[((sz * 2 + sy) * Wo + 2 * x1 + sx) * (a.CB + 1) + cl] = v[n] * kHaar3;
      else
        lds_out[((cl * 2 + sz) * 2 + sy) * Wo + 2 * x1 + sx] = v[n] * kHaar3;
    }
  }
  __syncthreads();
  float* obase = a.out + b * a.out_bstride;
  if (CL) {
    // item = (row r = (sz, sy), position xo, channel cl), channels fastest
    const int n = 4 * Wo * CB;
    for (int item = threadIdx.x; item < n; item += blockDim.x) {
      const int cl = item % CB, q = item / CB;
      const int xo = q % Wo, r = q / Wo;
      const int zo = 2 * z1 + (r >> 1), yo = 2 * y1 + (r & 1);
      obase[(((int64_t)zo * Ho + yo) * Wo + xo) * a.ldo + c0 + cl] = lds_out[q * (a.CB + 1) + cl];
    }
    return;
  }
  const int64_t plane = (int64_t)Do * Ho * Wo;
  const int nrows = CB * 4;
  for (int item = threadIdx.x; item < nrows * Wo; item += blockDim.x) {
    const int xo = item % Wo, r = item / Wo;
    const int cl = r >> 2, sz = (r >> 1) & 1, sy = r & 1;
    const int zo = 2 * z1 + sz, yo = 2 * y1 + sy;
    obase[(int64_t)(c0 + cl) * plane + ((int64_t)zo * Ho + yo) * Wo + xo] = lds_out[r * Wo + xo];
  }
}

// ---------------------------------------------------------------------------------------
// Channel-last in, channel-last out (the decoder's path: LL from the previous decoder stage,
// details = channel-last views of the DWT's band tensor, output = the concat buffer): a pure
// per-position stream, so no LDS.  One thread = one finest-level cube (b, z1, y1, x1) x 4
// channels, channels fastest: every load and store is 16 B per lane and consecutive lanes
// touch consecutive 16 B (LL row, each band row, each output position row).  The coarser
// levels (L > 1) are re-read by the 8^l descendants of a coefficient; they are 1/8 of the
// level below and hit L2.
// ---------------------------------------------------------------------------------------
// CAT: the fused torch.cat with the skip (wf_idwt3d_haar_cl_cat) -- a separate instantiation
// so counter passes and kernel traces tell the two launch kinds apart
template <bool CAT>
__global__ __launch_bounds__(256) void idwt3d_haar_cl4_kernel(IdwtArgs a, int64_t total) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  const int L = a.levels, C4 = a.C >> 2;
  const int w1 = a.w << (L - 1), h1 = a.h << (L - 1), d1 = a.d << (L - 1);
  // decoded in 32 bits (the host launches this kernel for total < 2^31): 64-bit divisions are
  // software routines, five of them per 256 B moved
  uint32_t r = (uint32_t)t;
  const int c = 4 * (int)(r % (uint32_t)C4);
  r /= (uint32_t)C4;
  const int x1 = (int)(r % (uint32_t)w1);
  r /= (uint32_t)w1;
  const int y1 = (int)(r % (uint32_t)h1);
  r /= (uint32_t)h1;
  const int z1 = (int)(r % (uint32_t)d1);
  const int b = (int)(r / (uint32_t)d1);
  auto coef4 = [&](int l, int k, int z, int y, int x) {
    const int64_t Wl = (int64_t)a.w << l;
    const int64_t off = b * a.ds[4 * l] + c + z * a.ds[4 * l + 2] + ((int64_t)y * Wl + x) * a.ds[4 * l + 3];
    return *reinterpret_cast<const f32x4*>(a.det[l * 7 + k] + off);
  };
  const int zc = z1 >> (L - 1), yc = y1 >> (L - 1), xc = x1 >> (L - 1);
  f32x4 ll = *reinterpret_cast<const f32x4*>(
      a.ll + b * a.ll_bstride + c + (((int64_t)zc * a.h + yc) * a.w + xc) * a.ll_ps);
  for (int l = 0; l < L - 1; ++l) {
    const int sh = L - 1 - l;
    const int zl = z1 >> sh, yl = y1 >> sh, xl = x1 >> sh;
    const int sz = (z1 >> (sh - 1)) & 1, sy = (y1 >> (sh - 1)) & 1, sx = (x1 >> (sh - 1)) & 1;
    f32x4 cv[7];
#pragma unroll
    for (int k = 1; k < 8; ++k) cv[k - 1] = coef4(l, k - 1, zl, yl, xl);
    f32x4 acc = ll;
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const int neg = (((k >> 2) & 1) & sz) ^ (((k >> 1) & 1) & sy) ^ ((k & 1) & sx);
      acc = neg ? acc - cv[k - 1] : acc + cv[k - 1];
    }
    ll = acc * kHaar3;
  }
  f32x4 v[8];
  v[0] = ll;
#pragma unroll
  for (int k = 1; k < 8; ++k) v[k] = coef4(L - 1, k - 1, z1, y1, x1);
#pragma unroll
  for (int bit = 1; bit < 8; bit <<= 1) {
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      if (!(n & bit)) {
        const f32x4 s0 = v[n], s1 = v[n | bit];
        v[n] = s0 + s1;
        v[n | bit] = s0 - s1;
      }
    }
  }
  const int Wo = 2 * w1, Ho = 2 * h1;
  float* ob = a.out + b * a.out_bstride + c;
  if (CAT) {  // torch.cat((out, skip), 1): the same 4 channels of the skip, C further
    const float* sb = a.skip + b * a.skip_bstride + c;
    f32x4 sk[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int zo = 2 * z1 + (n >> 2), yo = 2 * y1 + ((n >> 1) & 1), xo = 2 * x1 + (n & 1);
      sk[n] = *reinterpret_cast<const f32x4*>(sb + (((int64_t)zo * Ho + yo) * Wo + xo) * a.skip_ld);
    }
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int zo = 2 * z1 + (n >> 2), yo = 2 * y1 + ((n >> 1) & 1), xo = 2 * x1 + (n & 1);
      float* o = ob + (((int64_t)zo * Ho + yo) * Wo + xo) * a.ldo;
      *reinterpret_cast<f32x4*>(o) = v[n] * kHaar3;
      *reinterpret_cast<f32x4*>(o + a.C) = sk[n];
    }
    return;
  }
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    const int zo = 2 * z1 + (n >> 2), yo = 2 * y1 + ((n >> 1) & 1), xo = 2 * x1 + (n & 1);
    *reinterpret_cast<f32x4*>(ob + (((int64_t)zo * Ho + yo) * Wo + xo) * a.ldo) = v[n] * kHaar3;
  }
}

// ---------------------------------------------------------------------------------------
// Channel-last details, NCDHW LL and NCDHW output (the autograd path and wfa.idwt3d_haar
// without an output buffer).  One workgroup = one finest row (b, z1, y1) x a block of CB
// channels (a multiple of 4):
//   1. the CB LL rows are read coalesced along x (NCDHW rows) into LDS [CB][w1 + 1];
//   2. item = (x1, channel quad), quads fastest: the 7 finest bands as 16-B loads (consecutive
//      lanes on consecutive 16 B of a band row), coarser levels likewise, LL from LDS; the 8
//      outputs x 4 channels go to the LDS image [2][2][CB][Wo + 2] as 8-B (x pair) stores
//      (channel rows Wo + 2 floats apart: consecutive quads land 8 banks apart, <= 3-way);
//   3. the image's rows (Wo floats per (z, y, channel)) go out as 16-B stores.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void idwt3d_haar_nc4_kernel(IdwtArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_nc[];
  const int L = a.levels;
  const int w1 = a.w << (L - 1), h1 = a.h << (L - 1), d1 = a.d << (L - 1);
  const int Wo = 2 * w1, Ho = 2 * h1, Do = 2 * d1, WP = Wo + 2, LP = w1 + 1;
  // 1-D grid of (row, channel block) with the channel blocks of a row adjacent and every XCD
  // given a contiguous run: the blocks of one row read disjoint channel slices of the same
  // channel-last detail lines, which now meet in one XCD's L2 (dealt round-robin over the XCDs,
  // each block's 64-B slices pulled every 192-B position line again: 1.44x the algorithmic
  // bytes)
  const int ncb = (a.C + a.CB - 1) / a.CB;
  const int nb = gridDim.x, xcd = blockIdx.x & 7, q8 = nb >> 3, r8 = nb & 7;
  const int lb = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
  int row = lb / ncb;
  const int y1 = row % h1;
  row /= h1;
  const int z1 = row % d1;
  const int b = row / d1;
  const int c0 = (lb - (lb / ncb) * ncb) * a.CB;
  const int CB = min(a.CB, a.C - c0);
  const int CB4 = CB >> 2;
  float* lds_ll = lds_nc + (size_t)a.CB * 4 * WP;
  // 1. LL rows of the coarsest ancestor row (x varies by x1 >> (L-1))
  const int zc = z1 >> (L - 1), yc = y1 >> (L - 1);
  for (int i = threadIdx.x; i < CB * a.w; i += blockDim.x) {
    const int cl = i / a.w, xc = i - cl * a.w;
    lds_ll[cl * LP + xc] =
        a.ll[b * a.ll_bstride + (int64_t)(c0 + cl) * a.ll_cs + ((int64_t)zc * a.h + yc) * a.w + xc];
  }
  __syncthreads();
  for (int item = threadIdx.x; item < CB4 * w1; item += blockDim.x) {
    const int q = item % CB4, x1 = item / CB4;
    const int cl = 4 * q, c = c0 + cl;
    auto coef4 = [&](int l, int k, int z, int y, int x) {
      const int64_t Wl = (int64_t)a.w << l;
      const int64_t off = b * a.ds[4 * l] + c + z * a.ds[4 * l + 2] + ((int64_t)y * Wl + x) * a.ds[4 * l + 3];
      return *reinterpret_cast<const f32x4*>(a.det[l * 7 + k] + off);
    };
    const int xc = x1 >> (L - 1);
    f32x4 ll = f32x4{lds_ll[cl * LP + xc], lds_ll[(cl + 1) * LP + xc], lds_ll[(cl + 2) * LP + xc],
                     lds_ll[(cl + 3) * LP + xc]};
    for (int l = 0; l < L - 1; ++l) {
      const int sh = L - 1 - l;
      const int zl = z1 >> sh, yl = y1 >> sh, xl = x1 >> sh;
      const int sz = (z1 >> (sh - 1)) & 1, sy = (y1 >> (sh - 1)) & 1, sx = (x1 >> (sh - 1)) & 1;
      f32x4 cv[7];
#pragma unroll
      for (int k = 1; k < 8; ++k) cv[k - 1] = coef4(l, k - 1, zl, yl, xl);
      f32x4 acc = ll;
#pragma unroll
      for (int k = 1; k < 8; ++k) {
        const int neg = (((k >> 2) & 1) & sz) ^ (((k >> 1) & 1) & sy) ^ ((k & 1) & sx);
        acc = neg ? acc - cv[k - 1] : acc + cv[k - 1];
      }
      ll = acc * kHaar3;
    }
    f32x4 v[8];
    v[0] = ll;
#pragma unroll
    for (int k = 1; k < 8; ++k) v[k] = coef4(L - 1, k - 1, z1, y1, x1);
#pragma unroll
    for (int bit = 1; bit < 8; bit <<= 1) {
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        if (!(n & bit)) {
          const f32x4 s0 = v[n], s1 = v[n | bit];
          v[n] = s0 + s1;
          v[n | bit] = s0 - s1;
        }
      }
    }
    // slot n = (sz, sy, sx); the sx pair is adjacent in a row: one 8-B store per channel
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const f32x4 e = v[2 * r] * kHaar3, o = v[2 * r + 1] * kHaar3;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<f32x2*>(lds_nc + (r * a.CB + cl + j) * WP + 2 * x1) = f32x2{e[j], o[j]};
    }
  }
  __syncthreads();
  // 3. rows: (cl, r) x Wo floats, 16 B per lane
  float* obase = a.out + b * a.out_bstride;
  const int64_t plane = (int64_t)Do * Ho * Wo;
  const int V4 = Wo >> 2;
  for (int item = threadIdx.x; item < CB * 4 * V4; item += blockDim.x) {
    const int xv = item % V4, rr = item / V4;
    const int cl = rr % CB, r = rr / CB;
    const int zo = 2 * z1 + (r >> 1), yo = 2 * y1 + (r & 1);
    const float* src = lds_nc + (r * a.CB + cl) * WP + 4 * xv;
    const f32x2 lo = *reinterpret_cast<const f32x2*>(src), hi = *reinterpret_cast<const f32x2*>(src + 2);
    *reinterpret_cast<f32x4*>(obase + (int64_t)(c0 + cl) * plane + ((int64_t)zo * Ho + yo) * Wo + 4 * xv) =
        f32x4{lo.x, lo.y, hi.x, hi.y};
  }
}

}  // namespace wf

using namespace wf;

template <int NB>
static int dwt_haar_fwd(const float* x, const float* ln_w, const float* ln_b, float ln_eps,
                        float* bands, int64_t B, int64_t C, int64_t D, int64_t H, int64_t W,
                        void* stream) {
  WF_REQUIRE(B >= 1 && C >= 4 && C % 4 == 0, "need B >= 1 and C a positive multiple of 4");
  WF_REQUIRE(D >= 2 && H >= 2 && W >= 2 && D % 2 == 0 && H % 2 == 0 && W % 2 == 0,
             "D, H, W must be even (ptwt 'zero' mode with odd sizes is not supported)");
  WF_REQUIRE((int64_t)B * D * H * W * C < ((int64_t)1 << 31) * 4, "tensor too large");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(bands);
  const bool ln = ln_w != nullptr;
  if (ln) WF_REQUIRE_PTR(ln_b);
  const int64_t total = B * (D / 2) * (H / 2) * (W / 2);
  auto go = [&](auto G_, auto V_) -> int {
    constexpr int G = decltype(G_)::value, V = decltype(V_)::value;
    const int gpb = 256 / G;
    int64_t blocks = cdiv(total, gpb);
    if (blocks > 8192) blocks = 8192;
    if (ln)
      hipLaunchKernelGGL((dwt3d_haar_fwd_kernel<G, V, true, NB>), dim3((unsigned)blocks),
                         dim3(256), 0, (hipStream_t)stream, x, ln_w, ln_b, ln_eps, bands, (int)B,
                         (int)C, (int)D, (int)H, (int)W);
    else
      hipLaunchKernelGGL((dwt3d_haar_fwd_kernel<G, V, false, NB>), dim3((unsigned)blocks),
                         dim3(256), 0, (hipStream_t)stream, x, ln_w, ln_b, ln_eps, bands, (int)B,
                         (int)C, (int)D, (int)H, (int)W);
    return check_launch("wf_dwt3d_haar_fwd");
  };
  // C = 48 (stage 1, the 400 MB launch): 16 lanes x 1 float4 per position instead of 4 x 3
  // (4 idle lanes) -- 32 data VGPRs instead of 96, so the whole grid is resident at once
  static const bool wide = getenv("WF_DWT_G4") == nullptr;
  if (wide && C == 48) return go(ic<16>{}, ic<1>{});
  return dispatch_gv(C / 4, go);
}

extern "C" int wf_dwt3d_haar_fwd(const float* x, const float* ln_w, const float* ln_b,
                                 float ln_eps, float* bands, int64_t B, int64_t C, int64_t D,
                                 int64_t H, int64_t W, void* stream) {
  return dwt_haar_fwd<8>(x, ln_w, ln_b, ln_eps, bands, B, C, D, H, W, stream);
}

extern "C" int wf_dwt3d_haar_fwd_ll(const float* x, const float* ln_w, const float* ln_b,
                                    float ln_eps, float* ll, int64_t B, int64_t C, int64_t D,
                                    int64_t H, int64_t W, void* stream) {
  return dwt_haar_fwd<1>(x, ln_w, ln_b, ln_eps, ll, B, C, D, H, W, stream);
}

static int idwt_launch(const float* ll, int64_t ll_bstride, int64_t ll_cs, int64_t ll_ps,
                       const float* const* det, const int64_t* det_s, int levels, float* out,
                       int64_t out_bstride, int64_t ldo, int64_t B, int64_t C, int64_t d,
                       int64_t h, int64_t w, void* stream, const float* skip = nullptr,
                       int64_t skip_bstride = 0, int64_t skip_ld = 0) {
  WF_REQUIRE(levels >= 1 && levels <= kMaxLevels, "levels must be in [1, 4]");
  WF_REQUIRE(B >= 1 && C >= 1 && d >= 1 && h >= 1 && w >= 1, "empty tensor");
  WF_REQUIRE_PTR(ll);
  WF_REQUIRE_PTR(det);
  WF_REQUIRE_PTR(det_s);
  WF_REQUIRE_PTR(out);
  IdwtArgs a{};
  a.ll = ll;
  a.ll_bstride = ll_bstride;
  a.ll_cs = ll_cs;
  a.ll_ps = ll_ps;
  for (int i = 0; i < levels * 7; ++i) {
    WF_REQUIRE_PTR(det[i]);
    a.det[i] = det[i];
  }
  for (int i = 0; i < levels * 4; ++i) a.ds[i] = det_s[i];
  a.out = out;
  a.out_bstride = out_bstride;
  a.levels = levels;
  a.B = (int)B;
  a.C = (int)C;
  a.d = (int)d;
  a.h = (int)h;
  a.w = (int)w;
  a.ldo = ldo;
  const bool cl = ldo > 0;
  const int64_t w1 = w << (levels - 1), h1 = h << (levels - 1), d1 = d << (levels - 1);
  WF_REQUIRE(w1 <= 4096, "row too long");
  // 16-B paths: channel quads contiguous in every band (and in the LL / output where they are
  // channel-last), every base and stride a multiple of 4 floats
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  bool vec = C % 4 == 0 && getenv("WF_IDWT_SCALAR") == nullptr;
  for (int l = 0; l < levels && vec; ++l) {
    vec = det_s[4 * l + 1] == 1 && det_s[4 * l] % 4 == 0 && det_s[4 * l + 2] % 4 == 0 &&
          det_s[4 * l + 3] % 4 == 0;
    for (int k = 0; k < 7 && vec; ++k) vec = al16(det[l * 7 + k]);
  }
  vec = vec && al16(out) && out_bstride % 4 == 0;
  if (skip) {
    WF_REQUIRE(vec && cl && ll_cs == 1 && ll_ps % 4 == 0 && ll_bstride % 4 == 0 && al16(ll) &&
                   ldo % 4 == 0 && ldo >= 2 * C && al16(skip) && skip_ld % 4 == 0 &&
                   skip_ld >= C && skip_bstride % 4 == 0,
               "fused concat: channel-last LL / details / skip / output, 16-B aligned, C % 4 == 0");
    WF_REQUIRE(B * d1 * h1 * w1 * (C / 4) < ((int64_t)1 << 31), "fused concat: volume too large");
    a.skip = skip;
    a.skip_bstride = skip_bstride;
    a.skip_ld = skip_ld;
  }
  if (vec && cl && ll_cs == 1 && ll_ps % 4 == 0 && ll_bstride % 4 == 0 && al16(ll) && ldo % 4 == 0 &&
      B * d1 * h1 * w1 * (C / 4) < ((int64_t)1 << 31)) {
    const int64_t total = B * d1 * h1 * w1 * (C / 4);
    if (skip)
      hipLaunchKernelGGL(idwt3d_haar_cl4_kernel<true>, dim3((unsigned)cdiv(total, 256)),
                         dim3(256), 0, (hipStream_t)stream, a, total);
    else
      hipLaunchKernelGGL(idwt3d_haar_cl4_kernel<false>, dim3((unsigned)cdiv(total, 256)),
                         dim3(256), 0, (hipStream_t)stream, a, total);
    return check_launch("wf_idwt3d_haar_cl");
  }
  if (vec && !cl && ll_ps == 1 && (2 * w1) % 4 == 0) {
    // LDS: [4][CB][2 w1 + 2] output image + [CB][w1 + 1] LL rows, ~40 KB (4 workgroups / CU)
    const int64_t per_c = 4 * (4 * (2 * w1 + 2)) + 4 * (w1 + 1);
    int64_t cb = (40 * 1024 / per_c) / 4 * 4;
    if (cb < 4) cb = 4;
    if (cb > C) cb = C;
    if (cb * per_c <= 64 * 1024) {
      a.CB = (int)cb;
      WF_REQUIRE(B * d1 * h1 * cdiv(C, cb) < ((int64_t)1 << 31), "wf_idwt3d_haar: grid too large");
      dim3 grid((unsigned)(B * d1 * h1 * cdiv(C, cb)));
      hipLaunchKernelGGL(idwt3d_haar_nc4_kernel, grid, dim3(256), (size_t)(cb * per_c),
                         (hipStream_t)stream, a);
      return check_launch("wf_idwt3d_haar");
    }
  }
  // LDS budget 48 KB: CB * 8 * w1 floats (+ 8 * w1 of padding in the channel-last image)
  int64_t cb = (48 * 1024 / 4) / (8 * w1) - (cl ? 1 : 0);
  if (cb < 1) cb = 1;
  if (cb > C) cb = C;
  a.CB = (int)cb;
  const size_t lds = (size_t)(cb + (cl ? 1 : 0)) * 8 * w1 * sizeof(float);
  dim3 grid((unsigned)(B * d1 * h1), (unsigned)cdiv(C, cb));
  if (cl)
    hipLaunchKernelGGL(idwt3d_haar_kernel<true>, grid, dim3(256), lds, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(idwt3d_haar_kernel<false>, grid, dim3(256), lds, (hipStream_t)stream, a);
  return check_launch("wf_idwt3d_haar");
}

extern "C" int wf_idwt3d_haar(const float* ll, int64_t ll_bstride, const float* const* det,
                              const int64_t* det_s, int levels, float* out, int64_t out_bstride,
                              int64_t B, int64_t C, int64_t d, int64_t h, int64_t w,
                              void* stream) {
  return idwt_launch(ll, ll_bstride, d * h * w, 1, det, det_s, levels, out, out_bstride, 0, B,
                     C, d, h, w, stream);
}

extern "C" int wf_idwt3d_haar_cl(const float* ll, int64_t ll_bstride, int64_t ll_cstride,
                                 int64_t ll_pstride, const float* const* det,
                                 const int64_t* det_s, int levels, float* out,
                                 int64_t out_bstride, int64_t ldo, int64_t B, int64_t C,
                                 int64_t d, int64_t h, int64_t w, void* stream) {
  WF_REQUIRE(ldo >= C, "channel-last output: ldo must be >= C");
  WF_REQUIRE(ll_cstride >= 1 && ll_pstride >= 1, "LL strides must be positive");
  return idwt_launch(ll, ll_bstride, ll_cstride, ll_pstride, det, det_s, levels, out,
                     out_bstride, ldo, B, C, d, h, w, stream);
}

extern "C" int wf_idwt3d_haar_cl_cat(const float* ll, int64_t ll_bstride, int64_t ll_cstride,
                                     int64_t ll_pstride, const float* const* det,
                                     const int64_t* det_s, int levels, const float* skip,
                                     int64_t skip_bstride, int64_t skip_ld, float* out,
                                     int64_t out_bstride, int64_t ldo, int64_t B, int64_t C,
                                     int64_t d, int64_t h, int64_t w, void* stream) {
  WF_REQUIRE_PTR(skip);
  WF_REQUIRE(ldo >= 2 * C, "fused concat: ldo must be >= 2C");
  return idwt_launch(ll, ll_bstride, ll_cstride, ll_pstride, det, det_s, levels, out,
                     out_bstride, ldo, B, C, d, h, w, stream, skip, skip_bstride, skip_ld);
}
