// ffn_dwfc.hip -- the back half of CCF_FFN fused into one kernel for the stage-1 shape
// (C = 48, hidden = 192; the largest FFN of the encoder):
//
//   h2  = dwconv3x3x3(h1) + b          (wave_helper.py:285, groups = hidden, pad 1)
//   g   = GELU(LN_eps2(h2))            (:286-287)
//   ffn = fc(g) + fc_b                 (:289, Linear hidden -> C)
//   out = x + (n2 + ffn) * bs          (Block residual + CCF_FFN residual, quirk Q4, :293/:509)
//         with n2 = LN(x; stats, n2_w, n2_b), or out = x + ffn * bs for a bare CCF_FFN.
//
// h2 never touches HBM (the unfused path writes and re-reads 2 x 805 MB of it per stage-1
// block at B = 4).  A workgroup owns a 4 x 8 (y, x) tile and marches z through a segment of
// ZS output planes:
//   1. the haloed 6 x 10 x 192 input plane of h1 is prefetched into registers two planes
//      ahead and committed to a double-buffered LDS plane (2 x 46 KB fp32) one plane ahead;
//   2. every thread owns two channels of one x column (768 threads = 96 channel pairs x 8
//      columns; 12 waves, the register-file limit at ~160 VGPRs) and scatters each input row
//      into the three output planes it feeds (rolling
//      accumulators, packed v_pk_fma_f32 on the channel pair, the 27 weight pairs in
//      registers): 27 FMAs per output and no re-reads of a plane;
//   3. when an output plane is complete its 32 x 192 h2 tile goes to LDS (25 KB);
//      16 lanes per position take the LayerNorm statistics, apply LN2 + GELU (packed) and
//      rewrite the row in place as bf16 hi/lo halves (the split MFMA operand);
//   4. six waves run the fc GEMM as 2 position tiles x 3 output-channel tiles of
//      v_mfma_f32_16x16x32_bf16 (x3 for the fp32-faithful split), the fc weight hi/lo planes
//      staged once per workgroup in LDS, and the epilogue adds bias + the Q4 residual and
//      stores 16-byte rows.
#include "kernels.hpp"

namespace wf {

template <int C, int HID, int TY, int TX>
struct DwFcCfg {
  static constexpr int NTH = (HID / 2) * TX;        // one thread per (channel pair, column)
  static constexpr int PY = TY + 2, PX = TX + 2, PP = PY * PX;
  static constexpr int NPOS = TY * TX;
  static constexpr int HS = HID + 4;                // h2 row stride in floats (bank spread)
  static constexpr int WKP = HID + 8;               // fc weight row stride in bf16
  static constexpr int PLANE_F = PP * HID;          // input plane floats
  static constexpr int H2_F = NPOS * HS;
  static constexpr int BUF_F = 2 * PLANE_F + H2_F;  // double-buffered plane + h2 tile
  static constexpr int NV = HID / 4;                // 16-byte fp32 vectors per row
  static constexpr int NLD = (PP * NV + NTH - 1) / NTH;
  static constexpr int WAVES = NTH / 64;
  static constexpr int RT = NPOS / 16, CT = C / 16;  // fc tiles
  static constexpr int LN_LANES = 16;               // lanes per position for LN2
  static constexpr int LN_CH = HID / LN_LANES;
  static_assert(NTH % 64 == 0, "whole waves");
  static_assert(RT * CT <= WAVES, "at most one fc tile per wave");
  static_assert(NPOS * LN_LANES <= NTH, "LN2 lanes");
  static_assert(LN_CH % 4 == 0, "LN2 vector width");
  static constexpr size_t LDS_BYTES = (size_t)BUF_F * 4 + (size_t)2 * C * WKP * 2 +
                                      (size_t)(2 * HID + 3 * C) * 4;
};

template <typename T>
struct H1Load;
template <>
struct H1Load<float> {
  typedef f32x4 raw;
  static __device__ __forceinline__ raw load(const float* p, int64_t i) {
    return *reinterpret_cast<const f32x4*>(p + i);
  }
  static __device__ __forceinline__ f32x4 up(raw u) { return u; }
};
template <>
struct H1Load<uint16_t> {
  typedef bf16x4 raw;
  static __device__ __forceinline__ raw load(const uint16_t* p, int64_t i) {
    return *reinterpret_cast<const bf16x4*>(p + i);
  }
  static __device__ __forceinline__ f32x4 up(raw u) {
    return f32x4{bf2f((uint16_t)u[0]), bf2f((uint16_t)u[1]), bf2f((uint16_t)u[2]),
                 bf2f((uint16_t)u[3])};
  }
};

template <int C, int HID, int TY, int TX, int P, typename T>
__global__ __launch_bounds__((HID / 2) * TX, (TX == 4 ? 3 : 1)) void ffn_dwfc_kernel(DwFcArgs a) {
  constexpr bool SPLIT = P == PREC_SPLIT;  // P: Prec (operand kind)
  typedef DwFcCfg<C, HID, TY, TX> K;
  typedef H1Load<T> L;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* planes = lds;                                           // [2][PP][HID]
  float* h2t = lds + 2 * K::PLANE_F;                              // [NPOS][HS]
  uint16_t* wf = reinterpret_cast<uint16_t*>(lds + K::BUF_F);     // [2][C][WKP]
  float* lnw = reinterpret_cast<float*>(wf + 2 * C * K::WKP);     // [HID]
  float* lnb = lnw + HID;                                         // [HID]
  float* fcb = lnb + HID;                                         // [C]
  float* n2w = fcb + C;                                           // [C] norm2 (1, 0 if none)
  float* n2b = n2w + C;

  const int tid = threadIdx.x;
  const int wid = tid >> 6;
  const int D = a.D, H = a.H, W = a.W;

  // ---- tile of this workgroup (XCD-contiguous order: neighbouring tiles, which share halo
  // rows of h1, run on the same XCD and meet in its L2)
  const int ntx = (W + TX - 1) / TX, nty = (H + TY - 1) / TY, nzs = (D + a.ZS - 1) / a.ZS;
  const int nb = gridDim.x;
  const int xcd = blockIdx.x & 7, q8 = nb >> 3, r8 = nb & 7;
  int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
  const int xt = t % ntx;
  t /= ntx;
  const int yt = t % nty;
  t /= nty;
  const int zt = t % nzs;
  const int b = t / nzs;
  const int x0 = xt * TX, y0 = yt * TY, z0 = zt * a.ZS, z1 = min(z0 + a.ZS, D);

  // ---- per-workgroup constants into LDS
  for (int i = tid; i < 2 * C * (HID / 8); i += K::NTH) {
    const int pl = i / (C * (HID / 8)), r = i % (C * (HID / 8));
    const int n = r / (HID / 8), k8 = r % (HID / 8);
    const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    const bf16x8 v = (SPLIT || pl == 0)
                         ? *reinterpret_cast<const bf16x8*>(a.fc + ((size_t)pl * C + n) * HID + 8 * k8)
                         : z8;
    *reinterpret_cast<bf16x8*>(wf + ((size_t)pl * C + n) * K::WKP + 8 * k8) = v;
  }
  for (int i = tid; i < HID; i += K::NTH) {  // halved: GELU is evaluated from x / 2
    lnw[i] = 0.5f * a.ln2_w[i];
    lnb[i] = 0.5f * a.ln2_b[i];
  }
  // depthwise weights, coalesced into the (not yet used) plane buffer, read back per thread
  for (int i = tid; i < HID * 27; i += K::NTH) planes[i] = a.dw_w[i];
  __syncthreads();
  for (int i = tid; i < C; i += K::NTH) {
    fcb[i] = a.fc_b ? a.fc_b[i] : 0.f;
    n2w[i] = a.stats ? a.n2_w[i] : 1.f;
    n2b[i] = a.stats ? a.n2_b[i] : 0.f;
  }

  // ---- depthwise role: channel pair cp, column xi
  const int cp = tid % (HID / 2), xi = tid / (HID / 2);
  f32x2 w2[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) w2[k] = f32x2{planes[(2 * cp) * 27 + k], planes[(2 * cp + 1) * 27 + k]};
  const f32x2 bias2 = f32x2{a.dw_b[2 * cp], a.dw_b[2 * cp + 1]};

  // ---- h1 plane staging: item i -> (haloed position i / NV, 4-channel vector i % NV).  The
  // in-plane offsets and the (y, x) validity of this thread's items are fixed for the whole
  // z march; a plane is one scalar base + 32-bit offsets, the loads are unconditional (clamped)
  // and the zero padding is applied at commit time, so nothing waits on them before then.
  const T* src = reinterpret_cast<const T*>(a.h1) + (int64_t)b * D * H * W * HID;
  const int64_t plane_elems = (int64_t)H * W * HID;
  int off[K::NLD];
  unsigned okmask = 0;
#pragma unroll
  for (int j = 0; j < K::NLD; ++j) {
    const int i = min(j * K::NTH + tid, K::PP * K::NV - 1);
    const int pos = i / K::NV, v = i - pos * K::NV;
    const int yy = y0 - 1 + pos / K::PX, xx = x0 - 1 + pos % K::PX;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    const int yc = min(max(yy, 0), H - 1), xc = min(max(xx, 0), W - 1);
    off[j] = (yc * W + xc) * HID + 4 * v;
    okmask |= (ok ? 1u : 0u) << j;
  }
  typename L::raw stg[K::NLD];
  auto fetch = [&](int p) {
    const T* base = src + (int64_t)min(max(p, 0), D - 1) * plane_elems;
#pragma unroll
    for (int j = 0; j < K::NLD; ++j) stg[j] = L::load(base, off[j]);
  };
  auto commit = [&](int p, float* dst) {
    const bool pz = p >= 0 && p < D;
#pragma unroll
    for (int j = 0; j < K::NLD; ++j) {
      const int i = j * K::NTH + tid;
      const bool ok = pz && ((okmask >> j) & 1u);
      const f32x4 u = L::up(stg[j]);
      if (i < K::PP * K::NV)
        *reinterpret_cast<f32x4*>(dst + (size_t)i * 4) = ok ? u : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  const int64_t plane_sz = (int64_t)H * W;
  // Epilogue inputs (x rows + norm2 stats of the fc lane's output row), issued right after the
  // commit (whose wait they do not extend) and before the next plane's fetch (which the fc's
  // wait for them therefore does not include); the LN2 phase runs while they are in flight.
  // Every load is unconditional -- a branch join on a load in flight makes the compiler wait
  // on the spot -- so without norm2 stats the stats pointer reads x and the values are
  // discarded.
  const float* sbase = a.stats ? a.stats : a.x;
  f32x4 xr = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x2 es = f32x2{0.f, 1.f};
  auto epi_fetch = [&](int zp) {
    int ltid = tid;
    asm volatile("" : "+v"(ltid));
    const int lwid = min(ltid >> 6, K::RT * K::CT - 1);  // waves without an fc tile load tile 5
    const int lp = (lwid / K::CT) * 16 + (ltid & 15);
    const int col = (lwid % K::CT) * 16 + 4 * ((ltid >> 4) & 3);
    const int yo = min(y0 + lp / TX, H - 1), xo = min(x0 + lp % TX, W - 1);
    const int64_t gpos = (int64_t)b * D * plane_sz + (int64_t)zp * plane_sz + yo * W + xo;
    xr = *reinterpret_cast<const f32x4*>(a.x + gpos * C + col);
    es = *reinterpret_cast<const f32x2*>(sbase + 2 * gpos);
  };
  const float bs = a.bscale ? a.bscale[b] : 1.f;  // DropPath factor of this sample

  f32x2 accA[TY], accB[TY], accC[TY];
#pragma unroll
  for (int o = 0; o < TY; ++o) accA[o] = accB[o] = accC[o] = f32x2{0.f, 0.f};

  // Schedule per input plane p (3 barriers): scatter(p) | C | commit(p+1) into the other plane
  // buffer, the epilogue rows of output p and the h1 plane p+2 fetched for later, h2 tile of
  // output p-1 | A | LN2 + GELU in place | B | fc + store.  Waves without an fc tile run ahead
  // into the next plane's scatter while the fc runs.
  fetch(z0 - 1);
  __syncthreads();  // the depthwise weights are read out of the plane buffer
  commit(z0 - 1, planes);
  fetch(z0);
  __syncthreads();
  for (int p = z0 - 1; p <= z1; ++p) {
    const float* cur = planes + ((p - z0 + 1) & 1) * K::PLANE_F;
    float* nxt = planes + ((p - z0) & 1) * K::PLANE_F;
    // ---- scatter plane p into output planes p+1 (kz 0), p (kz 1), p-1 (kz 2)
    {
      const float* Pin = cur + xi * HID + 2 * cp;
#pragma unroll
      for (int r = 0; r < K::PY; ++r) {
        const f32x2 v0 = *reinterpret_cast<const f32x2*>(Pin + (r * K::PX + 0) * HID);
        const f32x2 v1 = *reinterpret_cast<const f32x2*>(Pin + (r * K::PX + 1) * HID);
        const f32x2 v2 = *reinterpret_cast<const f32x2*>(Pin + (r * K::PX + 2) * HID);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int o = r - ky;
          if (o < 0 || o >= TY) continue;
          // one packed FMA per tap into the running sum
          const f32x2* w0 = w2 + ky * 3;
          accC[o] = w0[2] * v2 + (w0[1] * v1 + (w0[0] * v0 + accC[o]));
          accB[o] = w0[11] * v2 + (w0[10] * v1 + (w0[9] * v0 + accB[o]));
          accA[o] = w0[20] * v2 + (w0[19] * v1 + (w0[18] * v0 + accA[o]));
        }
        __builtin_amdgcn_sched_barrier(0);  // one input row in flight at a time (VGPRs)
      }
    }

    const int zo = p - 1;  // output plane completed by this input plane
    __syncthreads();  // C: scatter(p) done everywhere (nxt is free), fc(p-2) done (h2t is free)
    // retire the loads issued a plane ago on every path (an empty asm "reading" them): where
    // the commit or the fc is skipped their registers would otherwise stay pending, and the
    // compiler would then drain the loads issued just below before re-using the registers
    asm volatile("" ::"v"(xr), "v"(es));
#pragma unroll
    for (int j = 0; j < K::NLD; ++j) asm volatile("" ::"v"(stg[j]));
    if (p + 1 <= z1) commit(p + 1, nxt);
    if (zo >= z0) epi_fetch(zo);
    if (p + 2 <= z1) fetch(p + 2);  // in flight behind the next plane's work
    if (zo >= z0) {
      // ---- h2 tile (+ bias) into LDS: row = position o * TX + xi
#pragma unroll
      for (int o = 0; o < TY; ++o) {
        f32x2 h = accA[o] + bias2;
        if (sizeof(T) == 2) {  // bf16 mode: h2 carries bf16 rounding like the stored path
          h.x = bf2f(f2bf(h.x));
          h.y = bf2f(f2bf(h.y));
        }
        *reinterpret_cast<f32x2*>(h2t + (o * TX + xi) * K::HS + 2 * cp) = h;
      }
    }
    __syncthreads();  // A: h2 tile and plane p+1 visible
    if (zo >= z0) {
      // ---- LN2 + GELU per position, rewritten in place as bf16 {hi[HID], lo[HID]}
      // Loop-invariant per-lane values of the LN2 and epilogue phases are recomputed from a
      // laundered thread index every plane: hoisted out of the z loop they exceed the
      // 168-VGPR budget and spill.
      int ltid = tid;
      asm volatile("" : "+v"(ltid));
      if (ltid < K::NPOS * K::LN_LANES) {
        const int pos = ltid / K::LN_LANES, g = ltid % K::LN_LANES;
        float* row = h2t + pos * K::HS;
        float v[K::LN_CH];
#pragma unroll
        for (int j = 0; j < K::LN_CH / 4; ++j) {
          const f32x4 u = *reinterpret_cast<const f32x4*>(row + g * K::LN_CH + 4 * j);
          v[4 * j] = u.x;
          v[4 * j + 1] = u.y;
          v[4 * j + 2] = u.z;
          v[4 * j + 3] = u.w;
        }
        float sm = 0.f;
#pragma unroll
        for (int j = 0; j < K::LN_CH; ++j) sm += v[j];
        const float mean = group_sum<K::LN_LANES>(sm) * (1.f / HID);
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < K::LN_CH; ++j) {
          const float d = v[j] - mean;
          q += d * d;
        }
        const float rstd = rsqrtf(group_sum<K::LN_LANES>(q) * (1.f / HID) + a.eps2);
        const float nmr = -mean * rstd;
        uint16_t* rowh = reinterpret_cast<uint16_t*>(row);
#pragma unroll
        for (int j = 0; j < K::LN_CH / 4; ++j) {
          const int c = g * K::LN_CH + 4 * j;
          const f32x4 lw4 = *reinterpret_cast<const f32x4*>(lnw + c);
          const f32x4 lb4 = *reinterpret_cast<const f32x4*>(lnb + c);
          const f32x4 y = gelu_half4((f32x4{v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]} *
                                      rstd + nmr) * lw4 + lb4);
          bf16x4 hi4, lo4;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint16_t hb = op_cvt<P>(y[e]);
            hi4[e] = (short)hb;
            lo4[e] = op_lo<P>(y[e], hb);
          }
          *reinterpret_cast<bf16x4*>(rowh + c) = hi4;
          if (SPLIT) *reinterpret_cast<bf16x4*>(rowh + HID + c) = lo4;
        }
      }
      const int lln = ltid & 63, lwid = ltid >> 6;
      const int ct = lwid % K::CT, l15 = lln & 15, g4 = lln >> 4;  // fc tile of this wave
      const int lp = (lwid / K::CT) * 16 + l15;  // tile position of this lane's row
      const int yo = y0 + lp / TX, xo = x0 + lp % TX;
      const bool rv = yo < H && xo < W;
      const int64_t gpos = (int64_t)b * D * plane_sz + (int64_t)zo * plane_sz +
                           (int64_t)min(yo, H - 1) * W + min(xo, W - 1);
      const int col = ct * 16 + 4 * g4;
      const bool fcw = wid < K::RT * K::CT;  // this wave owns an fc tile
      __syncthreads();  // B: LN2 + GELU rows visible
      // ---- fc GEMM (waves 0 .. RT*CT-1): acc[i] = ffn[position lp][channel col + i]
      if (fcw) {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        const uint16_t* Bh = reinterpret_cast<const uint16_t*>(h2t) + (size_t)lp * (2 * K::HS);
        const uint16_t* Wh = wf + (size_t)(ct * 16 + l15) * K::WKP;
#pragma unroll
        for (int ks = 0; ks < HID / 32; ++ks) {
          const int k = ks * 32 + 8 * g4;
          const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Bh + k);
          const bf16x8 wh = *reinterpret_cast<const bf16x8*>(Wh + k);
          if (SPLIT) {
            const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Bh + HID + k);
            const bf16x8 wl = *reinterpret_cast<const bf16x8*>(Wh + C * K::WKP + k);
            acc = mma32<P>(wh, bl, acc);
            acc = mma32<P>(wl, bh, acc);
          }
          acc = mma32<P>(wh, bh, acc);
        }
        // ---- epilogue: bias + Q4 residual, 16-byte store
        f32x4 v = acc + *reinterpret_cast<const f32x4*>(fcb + col);
        if (a.stats) {
          const f32x4 lw = *reinterpret_cast<const f32x4*>(n2w + col);
          const f32x4 lb = *reinterpret_cast<const f32x4*>(n2b + col);
          const f32x4 n2 = (xr - es.x) * es.y * lw + lb;
          v = xr + (n2 + v) * bs;
        } else {
          v = xr + v * bs;
        }
        if (rv) *reinterpret_cast<f32x4*>(a.out + gpos * C + col) = v;
      }
    }
#pragma unroll
    for (int o = 0; o < TY; ++o) {
      accA[o] = accB[o];
      accB[o] = accC[o];
      accC[o] = f32x2{0.f, 0.f};
    }
  }
}

// ---------------------------------------------------------------------------------------
// Wave-specialised variant (same math, same tile): 6 "D" waves run the depthwise scatter while
// 6 "E" waves run everything else one output plane behind -- LN2 + GELU + split of plane z-2,
// its fc MFMAs and store, the staging of the next h1 plane -- so the two VALU-heavy phases
// overlap instead of taking turns between barriers.  Per input plane p, two barriers:
//   phase 1:  D  scatter rows 0..1 of plane p
//             E  epilogue rows of z = p-2, LN2 + GELU of h2 tile (p-2) in place (waves 6..9:
//                8 lanes x 24 channels)
//   phase 2:  D  scatter rows 2..5 of plane p -> output plane p-1 complete -> h2 tile (p-1)
//             E  commit plane p+1, fetch plane p+2, fc GEMM of tile (p-2) (6 waves: 2 row x
//                3 column tiles, weights in VGPRs) + bias + Q4 residual + store
// h2 tiles are double-buffered ((p-1) is written while (p-2) is read); 144 KB of LDS (the fc
// weights live in the E waves' registers instead).
// ---------------------------------------------------------------------------------------
template <int P, typename T>
__global__ __launch_bounds__(768, 1) void ffn_dwfc_ws_kernel(DwFcArgs a) {
  constexpr int C = 48, HID = 192, TY = 4, TX = 8;
  constexpr bool SPLIT = P == PREC_SPLIT;
  typedef DwFcCfg<C, HID, TY, TX> K;
  typedef H1Load<T> L;
  constexpr int NPAIR = HID / 2;                  // 96 channel pairs
  constexpr int NE = 384;                         // E threads
  constexpr int NLDE = (K::PP * K::NV + NE - 1) / NE;  // staged f32x4 per E thread (8)
  constexpr int H2F = K::NPOS * K::HS;            // one h2 tile (floats)
  // LN2 + GELU of an h2 tile: 16 lanes x 12 channels per position; positions 0..15 by the D
  // waves 0..3 in their phase 1 (they idle there otherwise: per plane the D waves' scatter is
  // ~2.8k cycles of work against ~5.3k for the E waves, measured with s_memtime probes),
  // positions 16..31 by the E waves 0..3
  constexpr int LNL = 16, LNC = HID / LNL;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* planes = lds;                                  // [2][PP][HID]
  float* h2b = lds + 2 * K::PLANE_F;                     // [2][NPOS][HS]
  float* lnw = h2b + 2 * H2F;                            // [HID] (halved: GELU from x / 2)
  float* lnb = lnw + HID;
  float* fcb = lnb + HID;                                // [C]
  float* n2w = fcb + C;
  float* n2b = n2w + C;

  const int tid = threadIdx.x;
  const int wid = tid >> 6;
  const bool isD = wid < 6;
  const int D = a.D, H = a.H, W = a.W;
  const int ntx = (W + TX - 1) / TX, nty = (H + TY - 1) / TY, nzs = (D + a.ZS - 1) / a.ZS;
  const int nb = gridDim.x;
  const int xcd = blockIdx.x & 7, q8 = nb >> 3, r8 = nb & 7;
  int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
  const int xt = t % ntx;
  t /= ntx;
  const int yt = t % nty;
  t /= nty;
  const int zt = t % nzs;
  const int b = t / nzs;
  const int x0 = xt * TX, y0 = yt * TY, z0 = zt * a.ZS, z1 = min(z0 + a.ZS, D);
  const int64_t plane_sz = (int64_t)H * W;

  for (int i = tid; i < HID; i += K::NTH) {
    lnw[i] = 0.5f * a.ln2_w[i];
    lnb[i] = 0.5f * a.ln2_b[i];
  }
  for (int i = tid; i < C; i += K::NTH) {
    fcb[i] = a.fc_b ? a.fc_b[i] : 0.f;
    n2w[i] = a.stats ? a.n2_w[i] : 1.f;
    n2b[i] = a.stats ? a.n2_b[i] : 0.f;
  }
  // depthwise weights, coalesced into the (not yet used) plane buffer
  for (int i = tid; i < HID * 27; i += K::NTH) planes[i] = a.dw_w[i];
  __syncthreads();

  const T* src = reinterpret_cast<const T*>(a.h1) + (int64_t)b * D * H * W * HID;
  const int64_t plane_elems = (int64_t)H * W * HID;
  const float bs = a.bscale ? a.bscale[b] : 1.f;

  // LN2 + GELU + the bf16 hi / lo split of one h2 tile row, rewritten in place (the row's
  // lanes are one 16-lane group of a wave: all reads precede the cross-lane reductions, which
  // precede every write)
  auto ln2_row = [&](float* h2t, int pos, int g) {
    float* row = h2t + pos * K::HS;
    float v[LNC];
#pragma unroll
    for (int j = 0; j < LNC / 4; ++j) {
      const f32x4 u = *reinterpret_cast<const f32x4*>(row + g * LNC + 4 * j);
      v[4 * j] = u.x;
      v[4 * j + 1] = u.y;
      v[4 * j + 2] = u.z;
      v[4 * j + 3] = u.w;
    }
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < LNC; ++j) sm += v[j];
    const float mean = group_sum<LNL>(sm) * (1.f / HID);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < LNC; ++j) {
      const float d = v[j] - mean;
      q += d * d;
    }
    const float rstd = rsqrtf(group_sum<LNL>(q) * (1.f / HID) + a.eps2);
    const float nmr = -mean * rstd;
    uint16_t* rowh = reinterpret_cast<uint16_t*>(row);
#pragma unroll
    for (int j = 0; j < LNC / 4; ++j) {
      const int c = g * LNC + 4 * j;
      const f32x4 lw4 = *reinterpret_cast<const f32x4*>(lnw + c);
      const f32x4 lb4 = *reinterpret_cast<const f32x4*>(lnb + c);
      const f32x4 y = gelu_half4((f32x4{v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]} *
                                  rstd + nmr) * lw4 + lb4);
      bf16x4 hi4, lo4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint16_t hb = op_cvt<P>(y[e]);
        hi4[e] = (short)hb;
        lo4[e] = op_lo<P>(y[e], hb);
      }
      *reinterpret_cast<bf16x4*>(rowh + c) = hi4;
      if (SPLIT) *reinterpret_cast<bf16x4*>(rowh + HID + c) = lo4;
    }
  };

  if (isD) {
    // ================================ D waves: depthwise scatter ==========================
    const int cp = tid % NPAIR, xg = tid / NPAIR;  // columns xg and xg + 4
    f32x2 w2[27];
#pragma unroll
    for (int k = 0; k < 27; ++k)
      w2[k] = f32x2{planes[(2 * cp) * 27 + k], planes[(2 * cp + 1) * 27 + k]};
    const f32x2 bias2 = f32x2{a.dw_b[2 * cp], a.dw_b[2 * cp + 1]};
    f32x2 aA[2][TY], aB[2][TY], aC[2][TY];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int o = 0; o < TY; ++o) aA[c][o] = aB[c][o] = aC[c][o] = f32x2{0.f, 0.f};
    __syncthreads();  // (prologue) weights read out of the plane buffer
    __syncthreads();  // (prologue) planes z0-1 committed
    auto rows = [&](const float* cur, int r_lo, int r_hi) {
#pragma unroll
      for (int r = 0; r < K::PY; ++r) {
        if (r < r_lo || r >= r_hi) continue;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const float* Pin = cur + (xg + 4 * c) * HID + 2 * cp;
          const f32x2 v0 = *reinterpret_cast<const f32x2*>(Pin + (r * K::PX + 0) * HID);
          const f32x2 v1 = *reinterpret_cast<const f32x2*>(Pin + (r * K::PX + 1) * HID);
          const f32x2 v2 = *reinterpret_cast<const f32x2*>(Pin + (r * K::PX + 2) * HID);
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) {
            const int o = r - ky;
            if (o < 0 || o >= TY) continue;
            const f32x2* w0 = w2 + ky * 3;
            aC[c][o] = w0[2] * v2 + (w0[1] * v1 + (w0[0] * v0 + aC[c][o]));
            aB[c][o] = w0[11] * v2 + (w0[10] * v1 + (w0[9] * v0 + aB[c][o]));
            aA[c][o] = w0[20] * v2 + (w0[19] * v1 + (w0[18] * v0 + aA[c][o]));
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // one input row in flight at a time (VGPRs)
      }
    };
    for (int p = z0 - 1; p <= z1 + 1; ++p) {
      const bool live = p <= z1;
      const float* cur = planes + ((p - z0 + 1) & 1) * K::PLANE_F;
      const bool dscat = !(a.dbg & 1);  // timing experiments only (WF_FFN_DBG)
      const int zl = p - 2;  // the h2 tile the E waves' fc takes in this iteration
      if (zl >= z0 && zl < z1 && tid < 16 * LNL && !(a.dbg & 2)) {
        int ltid = tid;
        asm volatile("" : "+v"(ltid));
        ln2_row(h2b + ((zl - z0) & 1) * H2F, ltid / LNL, ltid % LNL);
      }
      if (live && dscat) rows(cur, 0, a.ws_split);
      __syncthreads();  // 1 -> 2
      if (live) {
        if (dscat) rows(cur, a.ws_split, K::PY);
        const int zo = p - 1;
        if (zo >= z0) {
          float* h2t = h2b + ((zo - z0) & 1) * H2F;
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int o = 0; o < TY; ++o) {
              f32x2 h = aA[c][o] + bias2;
              if (sizeof(T) == 2) {
                h.x = bf2f(f2bf(h.x));
                h.y = bf2f(f2bf(h.y));
              }
              *reinterpret_cast<f32x2*>(h2t + (o * TX + xg + 4 * c) * K::HS + 2 * cp) = h;
            }
        }
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int o = 0; o < TY; ++o) {
            aA[c][o] = aB[c][o];
            aB[c][o] = aC[c][o];
            aC[c][o] = f32x2{0.f, 0.f};
          }
      }
      __syncthreads();  // 2 -> next 1
    }
    return;
  }

  // ================================== E waves ============================================
  const int et = tid - NE, ewid = et >> 6, eln = et & 63;
  const int l15 = eln & 15, g4 = eln >> 4;
  const int rt = ewid / 3, ct = ewid % 3;  // fc tile of this wave
  // fc weights in registers: A operand rows ct*16 + l15, k = ks*32 + 8 g4
  bf16x8 fwh[HID / 32], fwl[HID / 32];
  {
    const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint16_t* wr = a.fc + (size_t)(ct * 16 + l15) * HID + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < HID / 32; ++ks) {
      fwh[ks] = *reinterpret_cast<const bf16x8*>(wr + ks * 32);
      fwl[ks] = SPLIT ? *reinterpret_cast<const bf16x8*>(wr + (size_t)C * HID + ks * 32) : z8;
    }
  }
  // h1 plane staging: item j -> (haloed position, 4-channel vector); offsets fixed per tile
  int off[NLDE];
  unsigned okmask = 0;
#pragma unroll
  for (int j = 0; j < NLDE; ++j) {
    const int i = min(j * NE + et, K::PP * K::NV - 1);
    const int pos = i / K::NV, v = i - pos * K::NV;
    const int yy = y0 - 1 + pos / K::PX, xx = x0 - 1 + pos % K::PX;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    const int yc = min(max(yy, 0), H - 1), xc = min(max(xx, 0), W - 1);
    off[j] = (yc * W + xc) * HID + 4 * v;
    okmask |= (ok ? 1u : 0u) << j;
  }
  typename L::raw stg[NLDE];
  auto fetch = [&](int p) {
    const T* base = src + (int64_t)min(max(p, 0), D - 1) * plane_elems;
#pragma unroll
    for (int j = 0; j < NLDE; ++j) stg[j] = L::load(base, off[j]);
  };
  auto commit = [&](int p, float* dst) {
    const bool pz = p >= 0 && p < D;
#pragma unroll
    for (int j = 0; j < NLDE; ++j) {
      const int i = j * NE + et;
      const bool ok = pz && ((okmask >> j) & 1u);
      const f32x4 u = L::up(stg[j]);
      if (i < K::PP * K::NV)
        *reinterpret_cast<f32x4*>(dst + (size_t)i * 4) = ok ? u : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  const int lp = rt * 16 + l15;              // tile position of this lane's fc row
  const int yo = y0 + lp / TX, xo = x0 + lp % TX;
  const bool rv = yo < H && xo < W;
  const int col = ct * 16 + 4 * g4;
  const float* sbase = a.stats ? a.stats : a.x;
  f32x4 xr = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x2 es = f32x2{0.f, 1.f};

  fetch(z0 - 1);
  __syncthreads();  // (prologue) weights read out of the plane buffer
  commit(z0 - 1, planes);
  fetch(z0);
  __syncthreads();  // (prologue) plane z0-1 visible
  for (int p = z0 - 1; p <= z1 + 1; ++p) {
    const int zo = p - 2;  // output plane this iteration finishes
    const bool epi = zo >= z0 && zo < z1;
    // ---- phase 1: epilogue rows of plane p-2, LN2 + GELU of its h2 tile
    asm volatile("" ::"v"(xr), "v"(es));
    if (epi) {
      const int64_t gpos = (int64_t)b * D * plane_sz + (int64_t)zo * plane_sz +
                           (int64_t)min(yo, H - 1) * W + min(xo, W - 1);
      xr = *reinterpret_cast<const f32x4*>(a.x + gpos * C + col);
      es = *reinterpret_cast<const f32x2*>(sbase + 2 * gpos);
    }
    float* h2t = h2b + ((zo - z0) & 1) * H2F;
    if (epi && ewid < 4 && !(a.dbg & 2)) {
      int ltid = et;
      asm volatile("" : "+v"(ltid));
      ln2_row(h2t, 16 + ltid / LNL, ltid % LNL);
    }
    __syncthreads();  // 1 -> 2: LN rows of tile (p-2) visible
    // ---- phase 2: commit plane p+1 into the free buffer (D is done with plane p-1 since the
    // last barrier of iteration p-1), fetch p+2, fc GEMM of tile (p-2) + residual + store
#pragma unroll
    for (int j = 0; j < NLDE; ++j) asm volatile("" ::"v"(stg[j]));
    if (p + 1 <= z1 && !(a.dbg & 8)) commit(p + 1, planes + ((p - z0) & 1) * K::PLANE_F);
    if (p + 2 <= z1 && !(a.dbg & 8)) fetch(p + 2);
    if (epi && !(a.dbg & 4)) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      const uint16_t* Bh = reinterpret_cast<const uint16_t*>(h2t) + (size_t)lp * (2 * K::HS);
#pragma unroll
      for (int ks = 0; ks < HID / 32; ++ks) {
        const int k = ks * 32 + 8 * g4;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Bh + k);
        if (SPLIT) {
          const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Bh + HID + k);
          acc = mma32<P>(fwh[ks], bl, acc);
          acc = mma32<P>(fwl[ks], bh, acc);
        }
        acc = mma32<P>(fwh[ks], bh, acc);
      }
      f32x4 v = acc + *reinterpret_cast<const f32x4*>(fcb + col);
      if (a.stats) {
        const f32x4 lw = *reinterpret_cast<const f32x4*>(n2w + col);
        const f32x4 lb = *reinterpret_cast<const f32x4*>(n2b + col);
        const f32x4 n2 = (xr - es.x) * es.y * lw + lb;
        v = xr + (n2 + v) * bs;
      } else {
        v = xr + v * bs;
      }
      if (rv) {
        const int64_t gpos = (int64_t)b * D * plane_sz + (int64_t)zo * plane_sz +
                             (int64_t)yo * W + xo;
        *reinterpret_cast<f32x4*>(a.out + gpos * C + col) = v;
      }
    }
    __syncthreads();  // 2 -> next 1
  }
}

template <int TY, int TX>
static int go_dwfc(const DwFcArgs& a, int prec, hipStream_t s, int min_blocks) {
  constexpr int C = 48, HID = 192;
  typedef DwFcCfg<C, HID, TY, TX> K;
  DwFcArgs g = a;
  // z segment: enough workgroups for a few rounds over the CUs, but long enough that the two
  // halo planes per segment stay a small overhead
  const int64_t base = (int64_t)g.B * cdiv(g.H, TY) * cdiv(g.W, TX);
  int ZS = g.D;
  while (ZS > 8 && base * cdiv(g.D, ZS) < min_blocks) ZS = (ZS + 1) / 2;
  g.ZS = ZS;
  const int64_t blocks = base * cdiv(g.D, ZS);
  void (*kern)(DwFcArgs) = prec == PREC_SPLIT ? ffn_dwfc_kernel<C, HID, TY, TX, PREC_SPLIT, float>
                           : prec == PREC_FP16 ? ffn_dwfc_kernel<C, HID, TY, TX, PREC_FP16, float>
                                               : ffn_dwfc_kernel<C, HID, TY, TX, PREC_BF16, uint16_t>;
  set_max_lds(reinterpret_cast<const void*>(kern), (int)K::LDS_BYTES);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(K::NTH), K::LDS_BYTES, s, g);
  return check_launch("ffn_dwfc");
}

static int go_dwfc_ws(const DwFcArgs& a, int prec, hipStream_t s, int min_blocks) {
  constexpr int C = 48, HID = 192, TY = 4, TX = 8;
  typedef DwFcCfg<C, HID, TY, TX> K;
  DwFcArgs g = a;
  const int64_t base = (int64_t)g.B * cdiv(g.H, TY) * cdiv(g.W, TX);
  int ZS = g.D;
  while (ZS > 8 && base * cdiv(g.D, ZS) < min_blocks) ZS = (ZS + 1) / 2;
  g.ZS = ZS;
  const int64_t blocks = base * cdiv(g.D, ZS);
  const size_t lds = (size_t)(2 * K::PLANE_F + 2 * K::H2_F + 2 * HID + 3 * C) * 4;
  // D's input rows split over the two phases: rows 0..1 (3 of the 12 row-tap FMA groups)
  // alongside E's LN2 + GELU, rows 2..5 alongside E's commit + fetch + fc (B = 8 stage 1,
  // split 0..5: 916, 894, 879-888, 903, 934, 952 us; the classic kernel 1072 us)
  static const int split = getenv("WF_FFN_WS_SPLIT") ? atoi(getenv("WF_FFN_WS_SPLIT")) : 2;
  g.ws_split = split;
  static const int dbg = getenv("WF_FFN_DBG") ? atoi(getenv("WF_FFN_DBG")) : 0;
  g.dbg = dbg;  // timing experiments only: bit mask of phases skipped (results invalid)
  void (*kern)(DwFcArgs) = prec == PREC_SPLIT  ? ffn_dwfc_ws_kernel<PREC_SPLIT, float>
                           : prec == PREC_FP16 ? ffn_dwfc_ws_kernel<PREC_FP16, float>
                                               : ffn_dwfc_ws_kernel<PREC_BF16, uint16_t>;
  set_max_lds(reinterpret_cast<const void*>(kern), (int)lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(K::NTH), lds, s, g);
  return check_launch("ffn_dwfc_ws");
}

int launch_ffn_dwfc(const DwFcArgs& a, int prec, hipStream_t s) {
  // 4 x 8 tiles: 12 waves (the register-file limit at ~168 VGPRs) and ~154 KB of LDS, one
  // workgroup per CU.  (4 x 4 tiles with two 6-wave workgroups per CU measured 1.5x slower.)
  // Default: the wave-specialised kernel (947 vs 1072 us per stage-1 launch at B = 8);
  // WF_FFN_DWFC_CLASSIC=1 selects the all-waves-in-lockstep original for A/B
  static const bool classic = getenv("WF_FFN_DWFC_CLASSIC") != nullptr;
  if (!classic) return go_dwfc_ws(a, prec, s, 1024);
  return go_dwfc<4, 8>(a, prec, s, 1024);
}

}  // namespace wf
