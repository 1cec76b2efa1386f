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
//      accumulators, f32x2 FMAs on the channel pair (two v_fma_f32: no packed FP32 in this
//      build), the 27 weight pairs in
//      registers): 27 FMAs per output and no re-reads of a plane;
//   3. when an output plane is complete its 32 x 192 h2 tile goes to LDS (25 KB);
//      16 lanes per position take the LayerNorm statistics, apply LN2 + GELU (f32x2 pairs) and
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
          // one pair FMA per tap into the running sum
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

#ifdef WF_DWFC2_PROBE
// diagnostic builds only (ffn_dwfc_ws_kernel and ffn_dwfc2_kernel): per-wave cycles of
// workgroup 0 by phase between the kernel's barriers (work, then wait), read back by
// wf_debug_dwfc2_probe
__device__ long long g_dwfc2_probe[12 * 8];
extern "C" int wf_debug_dwfc2_probe(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dwfc2_probe), sizeof(g_dwfc2_probe));
}
#define PROBE_DECL                                                              \
  const bool probe_on = blockIdx.x == 0;                                         \
  long long pr_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pr_last = __builtin_amdgcn_s_memtime();
#define PROBE(i)                                                                \
  if (probe_on) {                                                               \
    const long long t_ = __builtin_amdgcn_s_memtime();                          \
    pr_acc[i] += t_ - pr_last;                                                  \
    pr_last = t_;                                                               \
  }
#define PROBE_DUMP                                                              \
  if (probe_on && (tid & 63) == 0)                                              \
    for (int i_ = 0; i_ < 8; ++i_) g_dwfc2_probe[wid * 8 + i_] = pr_acc[i_];
#else
#define PROBE_DECL
#define PROBE(i)
#define PROBE_DUMP
#endif

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
  // D's input rows split over the two phases: rows 0..1 (3 of the 12 row-tap FMA groups)
  // alongside E's LN2 + GELU, rows 2..5 alongside E's commit + fetch + fc (B = 8 stage 1,
  // split 0..5 measured 916, 894, 879-888, 903, 934, 952 us in round 2)
  constexpr int WS_SPLIT = 2;
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

  PROBE_DECL
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
    // input rows [r_lo, r_hi) (compile-time after inlining) of plane cur; each row's six LDS
    // reads are issued one row ahead of its FMAs, and unconditionally (a load pending across a
    // branch join is waited for at the join)
    auto rows = [&](const float* cur, int r_lo, int r_hi) {
      f32x2 nx[2][3];
      auto ld = [&](int r) {
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int k = 0; k < 3; ++k)
            nx[c][k] = *reinterpret_cast<const f32x2*>(cur + (xg + 4 * c) * HID + 2 * cp +
                                                       (r * K::PX + k) * HID);
      };
      ld(r_lo);
#pragma unroll
      for (int r = 0; r < K::PY; ++r) {
        if (r < r_lo || r >= r_hi) continue;
        f32x2 v[2][3];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int k = 0; k < 3; ++k) v[c][k] = nx[c][k];
        if (r + 1 < r_hi) ld(r + 1);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) {
            const int o = r - ky;
            if (o < 0 || o >= TY) continue;
            const f32x2* w0 = w2 + ky * 3;
            aC[c][o] = w0[2] * v[c][2] + (w0[1] * v[c][1] + (w0[0] * v[c][0] + aC[c][o]));
            aB[c][o] = w0[11] * v[c][2] + (w0[10] * v[c][1] + (w0[9] * v[c][0] + aB[c][o]));
            aA[c][o] = w0[20] * v[c][2] + (w0[19] * v[c][1] + (w0[18] * v[c][0] + aA[c][o]));
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // rows stay in order (VGPRs)
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
      if (live && dscat) rows(cur, 0, WS_SPLIT);
      PROBE(0)
      __syncthreads();  // 1 -> 2
      PROBE(1)
      if (live) {
        if (dscat) rows(cur, WS_SPLIT, K::PY);
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
      PROBE(2)
      __syncthreads();  // 2 -> next 1
      PROBE(3)
    }
    PROBE_DUMP
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
    PROBE(0)
    __syncthreads();  // 1 -> 2: LN rows of tile (p-2) visible
    PROBE(1)
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
    PROBE(2)
    __syncthreads();  // 2 -> next 1
    PROBE(3)
  }
  PROBE_DUMP
}

// ---------------------------------------------------------------------------------------
// SIMD-balanced variant (round 3, the default): the same tile, planes and h2 tiles, but the
// 12 waves get roles per SIMD so every SIMD carries the same VALU load -- the kernel is
// VALU-issue-bound (s_memtime probes: each SIMD's VALU saturated, ~4 cycles per instruction),
// and in ffn_dwfc_ws SIMDs 0/1 held two scatter waves + an LN2 wave against one on SIMDs 2/3:
//   on each SIMD, 2 "D" waves: LN2 + GELU + split of 4 of the 32 tile positions each (16
//        lanes x 12 channels per position), then the depthwise scatter of one tile column
//        (lane l owns channels l, l + 64 and l + 128: consecutive lanes read consecutive LDS
//        words; 27 weights per channel in VGPRs, LDS reads one row ahead, rolling
//        output-plane accumulators);
//   and 1 "E" wave: the h1 plane staging (fetch two planes ahead, commit one ahead) and the fc
//        of one 16-channel output column tile over both 16-position row tiles (weights hi in
//        VGPRs, lo in LDS; the E wave of the fourth SIMD has no fc tile) + bias + Q4 residual
//        + store.
// LN2 stays on the D waves: on a lone wave (the E wave) its dependent chains (reductions,
// transcendentals) ran latency-bound, ~2x slower than interleaved over two waves per SIMD.
// The E wave runs at raised priority: it is the youngest wave on its SIMD, and without it its
// few VALU instructions waited behind the two D waves' streams (probe: fc + staging took
// 3.3-3.5k cycles per plane against 1.9-2.4k for the scatter).
// Roles are taken from the wave's SIMD (HW_ID), first come first served, so the balance does
// not depend on how the dispatcher places waves; if a SIMD did not get exactly three waves the
// roles fall back to wave-id order (still correct, just unbalanced).
// Per input plane p, two barriers:
//   phase 1: D  LN2 of h2 tile (p-2); scatter rows [0, SB_SPLIT) of plane p
//            E  residual / norm2-statistics rows of output plane p-2
//   phase 2: D  scatter rows [SB_SPLIT, 6) of plane p -> output plane p-1 -> h2 tile (p-1)
//            E  commit plane p+1, fetch plane p+2, fc of tile (p-2) + epilogue + store
// The plane loop is unrolled by three so the rolling accumulators are renamed, not moved, and
// each output plane's first contribution assigns instead of accumulating.
//
// Measured at B = 8 (tools/gpu_ab3.sh, one box, three rounds): 1047-1055 us against
// 1056-1071 for ffn_dwfc_ws.  s_memtime probes put every SIMD's VALU ~86 % busy: the kernel is
// bound by FP32 VALU work (27 depthwise FMAs + ~25 for LN2 / GELU / split per element).  A
// build with packed-FP32 scatter and LN2 (the D waves read only LDS, so the packed-op hazard
// of DESIGN.md 6.1 could not apply) measured 1058-1066 us: v_pk_fma_f32 costs the issue time
// of two v_fma_f32 here, so it is not used.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int hw_simd_id() {
  // HW_ID (hwreg 4) bits [5:4]: the SIMD the wave runs on
  return (int)((__builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4)) & 3);
}

template <int P, typename T>
__global__ __launch_bounds__(768, 1) void ffn_dwfc_sb_kernel(DwFcArgs a) {
  constexpr int C = 48, HID = 192, TY = 4, TX = 8;
  constexpr bool SPLIT = P == PREC_SPLIT;
  typedef DwFcCfg<C, HID, TY, TX> K;
  typedef H1Load<T> L;
  constexpr int NE = 256;                              // E threads (4 waves)
  constexpr int NLDE = (K::PP * K::NV + NE - 1) / NE;  // staged vectors per E thread (12)
  constexpr int H2F = K::NPOS * K::HS;
  constexpr int LNL = 16, LNC = HID / LNL;             // LN2: 16 lanes x 12 channels / position
#ifndef WF_SB_LN2T  // LN2 statistics by short chains (round 4: 1009-1012 vs 1020-1027 us)
#define WF_SB_LN2T 1
#endif
#ifndef WF_SB_SPLIT
#define WF_SB_SPLIT 0
#endif
  constexpr int SB_SPLIT = WF_SB_SPLIT;                // D rows scattered in phase 1
  static_assert(TX == 8 && K::NPOS == 32 && HID == 3 * 64, "8 D waves = 8 tile columns");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* planes = lds;                                  // [2][PP][HID]
  float* h2b = lds + 2 * K::PLANE_F;                     // [2][NPOS][HS]
  float* lnw = h2b + 2 * H2F;                            // [HID] (halved: GELU from x / 2)
  float* lnb = lnw + HID;
  float* fcb = lnb + HID;                                // [C]
  float* n2w = fcb + C;
  float* n2b = n2w + C;
  // fc weight lo plane [C][HID] bf16 (the E waves keep only the hi plane in VGPRs)
  uint16_t* fwlo = reinterpret_cast<uint16_t*>(n2b + C);
  __shared__ int simd_cnt[4];

  const int tid = threadIdx.x;
  const int wid = tid >> 6, lane = tid & 63;
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

  if (tid < 4) simd_cnt[tid] = 0;
  for (int i = tid; i < HID; i += K::NTH) {
    lnw[i] = 0.5f * a.ln2_w[i];
    lnb[i] = 0.5f * a.ln2_b[i];
  }
  for (int i = tid; i < C; i += K::NTH) {
    fcb[i] = a.fc_b ? a.fc_b[i] : 0.f;
    n2w[i] = a.stats ? a.n2_w[i] : 1.f;
    n2b[i] = a.stats ? a.n2_b[i] : 0.f;
  }
  if (SPLIT)
    for (int i = tid; i < C * HID / 8; i += K::NTH)
      reinterpret_cast<bf16x8*>(fwlo)[i] = reinterpret_cast<const bf16x8*>(a.fc + C * HID)[i];
  // depthwise weights and bias, coalesced into the (not yet used) plane buffer
  for (int i = tid; i < HID * 27; i += K::NTH) planes[i] = a.dw_w[i];
  for (int i = tid; i < HID; i += K::NTH) planes[HID * 27 + i] = a.dw_b[i];
  __syncthreads();
  // ---- roles: per SIMD, arrival slots 0, 1 -> D waves 2 s, 2 s + 1; slot 2 -> E wave s
  const int simd = hw_simd_id();
  int slot = 0;
  if (lane == 0) slot = atomicAdd(&simd_cnt[simd], 1);
  slot = __builtin_amdgcn_readfirstlane(__shfl(slot, 0, 64));
  __syncthreads();
  const bool even = simd_cnt[0] == 3 && simd_cnt[1] == 3 && simd_cnt[2] == 3 && simd_cnt[3] == 3;
  int role = even ? (slot < 2 ? 2 * simd + slot : 8 + simd) : wid;  // 0..7 D, 8..11 E
  role = __builtin_amdgcn_readfirstlane(role);

  // LN2 + GELU + the bf16 hi / lo split of one h2 tile row, rewritten in place (16 lanes)
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
#if WF_SB_LN2T
    // short dependency chains: three-way column sums (depth 3 + 2 instead of 12), four
    // variance partials, the raw v_rsq_f32 (var + eps >= eps is a normal number)
    float s4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) s4[j] = (v[j] + v[j + 4]) + v[j + 8];
    const float mean = group_sum<LNL>((s4[0] + s4[1]) + (s4[2] + s4[3])) * (1.f / HID);
    float q4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d0 = v[j] - mean, d1 = v[j + 4] - mean, d2 = v[j + 8] - mean;
      q4[j] = d2 * d2 + (d1 * d1 + d0 * d0);
    }
    const float rstd = __builtin_amdgcn_rsqf(
        group_sum<LNL>((q4[0] + q4[1]) + (q4[2] + q4[3])) * (1.f / HID) + a.eps2);
#else
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
#endif
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
      for (int k = 0; k < 4; ++k) {
        const uint16_t hb = op_cvt<P>(y[k]);
        hi4[k] = (short)hb;
        lo4[k] = op_lo<P>(y[k], hb);
      }
      *reinterpret_cast<bf16x4*>(rowh + c) = hi4;
      if (SPLIT) *reinterpret_cast<bf16x4*>(rowh + HID + c) = lo4;
    }
  };

  PROBE_DECL
#ifdef WF_DWFC2_PROBE
  pr_acc[6] = role;
  pr_acc[7] = simd * 16 + slot + (even ? 256 : 0);
#endif
  if (role < 8) {
    // ================================ D waves: depthwise scatter ==========================
    const int xc = role;  // tile column
    f32x2 wp[27];         // channels l, l + 64 (a pair: two v_fma_f32 per operation)
    float wsg[27];        // channel l + 128
#pragma unroll
    for (int k = 0; k < 27; ++k) {
      wp[k] = f32x2{planes[lane * 27 + k], planes[(lane + 64) * 27 + k]};
      wsg[k] = planes[(lane + 128) * 27 + k];
    }
    const f32x2 biasp = f32x2{planes[HID * 27 + lane], planes[HID * 27 + lane + 64]};
    const float biass = planes[HID * 27 + lane + 128];
    f32x2 accp[3][TY];  // output-plane accumulators, slot (o - z0 + 2) mod 3
    float accs[3][TY];
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int o = 0; o < TY; ++o) {
        accp[s][o] = f32x2{0.f, 0.f};
        accs[s][o] = 0.f;
      }
    __syncthreads();  // (prologue) weights read out of the plane buffer
    __syncthreads();  // (prologue) plane z0-1 committed
    // input rows [r_lo, r_hi) of plane `cur` into A = acc[SA] (kz 2), B = acc[SB] (kz 1) and
    // C = acc[SC] (kz 0, first touch assigns); each row's LDS reads issued one row ahead
    auto rows = [&](const float* cur, auto SAc, auto SBc, auto SCc, int r_lo, int r_hi) {
      constexpr int SA = decltype(SAc)::value, SB = decltype(SBc)::value,
                    SC = decltype(SCc)::value;
      f32x2 nxp[3];
      float nxs[3];
      auto ld = [&](int r) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float* q = cur + (r * K::PX + xc + k) * HID + lane;
          nxp[k] = f32x2{q[0], q[64]};
          nxs[k] = q[128];
        }
      };
      if (r_lo < r_hi) ld(r_lo);
#pragma unroll
      for (int r = 0; r < K::PY; ++r) {
        if (r < r_lo || r >= r_hi) continue;
        f32x2 vp[3];
        float vs[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          vp[k] = nxp[k];
          vs[k] = nxs[k];
        }
        if (r + 1 < r_hi) ld(r + 1);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int o = r - ky;
          if (o < 0 || o >= TY) continue;
          const f32x2* w0 = wp + ky * 3;
          const float* s0 = wsg + ky * 3;
          if (ky == 0) {
            accp[SC][o] = w0[2] * vp[2] + (w0[1] * vp[1] + w0[0] * vp[0]);
            accs[SC][o] = s0[2] * vs[2] + (s0[1] * vs[1] + s0[0] * vs[0]);
          } else {
            accp[SC][o] = w0[2] * vp[2] + (w0[1] * vp[1] + (w0[0] * vp[0] + accp[SC][o]));
            accs[SC][o] = s0[2] * vs[2] + (s0[1] * vs[1] + (s0[0] * vs[0] + accs[SC][o]));
          }
          accp[SB][o] = w0[11] * vp[2] + (w0[10] * vp[1] + (w0[9] * vp[0] + accp[SB][o]));
          accs[SB][o] = s0[11] * vs[2] + (s0[10] * vs[1] + (s0[9] * vs[0] + accs[SB][o]));
          accp[SA][o] = w0[20] * vp[2] + (w0[19] * vp[1] + (w0[18] * vp[0] + accp[SA][o]));
          accs[SA][o] = s0[20] * vs[2] + (s0[19] * vs[1] + (s0[18] * vs[0] + accs[SA][o]));
        }
        __builtin_amdgcn_sched_barrier(0);  // rows stay in order (VGPRs)
      }
    };
    // one input plane p; R = (p - z0 + 1) mod 3 at compile time
    auto step = [&](int p, auto Rc) {
      constexpr int R = decltype(Rc)::value;
      typedef std::integral_constant<int, R> SA;
      typedef std::integral_constant<int, (R + 1) % 3> SB;
      typedef std::integral_constant<int, (R + 2) % 3> SC;
      const bool live = p <= z1;
      const float* cur = planes + ((p - z0 + 1) & 1) * K::PLANE_F;
      const bool dscat = !(a.dbg & 1);  // timing experiments only (WF_FFN_DBG)
      const int zl = p - 2;
      if (zl >= z0 && zl < z1 && !(a.dbg & 2)) {
        int ltid = lane;
        asm volatile("" : "+v"(ltid));
        ln2_row(h2b + ((zl - z0) & 1) * H2F, 4 * xc + ltid / LNL, ltid % LNL);
      }
      if (live && dscat) rows(cur, SA(), SB(), SC(), 0, SB_SPLIT);
      PROBE(0)
      __syncthreads();  // 1 -> 2
      PROBE(1)
      if (live) {
        if (dscat) rows(cur, SA(), SB(), SC(), SB_SPLIT, K::PY);
        const int zo = p - 1;
        if (zo >= z0) {
          float* h2t = h2b + ((zo - z0) & 1) * H2F;
#pragma unroll
          for (int o = 0; o < TY; ++o) {
            float h[3] = {accp[R][o].x + biasp.x, accp[R][o].y + biasp.y, accs[R][o] + biass};
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              if (sizeof(T) == 2) h[j] = bf2f(f2bf(h[j]));
              h2t[(o * TX + xc) * K::HS + lane + 64 * j] = h[j];
            }
          }
        }
      }
      PROBE(2)
      __syncthreads();  // 2 -> next 1
      PROBE(3)
    };
    // p - z0 + 1 = 0, 1, 2, ... : R cycles 0, 1, 2
    for (int p = z0 - 1; p <= z1 + 1; p += 3) {
      step(p, std::integral_constant<int, 0>());
      if (p + 1 <= z1 + 1) step(p + 1, std::integral_constant<int, 1>());
      if (p + 2 <= z1 + 1) step(p + 2, std::integral_constant<int, 2>());
    }
    PROBE_DUMP
    return;
  }

  // ================================== E waves ============================================
  __builtin_amdgcn_s_setprio(3);
  const int e = role - 8, et = e * 64 + lane;
  const int l15 = lane & 15, g4 = lane >> 4;
  const bool has_fc = e < C / 16;  // E waves 0..2: one output column tile each
  const int ct = has_fc ? e : 0;
  const T* src = reinterpret_cast<const T*>(a.h1) + (int64_t)b * D * H * W * HID;
  const int64_t plane_elems = (int64_t)H * W * HID;
  const float bs = a.bscale ? a.bscale[b] : 1.f;

  // fc weights hi in registers: A operand rows ct*16 + l15, k = ks*32 + 8 g4; lo from LDS
  bf16x8 fwh[HID / 32];
  const uint16_t* fwl = fwlo + (ct * 16 + l15) * HID + 8 * g4;
  {
    const uint16_t* wr = a.fc + (size_t)(ct * 16 + l15) * HID + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < HID / 32; ++ks) fwh[ks] = *reinterpret_cast<const bf16x8*>(wr + ks * 32);
  }
  // h1 staging: byte offsets inside one plane, loaded through a per-plane buffer descriptor
  // (32-bit voffsets).  Halo positions outside the volume get an offset past the descriptor's
  // range and planes outside [0, D) a zero-range descriptor: the loads return the zero
  // padding themselves and the commit is a plain copy.
  uint32_t off[NLDE];
#pragma unroll
  for (int j = 0; j < NLDE; ++j) {
    const int i = min(j * NE + et, K::PP * K::NV - 1);
    const int pos = i / K::NV, v = i - pos * K::NV;
    const int yy = y0 - 1 + pos / K::PX, xx = x0 - 1 + pos % K::PX;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    off[j] = ok ? (uint32_t)(((yy * W + xx) * HID + 4 * v) * (int)sizeof(T)) : 0x80000000u;
  }
  typename L::raw stg[NLDE];
  auto fetch = [&](int p) {
    const bool pz = p >= 0 && p < D;
    const T* base = src + (int64_t)min(max(p, 0), D - 1) * plane_elems;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T*>(base), 0, pz ? (int)(plane_elems * (int64_t)sizeof(T)) : 0, 0x00020000);
#pragma unroll
    for (int j = 0; j < NLDE; ++j) {
      if constexpr (sizeof(T) == 4)
        stg[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off[j], 0, 0));
      else
        stg[j] = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(rs, off[j], 0, 0));
    }
  };
  auto commit = [&](float* dst) {
    float* d0 = dst + et * 4;
#pragma unroll
    for (int j = 0; j < NLDE; ++j)
      if ((j + 1) * NE <= K::PP * K::NV || j * NE + et < K::PP * K::NV)
        *reinterpret_cast<f32x4*>(d0 + j * NE * 4) = L::up(stg[j]);
  };
  const int col = ct * 16 + 4 * g4;
  const float* sbase = a.stats ? a.stats : a.x;
  // output position of this lane's fc row in row tile rt
  auto gpos_of = [&](int zo, int rt, bool clamp) {
    const int lp = rt * 16 + l15;
    int yo = y0 + lp / TX, xo = x0 + lp % TX;
    if (clamp) {
      yo = min(yo, H - 1);
      xo = min(xo, W - 1);
    }
    return (int64_t)b * D * plane_sz + (int64_t)zo * plane_sz + (int64_t)yo * W + xo;
  };
  auto row_ok = [&](int rt) {
    const int lp = rt * 16 + l15;
    return y0 + lp / TX < H && x0 + lp % TX < W;
  };
  f32x4 xr[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  f32x2 es[2] = {f32x2{0.f, 1.f}, f32x2{0.f, 1.f}};
  auto load_resid = [&](int zo, int rt) {
    const int64_t g = gpos_of(zo, rt, true);
    xr[rt] = *reinterpret_cast<const f32x4*>(a.x + g * C + col);
    es[rt] = *reinterpret_cast<const f32x2*>(sbase + 2 * g);
  };
  // fc of row tile rt of h2 tile h2t + bias + Q4 residual + store of output plane zo
  auto fc_store = [&](const float* h2t, int zo, int rt) {
    const int lp = rt * 16 + l15;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint16_t* Bh = reinterpret_cast<const uint16_t*>(h2t) + (size_t)lp * (2 * K::HS);
#pragma unroll
    for (int ks = 0; ks < HID / 32; ++ks) {
      const int k = ks * 32 + 8 * g4;
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Bh + k);
      if (SPLIT) {
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Bh + HID + k);
        acc = mma32<P>(fwh[ks], bl, acc);
        acc = mma32<P>(*reinterpret_cast<const bf16x8*>(fwl + ks * 32), bh, acc);
      }
      acc = mma32<P>(fwh[ks], bh, acc);
    }
    f32x4 v = acc + *reinterpret_cast<const f32x4*>(fcb + col);
    const f32x4 xv = xr[rt];
    if (a.stats) {
      const f32x4 lw = *reinterpret_cast<const f32x4*>(n2w + col);
      const f32x4 lb = *reinterpret_cast<const f32x4*>(n2b + col);
      const float em = es[rt].x, er = es[rt].y;
      const f32x4 n2 = (xv - em) * er * lw + lb;
      v = xv + (n2 + v) * bs;
    } else {
      v = xv + v * bs;
    }
    if (row_ok(rt)) *reinterpret_cast<f32x4*>(a.out + gpos_of(zo, rt, false) * C + col) = v;
  };

  fetch(z0 - 1);
  __syncthreads();  // (prologue) weights read out of the plane buffer
  commit(planes);
  fetch(z0);
  __syncthreads();  // (prologue) plane z0-1 visible
  for (int p = z0 - 1; p <= z1 + 1; ++p) {
    const int zo = p - 2;  // output plane this iteration finishes
    const bool epi = has_fc && zo >= z0 && zo < z1;
    float* h2t = h2b + ((zo - z0) & 1) * H2F;
    // ---- phase 1: residual / statistics rows of plane p-2
    if (epi) {
      load_resid(zo, 0);
      load_resid(zo, 1);
    }
    PROBE(0)
    __syncthreads();  // 1 -> 2: LN rows of tile (p-2) visible
    PROBE(1)
    // ---- phase 2: commit plane p+1 into the free buffer, fetch p+2, fc of tile (p-2)
#pragma unroll
    for (int j = 0; j < NLDE; ++j) asm volatile("" ::"v"(stg[j]));
    if (p + 1 <= z1 && !(a.dbg & 8)) commit(planes + ((p - z0) & 1) * K::PLANE_F);
    if (p + 2 <= z1 && !(a.dbg & 8)) fetch(p + 2);
    if (epi && !(a.dbg & 4)) {
      fc_store(h2t, zo, 0);
      fc_store(h2t, zo, 1);
    }
    PROBE(2)
    __syncthreads();  // 2 -> next 1
    PROBE(3)
  }
  PROBE_DUMP
}

// ---------------------------------------------------------------------------------------
// Stage-2 shape (C = 96, hidden = 384): the same back half, re-tiled for a 4C row twice as
// wide.  Double-buffered planes and h2 tiles no longer fit next to the fc weights, so this one
// keeps ONE plane buffer (the next plane waits in registers) and 4 x 4 tiles:
//   LDS = haloed 6 x 6 x 384 plane (55 KB) + 16 x 384 h2 tile (25 KB) + the fc weight's hi
//         half (96 x 384 bf16, 75 KB) + LN2 / bias vectors = 159.6 KB, one workgroup per CU.
//   depthwise (all 12 waves): thread = (channel c, column pair xp) -- 384 x 2 = 768 threads;
//         one channel's 27 taps in VGPRs, four scalar LDS reads per input row (64 consecutive
//         channels per wave: conflict-free), rolling accumulators over the 3 output planes.
// Two roles with separate loops (same barrier sequence), so neither holds the other's
// registers and neither's loads sit in front of the other's in the in-order load counter:
//   F (waves 0..5): the fc, one 16-channel output tile each over the 16-position tile; A =
//         weight hi from LDS and (split) weight lo held in VGPRs for the whole march; + bias +
//         Q4 residual; the residual rows are prefetched one plane ahead;
//   G (waves 6..11): the h1 plane staging (fetched two planes ahead, committed one ahead);
//         waves 8..11 (one per SIMD) run LN2 + GELU + split, 16 lanes x 24 channels per
//         position (lane g owns the 16-byte chunks 4g + 64 j), in place as bf16 {hi, lo}.
// Per iteration p (3 barriers), with zo = p - 1 the output plane scatter(p) completed:
//   C | G commit(p+1); all write the fp32 h2 tile (zo); F issue the next plane's residual
//   loads | A | G fetch(p+2); waves 8..11 LN2(zo), the rest scatter(p+1) rows 0..s-1 | B |
//   F fc(zo) + store; everyone finishes scatter(p+1).
// (A variant that split LN2 into statistics on 4 waves + normalise / GELU / split by every
// thread from its own registers, behind a fourth barrier, measured 380 vs 361 us.)
// ---------------------------------------------------------------------------------------

struct DwFc2 {
  static constexpr int C = 96, HID = 384, TY = 4, TX = 4;
  static constexpr int NTH = 768, PY = TY + 2, PX = TX + 2, PP = PY * PX, NPOS = TY * TX;
  static constexpr int HS = HID + 4, WKP = HID + 8;
  static constexpr int PLANE_F = PP * HID, H2_F = NPOS * HS;
  static constexpr int NG = 384;                                   // G threads (staging)
  static constexpr int NV = HID / 4, NLD = (PP * NV + NG - 1) / NG;
  static constexpr int CT = C / 16, KS = HID / 32;
  static constexpr int LNL = 16, LNC = HID / LNL, LN_W0 = 8;      // LN2 rows: waves 8..11
  static constexpr size_t LDS_BYTES =
      (size_t)(PLANE_F + H2_F) * 4 + (size_t)C * WKP * 2 + (size_t)(2 * HID + 3 * C) * 4;
  static_assert(NPOS * LNL == NTH - 64 * LN_W0, "LN2 waves cover the tile");
  static_assert(CT * 64 == NTH - NG, "one F wave per fc column tile");
  static_assert(LDS_BYTES <= 160 * 1024, "one workgroup per CU");
  static_assert(HID * 27 <= PLANE_F, "depthwise weights staged in the plane buffer");
};

template <int P, typename T>
__global__ __launch_bounds__(768, 1) void ffn_dwfc2_kernel(DwFcArgs a) {
  typedef DwFc2 K;
  constexpr int C = K::C, HID = K::HID, TY = K::TY, TX = K::TX;
  constexpr bool SPLIT = P == PREC_SPLIT;
  typedef H1Load<T> L;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* plane = lds;                                            // [PP][HID]
  float* h2t = lds + K::PLANE_F;                                 // [NPOS][HS]
  uint16_t* wf = reinterpret_cast<uint16_t*>(h2t + K::H2_F);     // [C][WKP] fc weight hi
  float* lnw = reinterpret_cast<float*>(wf + C * K::WKP);        // [HID] halved
  float* lnb = lnw + HID;
  float* fcb = lnb + HID;                                        // [C]
  float* n2w = fcb + C;
  float* n2b = n2w + C;

  const int tid = threadIdx.x;
  // wave-uniform (scalar) wave index: role branches are real branches
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
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

  for (int i = tid; i < C * (HID / 8); i += K::NTH) {
    const int n = i / (HID / 8), k8 = i % (HID / 8);
    *reinterpret_cast<bf16x8*>(wf + n * K::WKP + 8 * k8) =
        *reinterpret_cast<const bf16x8*>(a.fc + (size_t)n * HID + 8 * k8);
  }
  for (int i = tid; i < HID; i += K::NTH) {  // halved: GELU is evaluated from x / 2
    lnw[i] = 0.5f * a.ln2_w[i];
    lnb[i] = 0.5f * a.ln2_b[i];
  }
  for (int i = tid; i < C; i += K::NTH) {
    fcb[i] = a.fc_b ? a.fc_b[i] : 0.f;
    n2w[i] = a.stats ? a.n2_w[i] : 1.f;
    n2b[i] = a.stats ? a.n2_b[i] : 0.f;
  }
  for (int i = tid; i < HID * 27; i += K::NTH) plane[i] = a.dw_w[i];
  __syncthreads();  // S0

  // ---- depthwise role (everyone): channel c, output columns 2 xp and 2 xp + 1
  const int c = tid % HID, xp = tid / HID;
  float w[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) w[k] = plane[c * 27 + k];
  const float bias = a.dw_b[c];
  float aA[2][TY], aB[2][TY], aC[2][TY];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int o = 0; o < TY; ++o) aA[q][o] = aB[q][o] = aC[q][o] = 0.f;
  const bool dscat = !(a.dbg & 1);  // timing experiments only (WF_FFN_DBG)
  // input rows [r_lo, r_hi) (compile-time after inlining) of the current plane into output
  // planes +1 (aC), 0 (aB), -1 (aA); each row's four LDS reads are issued one row ahead of its
  // FMAs, unconditionally (a load pending across a branch join is waited for at the join)
  auto rows = [&](int r_lo, int r_hi) {
    if (!dscat) return;
    const float* Pin = plane + 2 * xp * HID + c;
    float nx[4];
    auto ld = [&](int r) {
#pragma unroll
      for (int k = 0; k < 4; ++k) nx[k] = Pin[(r * K::PX + k) * HID];
    };
    ld(r_lo);
#pragma unroll
    for (int r = 0; r < K::PY; ++r) {
      if (r < r_lo || r >= r_hi) continue;
      const float u0 = nx[0], u1 = nx[1], u2 = nx[2], u3 = nx[3];
      if (r + 1 < r_hi) ld(r + 1);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int o = r - ky;
        if (o < 0 || o >= TY) continue;
        const float* w0 = w + ky * 3;
        aC[0][o] = fmaf(w0[2], u2, fmaf(w0[1], u1, fmaf(w0[0], u0, aC[0][o])));
        aC[1][o] = fmaf(w0[2], u3, fmaf(w0[1], u2, fmaf(w0[0], u1, aC[1][o])));
        aB[0][o] = fmaf(w0[11], u2, fmaf(w0[10], u1, fmaf(w0[9], u0, aB[0][o])));
        aB[1][o] = fmaf(w0[11], u3, fmaf(w0[10], u2, fmaf(w0[9], u1, aB[1][o])));
        aA[0][o] = fmaf(w0[20], u2, fmaf(w0[19], u1, fmaf(w0[18], u0, aA[0][o])));
        aA[1][o] = fmaf(w0[20], u3, fmaf(w0[19], u2, fmaf(w0[18], u1, aA[1][o])));
      }
      __builtin_amdgcn_sched_barrier(0);  // rows stay in order (VGPRs)
    }
  };
  // the completed output plane (aA + bias) into the fp32 h2 tile, then the accumulators roll
  auto h2_out = [&](bool valid) {
    if (valid) {
#pragma unroll
      for (int o = 0; o < TY; ++o)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          float h = aA[q][o] + bias;
          if (sizeof(T) == 2) h = bf2f(f2bf(h));
          h2t[(o * TX + 2 * xp + q) * K::HS + c] = h;
        }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int o = 0; o < TY; ++o) {
        aA[q][o] = aB[q][o];
        aB[q][o] = aC[q][o];
        aC[q][o] = 0.f;
      }
  };
  // LN2 + GELU + split of one tile position per 16 lanes (24 channels each, lane g owns the
  // 16-byte chunks 4g + 64 j), rewritten in place as bf16 {hi[HID], lo[HID]}: the lanes of a
  // row are one 16-lane group of a wave, so all its reads precede its writes
  auto ln2_row = [&]() {
    const int ltid = tid - 64 * K::LN_W0;
    const int pos = ltid / K::LNL, g = ltid % K::LNL;
    float* row = h2t + pos * K::HS;
    f32x4 v[K::LNC / 4];
#pragma unroll
    for (int j = 0; j < K::LNC / 4; ++j) v[j] = *reinterpret_cast<const f32x4*>(row + 4 * g + 64 * j);
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < K::LNC / 4; ++j) sm += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    const float mean = group_sum<K::LNL>(sm) * (1.f / HID);
    float qs = 0.f;
#pragma unroll
    for (int j = 0; j < K::LNC / 4; ++j) {
      const f32x4 d = v[j] - mean;
      qs += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
    const float rstd = rsqrtf(group_sum<K::LNL>(qs) * (1.f / HID) + a.eps2);
    const float nmr = -mean * rstd;
    uint16_t* rowh = reinterpret_cast<uint16_t*>(row);
#pragma unroll
    for (int j = 0; j < K::LNC / 4; ++j) {
      const int cc = 4 * g + 64 * j;
      const f32x4 lw4 = *reinterpret_cast<const f32x4*>(lnw + cc);
      const f32x4 lb4 = *reinterpret_cast<const f32x4*>(lnb + cc);
      const f32x4 y = gelu_half4((v[j] * rstd + nmr) * lw4 + lb4);
      uint32_t h0, h1, l0, l1;  // hi / lo operand words (split_pair: lo from v_dot2c)
      split_pair<P>(y[0], y[1], h0, l0);
      split_pair<P>(y[2], y[3], h1, l1);
      *reinterpret_cast<u32x2*>(rowh + cc) = u32x2{h0, h1};
      if (SPLIT) *reinterpret_cast<u32x2*>(rowh + HID + cc) = u32x2{l0, l1};
    }
  };
  // depthwise input rows scattered before barrier B by the F waves (sF) and waves 6, 7 (sG)
  // (B = 8 stage 2, runtime-swept: (sF, sG) = (3, 3) 352 us, (6, 3) 337, (2, 2) 361, (4, 4)
  // 337, (6, 6) 345)
  constexpr int sF = 4, sG = 4;
  PROBE_DECL

  if (wid < K::CT) {
    // ================================ F waves: fc + epilogue ==============================
    const int lln = tid & 63, l15 = lln & 15, g4 = lln >> 4;
    const int ct = wid;
    const int col = ct * 16 + 4 * g4;
    const int yo = y0 + l15 / TX, xo = x0 + l15 % TX;
    const bool rv = yo < H && xo < W;
    const int64_t gpos0 =
        (int64_t)b * D * plane_sz + (int64_t)min(yo, H - 1) * W + min(xo, W - 1);
    const float* sbase = a.stats ? a.stats : a.x;
    const float bs = a.bscale ? a.bscale[b] : 1.f;
    const uint16_t* wr = a.fc + (size_t)(C + ct * 16 + l15) * HID + 8 * g4;
    // residual rows of output plane z (unconditional, clamped to the volume: the values of a
    // plane outside the segment are never used)
    f32x4 xr, xrn;
    f32x2 es, esn;
    auto epi_load = [&](int z, f32x4& xv, f32x2& ev) {
      const int64_t gpos = gpos0 + (int64_t)min(max(z, 0), D - 1) * plane_sz;
      xv = *reinterpret_cast<const f32x4*>(a.x + gpos * C + col);
      ev = *reinterpret_cast<const f32x2*>(sbase + 2 * gpos);
    };
    // the fc weight's lo half of this wave's 16 output channels stays in VGPRs for the whole
    // z march (48 VGPRs; per plane it would be 1.3x the h1 plane's bytes through the load path)
    bf16x8 fwl[K::KS];
#pragma unroll
    for (int ks = 0; ks < K::KS; ++ks)
      fwl[ks] = SPLIT ? *reinterpret_cast<const bf16x8*>(wr + ks * 32) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    epi_load(z0, xrn, esn);
    __syncthreads();  // S1
    __syncthreads();  // S2: plane z0-1 visible
    rows(0, K::PY);
    for (int p = z0 - 1; p <= z1; ++p) {
      const int zo = p - 1;
      const bool valid = zo >= z0, more = p + 1 <= z1;
      __syncthreads();  // C: scatter(p) done everywhere, fc(zo-1) done
      PROBE(5)
      h2_out(valid);
      // issued unconditionally (a load pending across a branch join makes the compiler wait
      // for it right there)
      xr = xrn;
      es = esn;
      epi_load(zo + 1, xrn, esn);
      PROBE(0)
      __syncthreads();  // A: fp32 h2 tile (zo) and plane p+1 visible
      PROBE(1)
      if (more) rows(0, sF);
      PROBE(2)
      __syncthreads();  // B: bf16 {hi, lo} tile visible
      PROBE(3)
      if (valid && !(a.dbg & 4)) {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        const uint16_t* Bh = reinterpret_cast<const uint16_t*>(h2t) + (size_t)l15 * (2 * K::HS);
        const uint16_t* Wh = wf + (size_t)(ct * 16 + l15) * K::WKP;
#pragma unroll
        for (int ks = 0; ks < K::KS; ++ks) {
          const int k = ks * 32 + 8 * g4;
          const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Bh + k);
          const bf16x8 wh = *reinterpret_cast<const bf16x8*>(Wh + k);
          if (SPLIT) {
            const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Bh + HID + k);
            acc = mma32<P>(wh, bl, acc);
            acc = mma32<P>(fwl[ks], bh, acc);
          }
          acc = mma32<P>(wh, bh, acc);
        }
        f32x4 v = acc + *reinterpret_cast<const f32x4*>(fcb + col);
        if (a.stats) {
          const f32x4 nw = *reinterpret_cast<const f32x4*>(n2w + col);
          const f32x4 nbv = *reinterpret_cast<const f32x4*>(n2b + col);
          const f32x4 n2 = (xr - es.x) * es.y * nw + nbv;
          v = xr + (n2 + v) * bs;
        } else {
          v = xr + v * bs;
        }
        if (rv) *reinterpret_cast<f32x4*>(a.out + (gpos0 + (int64_t)zo * plane_sz) * C + col) = v;
      }
      if (more) rows(sF, K::PY);
      PROBE(4)
    }
    PROBE_DUMP
    return;
  }

  // ================================== G waves ============================================
  const int gt = tid - 64 * K::CT;
  const T* src = reinterpret_cast<const T*>(a.h1) + (int64_t)b * D * plane_sz * HID;
  const int64_t plane_elems = plane_sz * HID;
  int off[K::NLD];
  unsigned okmask = 0;
#pragma unroll
  for (int j = 0; j < K::NLD; ++j) {
    const int i = min(j * K::NG + gt, K::PP * K::NV - 1);
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
  auto commit = [&](int p) {
    const bool pz = p >= 0 && p < D;
#pragma unroll
    for (int j = 0; j < K::NLD; ++j) {
      const int i = j * K::NG + gt;
      const bool ok = pz && ((okmask >> j) & 1u);
      const f32x4 u = L::up(stg[j]);
      if (i < K::PP * K::NV)
        *reinterpret_cast<f32x4*>(plane + (size_t)i * 4) = ok ? u : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  const bool stat_role = wid >= K::LN_W0;  // LN2 rows
  fetch(z0 - 1);
  __syncthreads();  // S1: depthwise weights read out of the plane buffer
  commit(z0 - 1);
  fetch(z0);
  __syncthreads();  // S2
  rows(0, K::PY);
  for (int p = z0 - 1; p <= z1; ++p) {
    const int zo = p - 1;
    const bool valid = zo >= z0, more = p + 1 <= z1;
    __syncthreads();  // C
    PROBE(5)
#pragma unroll
    for (int j = 0; j < K::NLD; ++j) asm volatile("" ::"v"(stg[j]));
    if (more && !(a.dbg & 8)) commit(p + 1);
    h2_out(valid);
    PROBE(0)
    __syncthreads();  // A
    PROBE(1)
    // the plane after next: issued here so its address work and load issue overlap the LN2 /
    // scatter VALU work rather than the commit (latency: one full iteration)
    if (p + 2 <= z1 && !(a.dbg & 8)) fetch(p + 2);
    if (stat_role) {
      if (valid && !(a.dbg & 2)) ln2_row();
    } else if (more) {
      rows(0, sG);
    }
    PROBE(2)
    __syncthreads();  // B
    PROBE(3)
    if (more) rows(stat_role ? 0 : sG, K::PY);
    PROBE(4)
  }
  PROBE_DUMP
}

int launch_ffn_dwfc2(const DwFcArgs& a, int prec, hipStream_t s) {
  typedef DwFc2 K;
  DwFcArgs g = a;
  // z segment: whole columns where that still gives two workgroups per CU (B = 8 at 32^3:
  // 512 tiles of 4 x 4 x 32), shorter segments for small batches
  const int64_t base = (int64_t)g.B * cdiv(g.H, K::TY) * cdiv(g.W, K::TX);
  int ZS = g.D;
  while (ZS > 8 && base * cdiv(g.D, ZS) < 512) ZS = (ZS + 1) / 2;
  g.ZS = ZS;
  g.dbg = getenv("WF_FFN_DBG") ? atoi(getenv("WF_FFN_DBG")) : 0;  // timing experiments only
  const int64_t blocks = base * cdiv(g.D, ZS);
  void (*kern)(DwFcArgs) = prec == PREC_SPLIT  ? ffn_dwfc2_kernel<PREC_SPLIT, float>
                           : prec == PREC_FP16 ? ffn_dwfc2_kernel<PREC_FP16, float>
                                               : ffn_dwfc2_kernel<PREC_BF16, uint16_t>;
  set_max_lds(reinterpret_cast<const void*>(kern), (int)K::LDS_BYTES);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(K::NTH), K::LDS_BYTES, s, g);
  return check_launch("ffn_dwfc2");
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
  // + the fc weight lo plane for the SIMD-balanced kernel (bf16x3 only)
  const size_t lds = (size_t)(2 * K::PLANE_F + 2 * K::H2_F + 2 * HID + 3 * C) * 4 +
                     (prec == PREC_SPLIT ? (size_t)C * HID * 2 : 0);
  static const int dbg = getenv("WF_FFN_DBG") ? atoi(getenv("WF_FFN_DBG")) : 0;
  g.dbg = dbg;  // timing experiments only: bit mask of phases skipped (results invalid)
  // WF_FFN_DWFC_WS=1: the round-2 wave-specialised kernel (A/B); default the SIMD-balanced one
  static const bool ws = getenv("WF_FFN_DWFC_WS") != nullptr;
  // WF_FFN_DWFC_TB=1: three VALU waves per SIMD, one barrier per plane (ffn_dwfc_tb.hip;
  // round 4, under tuning)
  // default (round 4, fp32 h1): ffn_dwfc_tb4 -- three VALU waves per SIMD on 4 x 8 tiles,
  // LDS-DMA staging (977-989 vs 1027-1043 us for ffn_dwfc_sb at B = 8, profiles/r4_ffn_tb/);
  // WF_FFN_DWFC_SB=1 keeps the round-3 kernel, WF_FFN_DWFC_TB=1 the 3 x 8 single-barrier one
  static const char* tbv = getenv("WF_FFN_DWFC_TB");
  static const bool sbv = getenv("WF_FFN_DWFC_SB") != nullptr;
  // tb4 writes its output through buffer stores whose 32-bit byte offsets cover 2 GiB: larger
  // outputs (stage 1 of a 128^3 input at B >= 43) take the SIMD-balanced kernel, which has no
  // such limit
  const bool tb4_fits = (int64_t)g.B * g.D * g.H * g.W * C * 4 < ((int64_t)1 << 31);
  if (!ws && !sbv && prec != PREC_BF16 && (tb4_fits || (tbv && tbv[0] == '1')))
    return (tbv && tbv[0] == '1') ? launch_ffn_dwfc_tb(a, prec, s) : launch_ffn_dwfc_tb4(a, prec, s);
  void (*kern)(DwFcArgs) =
      ws ? (prec == PREC_SPLIT  ? ffn_dwfc_ws_kernel<PREC_SPLIT, float>
            : prec == PREC_FP16 ? ffn_dwfc_ws_kernel<PREC_FP16, float>
                                : ffn_dwfc_ws_kernel<PREC_BF16, uint16_t>)
         : (prec == PREC_SPLIT  ? ffn_dwfc_sb_kernel<PREC_SPLIT, float>
            : prec == PREC_FP16 ? ffn_dwfc_sb_kernel<PREC_FP16, float>
                                : ffn_dwfc_sb_kernel<PREC_BF16, uint16_t>);
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
