// ffn_dwfc_tb.hip -- the stage-1 CCF_FFN back half (C = 48, hidden = 192; SURVEY 8a a8, 8f
// row 1) with three VALU waves per SIMD and ONE barrier per plane (round 4, the default).
//
//   h2  = dwconv3x3x3(h1) + b          (wave_helper.py:285, groups = hidden, pad 1)
//   g   = GELU(LN_eps2(h2))            (:286-287)
//   ffn = fc(g) + fc_b                 (:289)
//   out = x + (n2 + ffn) * bs          (Block residual + CCF_FFN residual, quirk Q4, :293/:509)
//
// Why a new kernel (tools/ubench_valu.hip, profiles/r4_ubench_valu.txt): on gfx950 one wave
// issues a VALU instruction only every ~12 cycles, two waves of a SIMD together every ~3
// (v_fma_f32) to ~5.3 (v_fmac_f32 fed by ds_read_b32), and only three or more reach the
// SIMD-32 rate of 2 cycles.  ffn_dwfc_sb ran two VALU waves per SIMD (its 27 weights x 3
// channels per lane held 160 VGPRs): its D waves issued at ~4.4 cycles per instruction.
// Here every lane owns ONE channel, so a VALU wave fits 128 VGPRs and a SIMD holds three of
// them plus the staging / fc wave (16 waves, 1024 threads):
//
//   tile 3 (y) x 8 (x) positions, z-marching through ZS output planes;
//   D waves (12 = 3 per SIMD): lane = (channel c, column pair cp = the SIMD): the 27 taps of
//        channel c in VGPRs, per input row 4 ds_read_b32 (consecutive lanes = consecutive
//        channels: conflict-free) feed 2 columns x up to 3 output rows x 3 output planes;
//        and LN2 + GELU + the bf16 hi / lo split of 2 positions per wave (32 lanes x 6
//        channels per position: channel pairs 2g, 64 + 2g, 128 + 2g -> 8-B reads), placed
//        before, inside or after the scatter by the wave's slot so that the three waves of a
//        SIMD are not all in the LayerNorm's reduction chain at once.  96 VGPRs;
//   E waves (4 = 1 per SIMD, s_setprio 3): the haloed 5 x 10 x 192 h1 plane staged by
//        LDS-DMA (buffer_load_dwordx4 ... lds through a per-plane buffer descriptor, one plane
//        ahead; out-of-volume positions and planes come back as zeros), the fc of one
//        16-channel output column tile (waves 0..2) over the 24 positions on
//        v_mfma_f32_16x16x32 (x3 for bf16x3; weight hi in VGPRs, lo in LDS in fragment order),
//        bias + Q4 residual + 16-B stores.
// Probes (tools/tb_phase_times.py, -DWF_TB_PROBE): staging on the D waves through registers
// cost them 800-1400 cycles of a ~5600-cycle plane (12 waves' ds_write_b128 at once) and
// needed 112 VGPRs; on the E waves by registers it needed > 128 VGPRs (spills).  LDS-DMA
// needs neither.  fp32 h1 only (bf16x3, fp16 modes); the bf16 mode keeps ffn_dwfc_sb.
//
// Per iteration p (one barrier), with three h2 tiles rotating:
//   D: LN2 of h2 tile (p-2) in place;  scatter of plane p -> output plane p-1 complete ->
//      h2 tile (p-1)
//   E: LDS-DMA of plane p+1;  fc + epilogue of tile (p-3) -> output plane p-3
// Every producer -> consumer hand-off crosses exactly one barrier, so the phases of the D and
// E waves overlap freely inside an iteration.
//
// LDS: 2 x 38.4 KB planes + 3 x 18.8 KB h2 tiles + 18 KB fc lo fragments + vectors = 152 KB.
#include "kernels.hpp"

namespace wf {

#ifndef WF_TB_STAGGER
#define WF_TB_STAGGER 0
#endif
#ifndef WF_TB_EPRIO
#define WF_TB_EPRIO 3
#endif

namespace tb {
constexpr int C = 48, HID = 192, TY = 3, TX = 8;
constexpr int PY = TY + 2, PX = TX + 2, PP = PY * PX;  // haloed plane: 5 x 10
constexpr int NPOS = TY * TX;                          // 24
constexpr int HS = HID + 4;                            // h2 row stride (floats)
constexpr int PLANE_F = PP * HID;
constexpr int H2F = NPOS * HS;
constexpr int NV = HID / 4;                            // 16-B vectors per h1 row
constexpr int NPC = (PP * NV + 63) / 64;               // 1-KiB LDS-DMA pieces per plane (38)
constexpr int NPCE = (NPC + 3) / 4;                    // pieces per E wave
constexpr int KS = HID / 32;                           // fc k steps
constexpr int FWL_BYTES = (C / 16) * KS * 64 * 16;     // lo fragments [ct][ks][lane][8]
constexpr size_t LDS_BYTES = (size_t)(2 * PLANE_F + 3 * H2F + 2 * HID + 3 * C) * 4 + FWL_BYTES;
static_assert(LDS_BYTES <= 160 * 1024, "LDS");
}  // namespace tb

// sum over each 32-lane half: the DPP butterflies of group_sum<16>, then the two 16-lane rows
// exchanged by v_permlane16_swap (VALU; ds_swizzle would put an LDS round trip on the
// LayerNorm's dependency chain).  Every lane gets the same bits (lo + hi in both rows).
__device__ __forceinline__ float sum32(float v) {
  v = group_sum<16>(v);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

#ifdef WF_TB_PROBE
// diagnostic builds only: per-wave cycles of workgroup 0 by phase (read by wf_debug_tb_probe,
// tools/tb_phase_times.py); slots 6 / 7 = role / SIMD * 16 + arrival slot (+256 if balanced)
__device__ long long g_tb_probe[16 * 8];
extern "C" int wf_debug_tb_probe(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tb_probe), sizeof(g_tb_probe));
}
#define TB_PROBE_DECL                                                           \
  const bool probe_on = blockIdx.x == 0;                                        \
  long long pr_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pr_last = __builtin_amdgcn_s_memtime();
#define TB_PROBE(i)                                                             \
  if (probe_on) {                                                               \
    const long long t_ = __builtin_amdgcn_s_memtime();                          \
    pr_acc[i] += t_ - pr_last;                                                  \
    pr_last = t_;                                                               \
  }
#define TB_PROBE_DUMP                                                           \
  if (probe_on && lane == 0) {                                                  \
    pr_acc[6] = role;                                                           \
    pr_acc[7] = simd * 16 + slot + (even ? 256 : 0);                            \
    for (int i_ = 0; i_ < 8; ++i_) g_tb_probe[wid * 8 + i_] = pr_acc[i_];       \
  }
#else
#define TB_PROBE_DECL
#define TB_PROBE(i)
#define TB_PROBE_DUMP
#endif

__device__ __forceinline__ int tb_simd_id() {
  // HW_ID (hwreg 4) bits [5:4]: the SIMD the wave runs on
  return (int)((__builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4)) & 3);
}

template <int P, typename T>
__global__ __launch_bounds__(1024, 1) void ffn_dwfc_tb_kernel(DwFcArgs a) {
  using namespace tb;
  static_assert(sizeof(T) == 4, "the LDS-DMA staging copies fp32 h1 rows");
  constexpr bool SPLIT = P == PREC_SPLIT;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* planes = lds;                     // [2][PP][HID]
  float* h2b = lds + 2 * PLANE_F;          // [3][NPOS][HS]
  float* lnw = h2b + 3 * H2F;              // [HID] (halved: GELU from x / 2)
  float* lnb = lnw + HID;
  float* fcb = lnb + HID;                  // [C]
  float* n2w = fcb + C;
  float* n2b = n2w + C;
  bf16x8* fwlo = reinterpret_cast<bf16x8*>(n2b + C);  // [C/16][KS][64] fragments
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
  for (int i = tid; i < HID; i += 1024) {
    lnw[i] = 0.5f * a.ln2_w[i];
    lnb[i] = 0.5f * a.ln2_b[i];
  }
  for (int i = tid; i < C; i += 1024) {
    fcb[i] = a.fc_b ? a.fc_b[i] : 0.f;
    n2w[i] = a.stats ? a.n2_w[i] : 1.f;
    n2b[i] = a.stats ? a.n2_b[i] : 0.f;
  }
  if (SPLIT) {
    // lo plane in MFMA A-fragment order: fragment (ct, ks, l) = row ct*16 + (l & 15),
    // k = ks*32 + 8*(l >> 4): each fc lane later reads its own 16 contiguous bytes
    for (int i = tid; i < (C / 16) * KS * 64; i += 1024) {
      const int l = i & 63, ks = (i >> 6) % KS, ct = (i >> 6) / KS;
      fwlo[i] = *reinterpret_cast<const bf16x8*>(a.fc + (size_t)C * HID +
                                                 (size_t)(ct * 16 + (l & 15)) * HID + ks * 32 + 8 * (l >> 4));
    }
  }
  // depthwise weights and bias, coalesced into the (not yet used) plane buffer
  for (int i = tid; i < HID * 27; i += 1024) planes[i] = a.dw_w[i];
  for (int i = tid; i < HID; i += 1024) planes[HID * 27 + i] = a.dw_b[i];
  __syncthreads();
  // ---- roles: per SIMD, arrival slots 0..2 -> D waves, slot 3 -> the E wave
  const int simd = tb_simd_id();
  int slot = 0;
  if (lane == 0) slot = atomicAdd(&simd_cnt[simd], 1);
  slot = __builtin_amdgcn_readfirstlane(__shfl(slot, 0, 64));
  __syncthreads();
  const bool even = simd_cnt[0] == 4 && simd_cnt[1] == 4 && simd_cnt[2] == 4 && simd_cnt[3] == 4;
  // D role d = 3 * cp + k (cp = column pair, k = channel block of 64); E role 12 + e
  int role = even ? (slot < 3 ? 3 * simd + slot : 12 + simd) : wid;
  role = __builtin_amdgcn_readfirstlane(role);
  TB_PROBE_DECL

  if (role < 12) {
    // ================================ D waves ===========================================
    const int cp = role / 3, c = (role % 3) * 64 + lane;
    float w[27];
#pragma unroll
    for (int k = 0; k < 27; ++k) w[k] = planes[c * 27 + k];
    const float bias = planes[HID * 27 + c];
    float acc[3][TY][2];  // output-plane accumulators, slot (o - z0 + 2) mod 3
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int o = 0; o < TY; ++o) acc[s][o][0] = acc[s][o][1] = 0.f;
    // LN2 lanes: positions 2 * role + (lane >> 5), channel pairs 2g, 64 + 2g, 128 + 2g
    const int lpos = 2 * role + (lane >> 5), lg = lane & 31;
    const int kslot = __builtin_amdgcn_readfirstlane(role % 3);
    __syncthreads();  // (prologue) weights read out of the plane buffer
    __syncthreads();  // (prologue) plane z0-1 staged

    auto ln2_tile = [&](float* h2t) {
      float* row = h2t + lpos * HS;
      f32x2 v[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) v[j] = *reinterpret_cast<const f32x2*>(row + 64 * j + 2 * lg);
      const float s = (v[0].x + v[0].y) + ((v[1].x + v[1].y) + (v[2].x + v[2].y));
      const float mean = sum32(s) * (1.f / HID);
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float d0 = v[j].x - mean, d1 = v[j].y - mean;
        q += d0 * d0 + d1 * d1;
      }
      const float rstd = __builtin_amdgcn_rsqf(sum32(q) * (1.f / HID) + a.eps2);
      const float nmr = -mean * rstd;
      uint16_t* rowh = reinterpret_cast<uint16_t*>(row);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int cc = 64 * j + 2 * lg;
        const f32x2 lw2 = *reinterpret_cast<const f32x2*>(lnw + cc);
        const f32x2 lb2 = *reinterpret_cast<const f32x2*>(lnb + cc);
        const f32x2 y = gelu_half2((v[j] * rstd + nmr) * lw2 + lb2);
        const uint16_t h0 = op_cvt<P>(y.x), h1 = op_cvt<P>(y.y);
        *reinterpret_cast<uint32_t*>(rowh + cc) = (uint32_t)h0 | ((uint32_t)h1 << 16);
        if (SPLIT)
          *reinterpret_cast<uint32_t*>(rowh + HID + cc) =
              (uint32_t)(uint16_t)op_lo<P>(y.x, h0) | ((uint32_t)(uint16_t)op_lo<P>(y.y, h1) << 16);
      }
    };
    // input rows [LO, HI) of the plane (vin: all 5 rows x 4 columns, read at the start of the
    // step) into A = acc[SA] (kz 2), B = acc[SB] (kz 1), C = acc[SC] (kz 0, first touch
    // assigns)
    auto rows = [&](const float (&vin)[PY][4], auto SAc, auto SBc, auto SCc, auto LOc, auto HIc) {
      constexpr int SA = decltype(SAc)::value, SB = decltype(SBc)::value,
                    SC = decltype(SCc)::value, LO = decltype(LOc)::value, HI = decltype(HIc)::value;
#pragma unroll
      for (int r = LO; r < HI; ++r) {
        const float* v = vin[r];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int o = r - ky;
          if (o < 0 || o >= TY) continue;
          const float* w0 = w + ky * 3;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if (ky == 0)
              acc[SC][o][j] = w0[2] * v[j + 2] + (w0[1] * v[j + 1] + w0[0] * v[j]);
            else
              acc[SC][o][j] = w0[2] * v[j + 2] + (w0[1] * v[j + 1] + (w0[0] * v[j] + acc[SC][o][j]));
            acc[SB][o][j] = w0[11] * v[j + 2] + (w0[10] * v[j + 1] + (w0[9] * v[j] + acc[SB][o][j]));
            acc[SA][o][j] = w0[20] * v[j + 2] + (w0[19] * v[j + 1] + (w0[18] * v[j] + acc[SA][o][j]));
          }
        }
      }
    };
    typedef std::integral_constant<int, 0> I0;
    typedef std::integral_constant<int, 2> I2;
    typedef std::integral_constant<int, PY> IP;
    // one iteration p; R = (p - z0 + 1) mod 3 at compile time.  h2 tile of output plane z is
    // buffer (z - z0) mod 3: tile p-1 -> (R + 1) % 3, tile p-2 -> R
    auto step = [&](int p, auto Rc) {
      constexpr int R = decltype(Rc)::value;
      typedef std::integral_constant<int, R> SA;
      typedef std::integral_constant<int, (R + 1) % 3> SB;
      typedef std::integral_constant<int, (R + 2) % 3> SC;
      TB_PROBE(0)
      const bool live = p <= z1 && !(a.dbg & 1);
      const bool ln = p - 2 >= z0 && p - 2 < z1 && !(a.dbg & 2);
      float* h2ln = h2b + R * H2F;
      // the whole plane's 20 inputs of this lane first (10 ds_read2st64_b32 in flight)
      float vin[PY][4];
      if (live) {
        const float* q0 = planes + ((p - z0 + 1) & 1) * PLANE_F + 2 * cp * HID + c;
#pragma unroll
        for (int r = 0; r < PY; ++r)
#pragma unroll
          for (int k = 0; k < 4; ++k) vin[r][k] = q0[(r * PX + k) * HID];
      }
      // the three D waves of a SIMD place their LayerNorm (a latency-bound chain of
      // reductions) at different points of the scatter (slot 0: first, 1: after two input
      // rows, 2: last), so two of them issue independent FMAs while the third waits on it
#if WF_TB_STAGGER
      if (kslot == 0) {
        if (ln) ln2_tile(h2ln);
        if (live) rows(vin, SA(), SB(), SC(), I0(), IP());
      } else if (kslot == 1) {
        if (live) rows(vin, SA(), SB(), SC(), I0(), I2());
        if (ln) ln2_tile(h2ln);
        if (live) rows(vin, SA(), SB(), SC(), I2(), IP());
      } else
#endif
      {
        if (live) rows(vin, SA(), SB(), SC(), I0(), IP());
        if (ln) ln2_tile(h2ln);
      }
      TB_PROBE(2)
      if (live && p - 1 >= z0) {
        float* h2t = h2b + ((R + 1) % 3) * H2F;
#pragma unroll
        for (int o = 0; o < TY; ++o)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            float h = acc[R][o][j] + bias;
            if (sizeof(T) == 2) h = bf2f(f2bf(h));
            h2t[(o * TX + 2 * cp + j) * HS + c] = h;
          }
      }
      TB_PROBE(3)
      __syncthreads();
      TB_PROBE(4)
    };
    for (int p = z0 - 1; p <= z1 + 2; p += 3) {
      step(p, std::integral_constant<int, 0>());
      if (p + 1 <= z1 + 2) step(p + 1, std::integral_constant<int, 1>());
      if (p + 2 <= z1 + 2) step(p + 2, std::integral_constant<int, 2>());
    }
    TB_PROBE_DUMP
    return;
  }

  // ================================== E waves ============================================
  __builtin_amdgcn_s_setprio(WF_TB_EPRIO);
  const int e = role - 12;
  const int l15 = lane & 15, g4 = lane >> 4;
  const bool has_fc = e < C / 16;  // E waves 0..2: one output column tile each
  const int ct = has_fc ? e : 0;
  const float bs = a.bscale ? a.bscale[b] : 1.f;

  bf16x8 fwh[KS];
  {
    const uint16_t* wr = a.fc + (size_t)(ct * 16 + l15) * HID + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) fwh[ks] = *reinterpret_cast<const bf16x8*>(wr + ks * 32);
  }
  const bf16x8* fwl = fwlo + ct * KS * 64 + lane;
  // h1 plane staging by LDS-DMA (buffer_load_dwordx4 ... lds: no VGPR destination): piece
  // j = 4 k + e (1 KiB = 64 lanes x 16 B, lane-linear in the plane image [PP][HID]) of the
  // haloed plane; a halo position outside the volume gets an offset past the descriptor's
  // range and a plane outside [0, D) a zero-range descriptor, so the DMA writes the zero
  // padding itself
  const T* src = reinterpret_cast<const T*>(a.h1) + (int64_t)b * D * H * W * HID;
  const int64_t plane_elems = (int64_t)H * W * HID;
  uint32_t off[NPCE];
#pragma unroll
  for (int k = 0; k < NPCE; ++k) {
    const int i = min((4 * k + e) * 64 + lane, PP * NV - 1);
    const int pos = i / NV, v = i - pos * NV;
    const int yy = y0 - 1 + pos / PX, xx = x0 - 1 + pos % PX;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    off[k] = ok ? (uint32_t)(((yy * W + xx) * HID + 4 * v) * 4) : 0x80000000u;
  }
  auto stage = [&](int p, float* dst) {
    const bool pz = p >= 0 && p < D;
    const T* base = src + (int64_t)min(max(p, 0), D - 1) * plane_elems;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T*>(base), 0, pz ? (int)(plane_elems * 4) : 0, 0x00020000);
#pragma unroll
    for (int k = 0; k < NPCE; ++k) {
      const int j = 4 * k + e;
      if (j * 64 < PP * NV && (j * 64 + lane < PP * NV))
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(dst + j * 256), 16, off[k], 0, 0, 0);
    }
  };
  const int col = ct * 16 + 4 * g4;
  const float* sbase = a.stats ? a.stats : a.x;
  auto gpos_of = [&](int zo, int rt, bool clamp) {
    const int lp = min(rt * 16 + l15, NPOS - 1);
    int yo = y0 + lp / TX, xo = x0 + lp % TX;
    if (clamp) {
      yo = min(yo, H - 1);
      xo = min(xo, W - 1);
    }
    return (int64_t)b * D * plane_sz + (int64_t)zo * plane_sz + (int64_t)yo * W + xo;
  };
  auto row_ok = [&](int rt) {
    const int lp = rt * 16 + l15;
    return lp < NPOS && y0 + lp / TX < H && x0 + lp % TX < W;
  };
  f32x4 xr[2];
  f32x2 es[2];
  auto load_resid = [&](int zo, int rt) {
    const int64_t g = gpos_of(zo, rt, true);
    xr[rt] = *reinterpret_cast<const f32x4*>(a.x + g * C + col);
    es[rt] = *reinterpret_cast<const f32x2*>(sbase + 2 * g);
  };
  auto fc_store = [&](const float* h2t, int zo, int rt) {
    const int lp = min(rt * 16 + l15, NPOS - 1);
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint16_t* Bh = reinterpret_cast<const uint16_t*>(h2t) + (size_t)lp * (2 * HS);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = ks * 32 + 8 * g4;
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Bh + k);
      if (SPLIT) {
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Bh + HID + k);
        acc = mma32<P>(fwh[ks], bl, acc);
        acc = mma32<P>(fwl[ks * 64], bh, acc);
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

  __syncthreads();  // (prologue) weights read out of the plane buffer
  stage(z0 - 1, planes);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // (prologue) plane z0-1 staged
  for (int p = z0 - 1; p <= z1 + 2; ++p) {
    const int zo = p - 3;  // output plane this iteration stores
    // plane p+1 into the buffer plane p-1 left (scattered last iteration)
    if (p + 1 <= z1 && !(a.dbg & 8)) stage(p + 1, planes + ((p + 2 - z0) & 1) * PLANE_F);
    if (has_fc && zo >= z0 && zo < z1 && !(a.dbg & 4)) {
      const float* h2t = h2b + ((zo - z0) % 3) * H2F;
      fc_store(h2t, zo, 0);
      fc_store(h2t, zo, 1);
    }
    TB_PROBE(0)
    // the next iteration's residual / norm2-statistics rows, in flight across the barrier
    if (has_fc && zo + 1 >= z0 && zo + 1 < z1) {
      load_resid(zo + 1, 0);
      load_resid(zo + 1, 1);
    }
    TB_PROBE(1)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the staged plane has landed
    TB_PROBE(2)
    __syncthreads();
    TB_PROBE(4)
  }
  TB_PROBE_DUMP
}

// ---------------------------------------------------------------------------------------
// 4 x 8 variant (WF_FFN_DWFC_TB=4): the same three VALU waves per SIMD on the tile of
// ffn_dwfc_sb (no 3-row waste: 64 rows / 4), which leaves room for only two h2 tiles, so two
// barriers per plane as in ffn_dwfc_sb:
//   phase 1: D slots 0, 1: LN2 of h2 tile (p-2), 16 lanes x 12 channels per position, 4
//            positions per wave (8 per SIMD); D slot 2: scatter rows [0, TB4_S2) of plane p
//            E: LDS-DMA of plane p+1 into the buffer plane p-1 left; residual rows of p-2
//   phase 2: D slots 0, 1: scatter rows [0, 6); slot 2: rows [TB4_S2, 6); all D: h2 tile p-1
//            E: fc of tile (p-2) + epilogue + store; wait for the DMA
// LDS: 2 x 46 KB planes + 2 x 25 KB h2 tiles + 18 KB fc lo fragments + vectors = 162,880 B.
// ---------------------------------------------------------------------------------------
#ifndef TB4_S2
#define TB4_S2 4
#endif
#ifndef WF_TB4_EPIPE  // 0: the first version's E-wave memory pipeline, for A/B
#define WF_TB4_EPIPE 1
#endif
namespace tb4 {
constexpr int C = 48, HID = 192, TY = 4, TX = 8;
constexpr int PY = TY + 2, PX = TX + 2, PP = PY * PX;  // 6 x 10
constexpr int NPOS = TY * TX;                          // 32
// h2 rows are HID + 8 floats apart (50 16-B quads, 2 mod 16): the fc's B-fragment reads (16
// rows x 4 k-quads per ds_read_b128) then meet 16 distinct 4-bank groups in every lane group,
// and LN2 lane lg of row r takes the channel quads m, m + 16, m + 32 with m = (lg - 2 r) & 15,
// which cancels the row's bank offset, so its reads (and its bf16 hi / lo writes) are
// conflict-free as well.  Round 5's HID + 4 rows with 12 contiguous channels per LN2 lane had
// 0.95 bank-conflict cycles per LDS instruction.
constexpr int HS = HID + 8;
constexpr int PLANE_F = PP * HID;
constexpr int H2F = NPOS * HS;
constexpr int NV = HID / 4;
constexpr int NPC = (PP * NV + 63) / 64;               // 45 LDS-DMA pieces
constexpr int NPCE = (NPC + 3) / 4;
constexpr int KS = HID / 32;
constexpr int FWL_BYTES = (C / 16) * KS * 64 * 16;
// vectors: LN2 affine (HID each), fc bias + norm2 bias folded into one (C), norm2 weight (C)
constexpr size_t LDS_BYTES = (size_t)(2 * PLANE_F + 2 * H2F + 2 * HID + 2 * C) * 4 + FWL_BYTES;
static_assert(LDS_BYTES <= 160 * 1024, "LDS");
}  // namespace tb4

template <int P>
__global__ __launch_bounds__(1024, 1) void ffn_dwfc_tb4_kernel(DwFcArgs a) {
  using namespace tb4;
  constexpr bool SPLIT = P == PREC_SPLIT;
  // separate static LDS objects (not one dynamic array carved by offsets): the compiler's
  // wait insertion can then tell the planes the LDS-DMA writes from the h2 tiles and fc
  // fragments the E waves read, instead of waiting for every DMA before any LDS read
  __shared__ __attribute__((aligned(16))) float planes[2 * PLANE_F];  // [2][PP][HID]
  __shared__ __attribute__((aligned(16))) float h2b[2 * H2F];         // [2][NPOS][HS]
  __shared__ __attribute__((aligned(16))) float vecs[2 * HID + 2 * C];
  __shared__ bf16x8 fwlo[FWL_BYTES / 16];
  float* lnw = vecs;                       // [HID] (halved: GELU from x / 2)
  float* lnb = lnw + HID;
  float* fcl = lnb + HID;                  // [C] fc bias (+ norm2 bias when stats are given)
  float* n2w = fcl + C;                    // [C]
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
  for (int i = tid; i < HID; i += 1024) {
    lnw[i] = 0.5f * a.ln2_w[i];
    lnb[i] = 0.5f * a.ln2_b[i];
  }
  for (int i = tid; i < C; i += 1024) {
    fcl[i] = (a.fc_b ? a.fc_b[i] : 0.f) + (a.stats ? a.n2_b[i] : 0.f);
    n2w[i] = a.stats ? a.n2_w[i] : 1.f;
  }
  if (SPLIT) {
    for (int i = tid; i < (C / 16) * KS * 64; i += 1024) {
      const int l = i & 63, ks = (i >> 6) % KS, ct = (i >> 6) / KS;
      fwlo[i] = *reinterpret_cast<const bf16x8*>(a.fc + (size_t)C * HID +
                                                 (size_t)(ct * 16 + (l & 15)) * HID + ks * 32 + 8 * (l >> 4));
    }
  }
  for (int i = tid; i < HID * 27; i += 1024) planes[i] = a.dw_w[i];
  for (int i = tid; i < HID; i += 1024) planes[HID * 27 + i] = a.dw_b[i];
  __syncthreads();
  const int simd = tb_simd_id();
  int slot = 0;
  if (lane == 0) slot = atomicAdd(&simd_cnt[simd], 1);
  slot = __builtin_amdgcn_readfirstlane(__shfl(slot, 0, 64));
  __syncthreads();
  const bool even = simd_cnt[0] == 4 && simd_cnt[1] == 4 && simd_cnt[2] == 4 && simd_cnt[3] == 4;
  int role = even ? (slot < 3 ? 3 * simd + slot : 12 + simd) : wid;
  role = __builtin_amdgcn_readfirstlane(role);

  if (role < 12) {
    // ================================ D waves ===========================================
    const int cp = role / 3, kslot = role % 3, c = kslot * 64 + lane;
    float w[27];
#pragma unroll
    for (int k = 0; k < 27; ++k) w[k] = planes[c * 27 + k];
    const float bias = planes[HID * 27 + c];
    float acc[3][TY][2];
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int o = 0; o < TY; ++o) acc[s][o][0] = acc[s][o][1] = 0.f;
    // LN2 (slots 0, 1): position 8 cp + 4 kslot + (lane >> 4), channel quads m, m + 16, m + 32
    // of its row, m = (lg - 2 lpos) & 15 (conflict-free banks, see HS)
    const int lpos = 8 * cp + 4 * kslot + (lane >> 4), lg = lane & 15;
    const int cm = 4 * ((lg - 2 * lpos) & 15);
    __syncthreads();  // (prologue) weights read out of the plane buffer
    __syncthreads();  // (prologue) plane z0-1 staged

    auto ln2_rows = [&](float* h2t) {
      constexpr int LNC = HID / 16;
      float* row = h2t + lpos * HS;
      float v[LNC];
#pragma unroll
      for (int j = 0; j < LNC / 4; ++j) {
        const f32x4 u = *reinterpret_cast<const f32x4*>(row + cm + 64 * j);
        v[4 * j] = u.x;
        v[4 * j + 1] = u.y;
        v[4 * j + 2] = u.z;
        v[4 * j + 3] = u.w;
      }
      float s4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) s4[j] = (v[j] + v[j + 4]) + v[j + 8];
      const float mean = group_sum<16>((s4[0] + s4[1]) + (s4[2] + s4[3])) * (1.f / HID);
      float q4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d0 = v[j] - mean, d1 = v[j + 4] - mean, d2 = v[j + 8] - mean;
        q4[j] = d2 * d2 + (d1 * d1 + d0 * d0);
      }
      const float rstd = __builtin_amdgcn_rsqf(
          group_sum<16>((q4[0] + q4[1]) + (q4[2] + q4[3])) * (1.f / HID) + a.eps2);
      const float nmr = -mean * rstd;
      uint16_t* rowh = reinterpret_cast<uint16_t*>(row);
#pragma unroll
      for (int j = 0; j < LNC / 4; ++j) {
        const int cc = cm + 64 * j;
        const f32x4 lw4 = *reinterpret_cast<const f32x4*>(lnw + cc);
        const f32x4 lb4 = *reinterpret_cast<const f32x4*>(lnb + cc);
        const f32x4 y = gelu_half4((f32x4{v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]} *
                                    rstd + nmr) * lw4 + lb4);
        uint32_t h0, h1, l0, l1;
        split_pair<P>(y[0], y[1], h0, l0);
        split_pair<P>(y[2], y[3], h1, l1);
        *reinterpret_cast<u32x2*>(rowh + cc) = u32x2{h0, h1};
        if (SPLIT) *reinterpret_cast<u32x2*>(rowh + HID + cc) = u32x2{l0, l1};
      }
    };
    auto rows = [&](const float (&vin)[PY][4], auto SAc, auto SBc, auto SCc, auto LOc, auto HIc) {
      constexpr int SA = decltype(SAc)::value, SB = decltype(SBc)::value,
                    SC = decltype(SCc)::value, LO = decltype(LOc)::value, HI = decltype(HIc)::value;
#pragma unroll
      for (int r = LO; r < HI; ++r) {
        const float* v = vin[r];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int o = r - ky;
          if (o < 0 || o >= TY) continue;
          const float* w0 = w + ky * 3;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if (ky == 0)
              acc[SC][o][j] = w0[2] * v[j + 2] + (w0[1] * v[j + 1] + w0[0] * v[j]);
            else
              acc[SC][o][j] = w0[2] * v[j + 2] + (w0[1] * v[j + 1] + (w0[0] * v[j] + acc[SC][o][j]));
            acc[SB][o][j] = w0[11] * v[j + 2] + (w0[10] * v[j + 1] + (w0[9] * v[j] + acc[SB][o][j]));
            acc[SA][o][j] = w0[20] * v[j + 2] + (w0[19] * v[j + 1] + (w0[18] * v[j] + acc[SA][o][j]));
          }
        }
      }
    };
    typedef std::integral_constant<int, 0> I0;
    typedef std::integral_constant<int, TB4_S2> IS;
    typedef std::integral_constant<int, PY> IP;
    auto step = [&](int p, auto Rc) {
      constexpr int R = decltype(Rc)::value;
      typedef std::integral_constant<int, R> SA;
      typedef std::integral_constant<int, (R + 1) % 3> SB;
      typedef std::integral_constant<int, (R + 2) % 3> SC;
      const bool live = p <= z1 && !(a.dbg & 1);
      const bool ln = p - 2 >= z0 && p - 2 < z1 && !(a.dbg & 2);
      float vin[PY][4];
      const float* q0 = planes + ((p - z0 + 1) & 1) * PLANE_F + 2 * cp * HID + c;
      auto load_plane = [&]() {
#pragma unroll
        for (int r = 0; r < PY; ++r)
#pragma unroll
          for (int k = 0; k < 4; ++k) vin[r][k] = q0[(r * PX + k) * HID];
      };
      // ---- phase 1.  The LN2 slots read their plane inputs after the LN2 (issued before the
      // barrier, consumed after it), so the 24 input registers are not live beside LN2's
      if (kslot < 2) {
        if (ln) ln2_rows(h2b + ((p - 2 - z0) & 1) * H2F);
        if (live) load_plane();
      } else if (live) {
        load_plane();
        rows(vin, SA(), SB(), SC(), I0(), IS());
      }
      __syncthreads();  // 1 -> 2: LN2'd tile (p-2) visible to the fc
      // ---- phase 2
      if (live) {
        if (kslot < 2) rows(vin, SA(), SB(), SC(), I0(), IP());
        else rows(vin, SA(), SB(), SC(), IS(), IP());
        if (p - 1 >= z0) {
          float* h2t = h2b + ((p - 1 - z0) & 1) * H2F;
#pragma unroll
          for (int o = 0; o < TY; ++o)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              h2t[(o * TX + 2 * cp + j) * HS + c] = acc[R][o][j] + bias;
        }
      }
      __syncthreads();  // 2 -> next 1
    };
    for (int p = z0 - 1; p <= z1 + 1; p += 3) {
      step(p, std::integral_constant<int, 0>());
      if (p + 1 <= z1 + 1) step(p + 1, std::integral_constant<int, 1>());
      if (p + 2 <= z1 + 1) step(p + 2, std::integral_constant<int, 2>());
    }
    return;
  }

  // ================================== E waves ============================================
  __builtin_amdgcn_s_setprio(WF_TB_EPRIO);
  const int e = role - 12;
  const int l15 = lane & 15, g4 = lane >> 4;
  const bool has_fc = e < C / 16;
  const int ct = has_fc ? e : 0;
  const float bs = a.bscale ? a.bscale[b] : 1.f;
  bf16x8 fwh[KS];
  {
    const uint16_t* wr = a.fc + (size_t)(ct * 16 + l15) * HID + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) fwh[ks] = *reinterpret_cast<const bf16x8*>(wr + ks * 32);
  }
  const bf16x8* fwl = fwlo + ct * KS * 64 + lane;
  const float* src = reinterpret_cast<const float*>(a.h1) + (int64_t)b * D * H * W * HID;
  const int64_t plane_elems = (int64_t)H * W * HID;
  // the DMA pieces' source offsets (k-th piece of this E wave); recomputed per plane on the
  // EPIPE path -- the E waves have VALU to spare and the registers went to the residual sets
  auto piece_off = [&](int k) {
    const int i = min((4 * k + e) * 64 + lane, PP * NV - 1);
    const int pos = i / NV, v = i - pos * NV;
    const int yy = y0 - 1 + pos / PX, xx = x0 - 1 + pos % PX;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    return ok ? (uint32_t)(((yy * W + xx) * HID + 4 * v) * 4) : 0x80000000u;
  };
#if !WF_TB4_EPIPE
  uint32_t off[NPCE];
#pragma unroll
  for (int k = 0; k < NPCE; ++k) off[k] = piece_off(k);
#endif
  auto stage = [&](int p, float* dst) {
    const bool pz = p >= 0 && p < D;
    const float* base = src + (int64_t)min(max(p, 0), D - 1) * plane_elems;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base), 0, pz ? (int)(plane_elems * 4) : 0, 0x00020000);
#pragma unroll
    for (int k = 0; k < NPCE; ++k) {
      const int j = 4 * k + e;
#if WF_TB4_EPIPE
      const uint32_t o = piece_off(k);
#else
      const uint32_t o = off[k];
#endif
      if (j * 64 < PP * NV && (j * 64 + lane < PP * NV))
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(dst + j * 256), 16, o, 0, 0, 0);
    }
  };
  const int col = ct * 16 + 4 * g4;
  const float* sbase = a.stats ? a.stats : a.x;
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
#if WF_TB4_EPIPE
  // The E waves' memory pipeline (vmcnt retires in issue order and counts stores too):
  //   * the residual rows of output plane zo + 1 are loaded in iteration p (ahead of the plane
  //     DMA), into the register set of zo + 1's parity, and used by the fc one iteration later
  //     -- the fc never waits for a load younger than the DMA, i.e. never for the DMA itself;
  //   * the output rows go out as range-checked buffer stores (rows outside the volume get an
  //     out-of-range offset and are dropped), exactly two per fc wave, so the end-of-phase wait
  //     for the DMA is vmcnt(2): it no longer waits for the stores to reach memory.
  // The first version (WF_TB4_EPIPE=0) loaded the residual in the same iteration, behind the
  // DMA, so the fc waited for both, and drained vmcnt(0) over its stores: two memory round
  // trips per plane on the E wave's path to the barrier.
  // residual / statistics rows through 32-bit buffer offsets (64-bit pointer pairs for the two
  // register sets spilled: the host keeps the tensors under 2 GiB)
  f32x4 xr[2][2];
  f32x2 es[2][2];
  const int64_t npos = (int64_t)a.B * D * plane_sz;
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.x), 0, (int)(npos * C * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t srsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(sbase), 0, (int)(npos * 2 * 4), 0x00020000);
  auto load_resid = [&](int zo, f32x4 (&xv)[2], f32x2 (&ev)[2]) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int g = (int)gpos_of(zo, rt, true);
      xv[rt] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrsrc, (g * C + col) * 4, 0, 0));
      ev[rt] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(srsrc, g * 8, 0, 0));
    }
  };
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
      a.out, 0, (int)(npos * C * 4), 0x00020000);
  auto fc_store = [&](const float* h2t, int zo, int rt, const f32x4& xv, const f32x2& ev) {
    const int lp = rt * 16 + l15;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint16_t* Bh = reinterpret_cast<const uint16_t*>(h2t) + (size_t)lp * (2 * HS);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = ks * 32 + 8 * g4;
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Bh + k);
      if (SPLIT) {
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Bh + HID + k);
        acc = mma32<P>(fwh[ks], bl, acc);
        acc = mma32<P>(fwl[ks * 64], bh, acc);
      }
      acc = mma32<P>(fwh[ks], bh, acc);
    }
    // fc + bias (+ norm2's bias, folded) and, with stats, norm2's normalised x * weight
    f32x4 v = acc + *reinterpret_cast<const f32x4*>(fcl + col);
    if (a.stats) {
      const f32x4 lw = *reinterpret_cast<const f32x4*>(n2w + col);
      v = xv + ((xv - ev.x) * ev.y * lw + v) * bs;
    } else {
      v = xv + v * bs;
    }
    const int voff = row_ok(rt) ? (int)((gpos_of(zo, rt, false) * C + col) * 4) : (int)0x80000000;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), orsrc, voff, 0, 0);
  };

  __syncthreads();  // (prologue) weights read out of the plane buffer
  stage(z0 - 1, planes);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // (prologue) plane z0-1 staged
  // iteration p: zo = p - 2; register set of output plane z: (z - z0) & 1, a compile-time S
  // for the fc (zo) and S ^ 1 for the prefetch (zo + 1) with the loop unrolled by two
  auto iter = [&](int p, auto Sc) {
    constexpr int S = decltype(Sc)::value;
    const int zo = p - 2;
    const bool epi = has_fc && zo >= z0 && zo < z1;
    // ---- phase 1: residual rows of zo + 1, then plane p + 1 into the buffer p - 1 left
    if (has_fc && zo + 1 >= z0 && zo + 1 < z1) load_resid(zo + 1, xr[S ^ 1], es[S ^ 1]);
    if (p + 1 <= z1 && !(a.dbg & 8)) stage(p + 1, planes + ((p + 2 - z0) & 1) * PLANE_F);
    // 1 -> 2 as a bare s_barrier: __syncthreads()' workgroup release fence makes the compiler
    // drain vmcnt(0) first -- the LDS-DMA writes LDS, so the fence waited for the plane just
    // issued and put a full memory round trip in front of every plane's phase 2.  This wave
    // wrote no LDS in phase 1; the DMA is waited for at the end of phase 2.
    __builtin_amdgcn_s_barrier();
    // ---- phase 2: fc of tile zo + epilogue; the staged plane must land before the barrier,
    // the two stores may still be in flight
    if (epi && !(a.dbg & 4)) {
      const float* h2t = h2b + ((zo - z0) & 1) * H2F;
      fc_store(h2t, zo, 0, xr[S][0], es[S][0]);
      fc_store(h2t, zo, 1, xr[S][1], es[S][1]);
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // bare as well (its fence would drain the stores): the DMA has landed (waited above) and
    // the LDS reads of the fc are complete before the barrier (lgkmcnt)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // 2 -> next 1
  };
  // (zo - z0) & 1 at p = z0 - 1 + i is (i + 1) & 1: even i -> S = 1
  for (int p = z0 - 1; p <= z1 + 1; p += 2) {
    iter(p, std::integral_constant<int, 1>());
    if (p + 1 <= z1 + 1) iter(p + 1, std::integral_constant<int, 0>());
  }
}
#else
  f32x4 xr[2];
  f32x2 es[2];
  auto load_resid = [&](int zo, int rt) {
    const int64_t g = gpos_of(zo, rt, true);
    xr[rt] = *reinterpret_cast<const f32x4*>(a.x + g * C + col);
    es[rt] = *reinterpret_cast<const f32x2*>(sbase + 2 * g);
  };
  auto fc_store = [&](const float* h2t, int zo, int rt) {
    const int lp = rt * 16 + l15;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint16_t* Bh = reinterpret_cast<const uint16_t*>(h2t) + (size_t)lp * (2 * HS);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = ks * 32 + 8 * g4;
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Bh + k);
      if (SPLIT) {
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Bh + HID + k);
        acc = mma32<P>(fwh[ks], bl, acc);
        acc = mma32<P>(fwl[ks * 64], bh, acc);
      }
      acc = mma32<P>(fwh[ks], bh, acc);
    }
    f32x4 v = acc + *reinterpret_cast<const f32x4*>(fcl + col);
    const f32x4 xv = xr[rt];
    if (a.stats) {
      const f32x4 lw = *reinterpret_cast<const f32x4*>(n2w + col);
      const float em = es[rt].x, er = es[rt].y;
      v = xv + ((xv - em) * er * lw + v) * bs;
    } else {
      v = xv + v * bs;
    }
    if (row_ok(rt)) *reinterpret_cast<f32x4*>(a.out + gpos_of(zo, rt, false) * C + col) = v;
  };

  __syncthreads();  // (prologue) weights read out of the plane buffer
  stage(z0 - 1, planes);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // (prologue) plane z0-1 staged
  for (int p = z0 - 1; p <= z1 + 1; ++p) {
    const int zo = p - 2;
    const bool epi = has_fc && zo >= z0 && zo < z1;
    // ---- phase 1: plane p+1 into the buffer plane p-1 left; residual rows of zo
    if (p + 1 <= z1 && !(a.dbg & 8)) stage(p + 1, planes + ((p + 2 - z0) & 1) * PLANE_F);
    if (epi) {
      load_resid(zo, 0);
      load_resid(zo, 1);
    }
    __syncthreads();  // 1 -> 2
    // ---- phase 2: fc of tile zo + epilogue; the staged plane must land before the barrier
    if (epi && !(a.dbg & 4)) {
      const float* h2t = h2b + ((zo - z0) & 1) * H2F;
      fc_store(h2t, zo, 0);
      fc_store(h2t, zo, 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // 2 -> next 1
  }
}
#endif

int launch_ffn_dwfc_tb4(const DwFcArgs& a, int prec, hipStream_t s) {
  using namespace tb4;
  DwFcArgs g = a;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int64_t base = (int64_t)g.B * cdiv(g.H, TY) * cdiv(g.W, TX);
  int best_zs = g.D;
  int64_t best = -1;
  for (int nz = 1; nz <= 8 && nz <= g.D; ++nz) {
    const int zs = (int)cdiv(g.D, nz);
    const int64_t cost = cdiv(base * cdiv(g.D, zs), cus) * (zs + 3);
    if (best < 0 || cost < best) {
      best = cost;
      best_zs = zs;
    }
  }
  g.ZS = best_zs;
  static const int dbg = getenv("WF_FFN_DBG") ? atoi(getenv("WF_FFN_DBG")) : 0;
  g.dbg = dbg;
  const int64_t blocks = base * cdiv(g.D, g.ZS);
  if (prec != PREC_SPLIT && prec != PREC_FP16) return fail(WF_E_SHAPE, "ffn_dwfc_tb4: fp32 h1 only");
  if ((int64_t)g.B * g.D * g.H * g.W * C * 4 >= ((int64_t)1 << 31))
    return fail(WF_E_SHAPE, "ffn_dwfc_tb4: output beyond the 2 GiB buffer-store range");
  void (*kern)(DwFcArgs) = prec == PREC_SPLIT ? ffn_dwfc_tb4_kernel<PREC_SPLIT>
                                              : ffn_dwfc_tb4_kernel<PREC_FP16>;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(1024), 0, s, g);  // static LDS
  return check_launch("ffn_dwfc_tb4");
}

int launch_ffn_dwfc_tb(const DwFcArgs& a, int prec, hipStream_t s) {
  using namespace tb;
  DwFcArgs g = a;
  // z segments: minimise (rounds of workgroups over the CUs) x (planes + 4 pipeline steps)
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int64_t base = (int64_t)g.B * cdiv(g.H, TY) * cdiv(g.W, TX);
  int best_zs = g.D;
  int64_t best = -1;
  for (int nz = 1; nz <= 8 && nz <= g.D; ++nz) {
    const int zs = (int)cdiv(g.D, nz);
    const int64_t cost = cdiv(base * cdiv(g.D, zs), cus) * (zs + 4);
    if (best < 0 || cost < best) {
      best = cost;
      best_zs = zs;
    }
  }
  g.ZS = best_zs;
  static const int dbg = getenv("WF_FFN_DBG") ? atoi(getenv("WF_FFN_DBG")) : 0;
  g.dbg = dbg;  // timing experiments only: bit mask of phases skipped (results invalid)
  const int64_t blocks = base * cdiv(g.D, g.ZS);
  if (prec != PREC_SPLIT && prec != PREC_FP16) return fail(WF_E_SHAPE, "ffn_dwfc_tb: fp32 h1 only");
  void (*kern)(DwFcArgs) = prec == PREC_SPLIT ? ffn_dwfc_tb_kernel<PREC_SPLIT, float>
                                              : ffn_dwfc_tb_kernel<PREC_FP16, float>;
  set_max_lds(reinterpret_cast<const void*>(kern), (int)LDS_BYTES);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(1024), LDS_BYTES, s, g);
  return check_launch("ffn_dwfc_tb");
}

}  // namespace wf
