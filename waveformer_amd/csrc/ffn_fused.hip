// ffn_fused.hip -- the whole stage-1 CCF_FFN of a Block in one kernel (C = 48, hidden = 192;
// SURVEY 8a a7/a8, 8f row 1):
//
//   n2  = LN(x; stats, n2_w, n2_b)     (norm2, wave_helper.py:508; x itself for a bare CCF_FFN)
//   u1  = GELU(LN1(pw(n2) + pw_b))     (wave_helper.py:279-283, LN eps 1e-5)
//   h2  = dwconv3x3x3(u1) + dw_b       (:285, groups = hidden, zero padding of u1)
//   ffn = fc(GELU(LN2(h2))) + fc_b     (:286-289)
//   out = x + (n2 + ffn) * bs          (Block residual + CCF_FFN residual, quirk Q4, :293/:509)
//
// Neither h1 nor h2 touches HBM: the kernel reads x (+ its norm2 stats) and writes out, 392 B
// per position, against 2.4 GB of h1 round trip per stage-1 block at B = 8 on the staged path
// (gemm_rows writes h1, ffn_dwfc reads it back).  A workgroup owns a 4 x 8 (y, x) tile and
// marches z through a segment of ZS output planes.  Per input plane p (3 barriers):
//   S1  every thread (two channels of one x column) scatters the u1 plane p from LDS into the
//       three output planes it feeds (rolling accumulators, f32x2 pair FMAs, 27 weight pairs in
//       registers), exactly as ffn_dwfc;
//   S2  the haloed 6 x 10 positions of plane p+1 run the pw GEMM on MFMA: wave w takes 16
//       positions (w & 3) x 64 hidden channels (w >> 2).  Its B operand is built in registers
//       from x rows prefetched one plane ahead (norm2 applied, bf16 hi / lo split), the weight
//       fragments come from LDS; the raw h1 + bias goes to the LDS plane together with each
//       wave's (mean, M2) over its 64 channels.  The h2 tile of output plane p-1 leaves the
//       accumulators for LDS;
//   S3  LN1 (the three partial moments combined, Chan et al.) + GELU in place on the plane,
//       zero outside the volume (the depthwise conv's padding); LN2 + GELU + split of the
//       h2 tile (16 lanes per position);
//   S4  six waves run the fc GEMM (2 position tiles x 3 channel tiles, x3 for the split) and
//       the Q4 epilogue; the other waves run ahead into the next plane's scatter.
#include "kernels.hpp"

namespace wf {

namespace ff {
constexpr int C = 48, HID = 192, TY = 4, TX = 8;
constexpr int NTH = (HID / 2) * TX;        // 768: one thread per (channel pair, column)
constexpr int WAVES = NTH / 64;
constexpr int PY = TY + 2, PX = TX + 2, PP = PY * PX;  // haloed plane: 60 positions
constexpr int NPOS = TY * TX;
constexpr int HS = HID + 4;                // u1 / h2 row stride in floats (bank spread)
constexpr int WK1 = C + 8;                 // pw weight row stride in bf16
constexpr int WKP = HID + 8;               // fc weight row stride in bf16
constexpr int PT = 4, CG = 3;              // pw: 4 position tiles (64 >= 60) x 3 channel groups
constexpr int CG_CH = HID / CG;            // 64 channels = 4 MFMA tiles per group
constexpr int RT = NPOS / 16, CT = C / 16; // fc tiles
constexpr int LN_LANES = 16, LN_CH = HID / LN_LANES;
constexpr int NV1 = PP * (HID / 4);        // LN1 items (f32x4) per plane
// LDS carve-up, in floats
constexpr int U1_F = PP * HS;
constexpr int H2_F = NPOS * HS;
constexpr int PWW_F = (2 * HID * WK1) / 2;
constexpr int FCW_F = (2 * C * WKP) / 2;
constexpr int PST_F = CG * 64 * 2;
constexpr int PRM_F = 5 * HID + 3 * C;
constexpr size_t LDS_BYTES = (size_t)(U1_F + H2_F + PWW_F + FCW_F + PST_F + PRM_F) * 4;
static_assert(PT * CG == WAVES, "one pw unit per wave");
static_assert(RT * CT <= WAVES, "at most one fc tile per wave");
static_assert(NPOS * LN_LANES <= NTH, "LN2 lanes");
static_assert(LDS_BYTES <= 160 * 1024, "LDS");
}  // namespace ff

template <int P>
__global__ __launch_bounds__(ff::NTH, 1) void ffn_fused_kernel(DwFcArgs a) {
  constexpr bool SPLIT = P == PREC_SPLIT;  // P: Prec (operand kind)
  using namespace ff;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* u1 = lds;                                                 // [PP][HS]
  float* h2t = u1 + U1_F;                                          // [NPOS][HS]
  uint16_t* pww = reinterpret_cast<uint16_t*>(h2t + H2_F);         // [2][HID][WK1]
  uint16_t* fcw = reinterpret_cast<uint16_t*>(h2t + H2_F + PWW_F); // [2][C][WKP]
  float* pst = h2t + H2_F + PWW_F + FCW_F;                         // [CG][64][2] {mean, M2}
  float* pwb = pst + PST_F;                                        // [HID]
  float* l1w = pwb + HID;
  float* l1b = l1w + HID;
  float* l2w = l1b + HID;
  float* l2b = l2w + HID;
  float* fcb = l2b + HID;                                          // [C]
  float* n2w = fcb + C;
  float* n2b = n2w + C;

  const int tid = threadIdx.x;
  const int wid = tid >> 6, lane = tid & 63;
  const int l15 = lane & 15, g4 = lane >> 4;
  const int D = a.D, H = a.H, W = a.W;

  // ---- tile of this workgroup (XCD-contiguous: neighbouring tiles share halo x rows in L2)
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
  for (int i = tid; i < 2 * HID * (C / 8); i += NTH) {
    const int pl = i / (HID * (C / 8)), r = i % (HID * (C / 8));
    const int n = r / (C / 8), k8 = r % (C / 8);
    const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    const bf16x8 v = (SPLIT || pl == 0)
                         ? *reinterpret_cast<const bf16x8*>(a.pw + ((size_t)pl * HID + n) * C + 8 * k8)
                         : z8;
    *reinterpret_cast<bf16x8*>(pww + ((size_t)pl * HID + n) * WK1 + 8 * k8) = v;
  }
  for (int i = tid; i < 2 * C * (HID / 8); i += NTH) {
    const int pl = i / (C * (HID / 8)), r = i % (C * (HID / 8));
    const int n = r / (HID / 8), k8 = r % (HID / 8);
    const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    const bf16x8 v = (SPLIT || pl == 0)
                         ? *reinterpret_cast<const bf16x8*>(a.fc + ((size_t)pl * C + n) * HID + 8 * k8)
                         : z8;
    *reinterpret_cast<bf16x8*>(fcw + ((size_t)pl * C + n) * WKP + 8 * k8) = v;
  }
  // LN1 / LN2 affine parameters halved: GELU is evaluated from x / 2 (gelu_half2)
  for (int i = tid; i < HID; i += NTH) {
    pwb[i] = a.pw_b ? a.pw_b[i] : 0.f;
    l1w[i] = 0.5f * a.ln1_w[i];
    l1b[i] = 0.5f * a.ln1_b[i];
    l2w[i] = 0.5f * a.ln2_w[i];
    l2b[i] = 0.5f * a.ln2_b[i];
  }
  // depthwise weights, coalesced into the (still unused) u1 plane, read back per thread below
  for (int i = tid; i < HID * 27; i += NTH) u1[i] = a.dw_w[i];
  __syncthreads();
  for (int i = tid; i < C; i += NTH) {
    fcb[i] = a.fc_b ? a.fc_b[i] : 0.f;
    n2w[i] = a.stats ? a.n2_w[i] : 1.f;
    n2b[i] = a.stats ? a.n2_b[i] : 0.f;
  }

  // ---- depthwise role: channel pair cp, column xi
  const int cp = tid % (HID / 2), xi = tid / (HID / 2);
  f32x2 w2[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) w2[k] = f32x2{u1[(2 * cp) * 27 + k], u1[(2 * cp + 1) * 27 + k]};
  const f32x2 bias2 = f32x2{a.dw_b[2 * cp], a.dw_b[2 * cp + 1]};

  // ---- pw role: haloed position hp of this lane's column of the MFMA B operand.  The x rows
  // are loaded unconditionally from clamped addresses (invalid rows are zeroed in S3), so a
  // plane's loads are one scalar base + fixed 32-bit offsets.
  const int pt = wid & 3, cg = wid >> 2;
  const int hp = 16 * pt + l15;
  const int hpc = min(hp, PP - 1);
  const int yy = y0 - 1 + hpc / PX, xx = x0 - 1 + hpc % PX;
  const int yc = min(max(yy, 0), H - 1), xc = min(max(xx, 0), W - 1);
  const int64_t plane_sz = (int64_t)H * W;
  const float* xb = a.x + (int64_t)b * D * plane_sz * C;
  const int offr = (yc * W + xc) * C;            // row of this lane in a plane
  const int kc = 4 * g4;                         // K-step s holds channels 16 s + kc .. +3
  // Every load below is unconditional (no branch joins on a load in flight, which would make
  // the compiler wait for it on the spot): without norm2 stats the stats pointer reads x and
  // the values are discarded at use.
  const float* sbase = a.stats ? a.stats : a.x;
  f32x4 st0, st1, st2;                           // the row chunks in flight
  f32x2 sst;                                     // their norm2 (mean, rstd)
  auto fetch = [&](int q) {
    const int qc = min(max(q, 0), D - 1);
    const float* r = xb + (int64_t)qc * plane_sz * C + offr + kc;
    st0 = *reinterpret_cast<const f32x4*>(r);
    st1 = *reinterpret_cast<const f32x4*>(r + 16);
    st2 = *reinterpret_cast<const f32x4*>(r + 32);
    const int64_t gp = (int64_t)b * D * plane_sz + (int64_t)qc * plane_sz + yc * W + xc;
    sst = *reinterpret_cast<const f32x2*>(sbase + 2 * gp);
  };

  // S2 for plane q: pw MFMA of this wave's (16 positions, 64 channels) -> raw h1 + bias, kept
  // in the lane's registers; the group's (mean, M2) per position goes to pst.  K = 48 = three
  // v_mfma_f32_16x16x16_bf16 steps (x3 for the split): lane (g4, l15) holds channels
  // 16 s + 4 g4 .. +3 of position l15, and gets back channels 16 t + 4 g4 .. +3 of tile t.
  auto pw_plane = [&](f32x4 (&acc)[4]) {
    // lane-derived LDS offsets from a laundered thread index: hoisted out of the z loop, the
    // loop-invariant parameter / bias reads below would stay live in VGPRs across it and spill
    int ltid = tid;
    asm volatile("" : "+v"(ltid));
    const int ll15 = ltid & 15, lg4 = (ltid >> 4) & 3, lcg = ltid >> 8, lkc = 4 * lg4;
    bf16x4 bh[3], bl[3];
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const f32x4 u = ks == 0 ? st0 : (ks == 1 ? st1 : st2);
      const f32x4 w4 = *reinterpret_cast<const f32x4*>(n2w + 16 * ks + lkc);
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(n2b + 16 * ks + lkc);
      const float smu = a.stats ? sst.x : 0.f, srs = a.stats ? sst.y : 1.f;
      const f32x4 n = (u - smu) * srs * w4 + b4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint16_t hb = op_cvt<P>(n[e]);
        bh[ks][e] = (short)hb;
        bl[ks][e] = op_lo<P>(n[e], hb);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ct = 4 * lcg + j;
      const uint16_t* Wr = pww + (size_t)(ct * 16 + ll15) * WK1 + lkc;
      f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const bf16x4 wh = *reinterpret_cast<const bf16x4*>(Wr + 16 * ks);
        if (SPLIT) {
          const bf16x4 wl = *reinterpret_cast<const bf16x4*>(Wr + HID * WK1 + 16 * ks);
          c = mma16<P>(wh, bl[ks], c);
          c = mma16<P>(wl, bh[ks], c);
        }
        c = mma16<P>(wh, bh[ks], c);
      }
      acc[j] = c + *reinterpret_cast<const f32x4*>(pwb + ct * 16 + lkc);
    }
    // (mean, M2) of this position over the group's 64 channels: 16 per lane, 4 lanes
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) s += (acc[j].x + acc[j].y) + (acc[j].z + acc[j].w);
    s += swz_xor16(s);
    s = xsum32(s);
    const float gm = s * (1.f / CG_CH);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 d = acc[j] - gm;
      q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
    q += swz_xor16(q);
    q = xsum32(q);
    const int lhp = 16 * ((ltid >> 6) & 3) + ll15;
    if (lg4 == 0 && lhp < PP) *reinterpret_cast<f32x2*>(pst + (lcg * 64 + lhp) * 2) = f32x2{gm, q};
  };

  // S3 for plane q: LN1 (the three groups' moments combined, Chan et al.) + GELU of the lane's
  // 16 values in registers, into the u1 plane; zero where the position lies outside the volume
  // (the depthwise conv's padding) or the whole plane is padding (have_acc false)
  auto ln1_store = [&](const f32x4 (&acc)[4], bool have_acc) {
    int ltid = tid;
    asm volatile("" : "+v"(ltid));
    const int ll15 = ltid & 15, lg4 = (ltid >> 4) & 3, lcg = ltid >> 8, lkc = 4 * lg4;
    const int lhp = 16 * ((ltid >> 6) & 3) + ll15;
    if (lhp >= PP) return;
    const int py = y0 - 1 + lhp / PX, px = x0 - 1 + lhp % PX;
    const bool ok = have_acc && py >= 0 && py < H && px >= 0 && px < W;
    float* pu = u1 + lhp * HS + lkc;
    if (!ok) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<f32x4*>(pu + (4 * lcg + j) * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
      return;
    }
    const f32x2 m0 = *reinterpret_cast<const f32x2*>(pst + (0 * 64 + lhp) * 2);
    const f32x2 m1 = *reinterpret_cast<const f32x2*>(pst + (1 * 64 + lhp) * 2);
    const f32x2 m2 = *reinterpret_cast<const f32x2*>(pst + (2 * 64 + lhp) * 2);
    const float mean = (m0.x + m1.x + m2.x) * (1.f / 3.f);
    const float d0 = m0.x - mean, d1 = m1.x - mean, d2 = m2.x - mean;
    const float m2s = (m0.y + m1.y + m2.y) + (float)CG_CH * (d0 * d0 + d1 * d1 + d2 * d2);
    const float rstd = rsqrtf(m2s * (1.f / HID) + a.eps1);
    const float nmr = -mean * rstd;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = (4 * lcg + j) * 16;
      const f32x4 lw = *reinterpret_cast<const f32x4*>(l1w + c + lkc);
      const f32x4 lb = *reinterpret_cast<const f32x4*>(l1b + c + lkc);
      *reinterpret_cast<f32x4*>(pu + c) = gelu_half4((acc[j] * rstd + nmr) * lw + lb);
    }
  };

  // epilogue inputs (x rows + norm2 stats of the fc lane's output row), loaded one step ahead
  // Two register sets, used alternately by the 2x-unrolled z loop: a copy from a set whose load
  // is in flight would make the compiler wait for it at the copy.
  f32x4 xrA = f32x4{0.f, 0.f, 0.f, 0.f}, xrB = xrA;
  f32x2 esA = f32x2{0.f, 1.f}, esB = esA;
  auto epi_fetch = [&](int zp, f32x4& xr_n, f32x2& es_n) {
    int ltid = tid;
    asm volatile("" : "+v"(ltid));
    const int fw = max((ltid >> 6) - (WAVES - RT * CT), 0);  // non-fc waves load tile 0 too
    const int lp = (fw / CT) * 16 + (ltid & 15);
    const int col = (fw % CT) * 16 + 4 * ((ltid >> 4) & 3);
    const int yo = min(y0 + lp / TX, H - 1), xo = min(x0 + lp % TX, W - 1);
    const int64_t gpos = (int64_t)b * D * plane_sz + (int64_t)zp * plane_sz + yo * W + xo;
    xr_n = *reinterpret_cast<const f32x4*>(a.x + gpos * C + col);
    es_n = *reinterpret_cast<const f32x2*>(sbase + 2 * gpos);
  };
  const float bs = a.bscale ? a.bscale[b] : 1.f;  // DropPath factor of this sample

  f32x2 accA[TY], accB[TY], accC[TY];
#pragma unroll
  for (int o = 0; o < TY; ++o) accA[o] = accB[o] = accC[o] = f32x2{0.f, 0.f};

  // ---- prologue: u1 of plane z0 - 1
  fetch(z0 - 1);
  __syncthreads();  // constants in LDS
  {
    f32x4 acc[4];
    if (z0 - 1 >= 0) pw_plane(acc);
    fetch(z0);
    __syncthreads();
    ln1_store(acc, z0 - 1 >= 0);
  }
  __syncthreads();

  auto step = [&](int p, const f32x4& xr_c, const f32x2& es_c, f32x4& xr_n, f32x2& es_n) {
    // ---- S1: scatter plane p into output planes p+1 (kz 0), p (kz 1), p-1 (kz 2)
    if (!(a.dbg & 1)) {
      const float* Pin = u1 + xi * HS + 2 * cp;
#pragma unroll
      for (int r = 0; r < PY; ++r) {
        const f32x2 v0 = *reinterpret_cast<const f32x2*>(Pin + (r * PX + 0) * HS);
        const f32x2 v1 = *reinterpret_cast<const f32x2*>(Pin + (r * PX + 1) * HS);
        const f32x2 v2 = *reinterpret_cast<const f32x2*>(Pin + (r * PX + 2) * HS);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int o = r - ky;
          if (o < 0 || o >= TY) continue;
          const f32x2* w0 = w2 + ky * 3;
          accC[o] = w0[2] * v2 + (w0[1] * v1 + (w0[0] * v0 + accC[o]));
          accB[o] = w0[11] * v2 + (w0[10] * v1 + (w0[9] * v0 + accB[o]));
          accA[o] = w0[20] * v2 + (w0[19] * v1 + (w0[18] * v0 + accA[o]));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    const int zo = p - 1;  // output plane completed by this input plane
    const int q = p + 1;   // next input plane, built in S2 / S3
    __syncthreads();       // B1: the plane is consumed (u1 free), fc(p-2) done (h2t free)
    // ---- S2: pw GEMM of plane q; h2 tile of output zo
    // Retire the loads issued a step ago on every path (an empty asm "reading" them): where the
    // pw or the fc is skipped their registers would otherwise stay pending, and the compiler
    // would then drain the loads issued just below (vmcnt(0)) before re-using the registers.
    asm volatile("" ::"v"(st0), "v"(st1), "v"(st2), "v"(sst), "v"(xr_c), "v"(es_c));
    f32x4 hacc[4];
    const bool have = q <= z1 && q >= 0 && q < D && !(a.dbg & 2);
    if (have) pw_plane(hacc);
    // Loads for the next step, issued after the pw consumed this step's: the epilogue rows of
    // output plane p first, then the x rows of plane q + 1.  Both stay in flight behind S3, S4
    // and the next scatter; the compiler's (in-order) vmcnt waits before them only cover loads
    // issued a step earlier.
    if (p >= z0 && p < z1) epi_fetch(p, xr_n, es_n);
    if (q + 1 <= z1 && !(a.dbg & 32)) fetch(q + 1);
    if (zo >= z0 && !(a.dbg & 64)) {
#pragma unroll
      for (int o = 0; o < TY; ++o) {
        f32x2 h = accA[o] + bias2;
        if (P == PREC_BF16) {  // bf16 mode: h2 carries bf16 rounding like the staged path
          h.x = bf2f(f2bf(h.x));
          h.y = bf2f(f2bf(h.y));
        }
        *reinterpret_cast<f32x2*>(h2t + (o * TX + xi) * HS + 2 * cp) = h;
      }
    }
    __syncthreads();  // B2: the moments of plane q, the h2 tile visible
    // ---- S3: LN1 + GELU of plane q into u1; LN2 + GELU + split of the h2 tile
    if (q <= z1 && !(a.dbg & 4)) ln1_store(hacc, have);
    int ltid = tid;
    asm volatile("" : "+v"(ltid));
    const int lln = ltid & 63, lwid = ltid >> 6;
    const int fw = lwid - (WAVES - RT * CT);  // fc tile of this wave (the last RT*CT waves)
    const int ct = max(fw, 0) % CT, ll15 = lln & 15, lg4 = lln >> 4;
    const int lp = (max(fw, 0) / CT) * 16 + ll15;
    const int yo = y0 + lp / TX, xo = x0 + lp % TX;
    const bool rv = yo < H && xo < W;
    const int64_t gpos = (int64_t)b * D * plane_sz + (int64_t)max(zo, 0) * plane_sz +
                         (int64_t)min(yo, H - 1) * W + min(xo, W - 1);
    const int col = ct * 16 + 4 * lg4;
    const bool fcw_wave = fw >= 0;
    if (zo >= z0) {
      if (ltid < NPOS * LN_LANES && !(a.dbg & 8)) {
        const int pos = ltid / LN_LANES, gg = ltid % LN_LANES;
        float* row = h2t + pos * HS;
        float v[LN_CH];
#pragma unroll
        for (int j = 0; j < LN_CH / 4; ++j) {
          const f32x4 u = *reinterpret_cast<const f32x4*>(row + gg * LN_CH + 4 * j);
          v[4 * j] = u.x;
          v[4 * j + 1] = u.y;
          v[4 * j + 2] = u.z;
          v[4 * j + 3] = u.w;
        }
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < LN_CH; ++j) s += v[j];
        const float mean = group_sum<LN_LANES>(s) * (1.f / HID);
        float qq = 0.f;
#pragma unroll
        for (int j = 0; j < LN_CH; ++j) {
          const float d = v[j] - mean;
          qq += d * d;
        }
        const float rstd = rsqrtf(group_sum<LN_LANES>(qq) * (1.f / HID) + a.eps2);
        const float nmr = -mean * rstd;
        uint16_t* rowh = reinterpret_cast<uint16_t*>(row);
#pragma unroll
        for (int j = 0; j < LN_CH / 4; ++j) {
          const int c = gg * LN_CH + 4 * j;
          const f32x4 lw4 = *reinterpret_cast<const f32x4*>(l2w + c);
          const f32x4 lb4 = *reinterpret_cast<const f32x4*>(l2b + c);
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
    }
    __syncthreads();  // B3: plane q ready for the next scatter, LN2 rows visible
    // ---- S4: fc GEMM (the last RT*CT waves) + bias + Q4 residual
    if (zo >= z0 && fcw_wave && !(a.dbg & 16)) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      const uint16_t* Bh = reinterpret_cast<const uint16_t*>(h2t) + (size_t)lp * (2 * HS);
      const uint16_t* Wh = fcw + (size_t)(ct * 16 + ll15) * WKP;
#pragma unroll
      for (int ks = 0; ks < HID / 32; ++ks) {
        const int k = ks * 32 + 8 * lg4;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Bh + k);
        const bf16x8 wh = *reinterpret_cast<const bf16x8*>(Wh + k);
        if (SPLIT) {
          const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Bh + HID + k);
          const bf16x8 wl = *reinterpret_cast<const bf16x8*>(Wh + C * WKP + k);
          acc = mma32<P>(wh, bl, acc);
          acc = mma32<P>(wl, bh, acc);
        }
        acc = mma32<P>(wh, bh, acc);
      }
      f32x4 v = acc + *reinterpret_cast<const f32x4*>(fcb + col);
      if (a.stats) {
        const f32x4 lw = *reinterpret_cast<const f32x4*>(n2w + col);
        const f32x4 lb = *reinterpret_cast<const f32x4*>(n2b + col);
        const f32x4 n2 = (xr_c - es_c.x) * es_c.y * lw + lb;
        v = xr_c + (n2 + v) * bs;
      } else {
        v = xr_c + v * bs;
      }
      if (rv) *reinterpret_cast<f32x4*>(a.out + gpos * C + col) = v;
    }
#pragma unroll
    for (int o = 0; o < TY; ++o) {
      accA[o] = accB[o];
      accB[o] = accC[o];
      accC[o] = f32x2{0.f, 0.f};
    }
  };
  for (int p = z0 - 1; p <= z1; p += 2) {
    step(p, xrA, esA, xrB, esB);
    if (p + 1 <= z1) step(p + 1, xrB, esB, xrA, esA);
  }
}

int launch_ffn_fused(const DwFcArgs& a, int prec, hipStream_t s) {
  using namespace ff;
  DwFcArgs g = a;
  // z segment: enough workgroups for a few rounds over the 256 CUs (one workgroup per CU, LDS
  // bound), long enough that the two halo planes per segment stay a small overhead
  const int64_t base = (int64_t)g.B * cdiv(g.H, TY) * cdiv(g.W, TX);
  int ZS = g.D;
  while (ZS > 8 && base * cdiv(g.D, ZS) < 1024) ZS = (ZS + 1) / 2;
  g.ZS = ZS;
  const char* dbg = getenv("WF_FFN_DBG");  // timing experiments: phases to skip (bit mask)
  g.dbg = dbg ? atoi(dbg) : 0;
  const int64_t blocks = base * cdiv(g.D, ZS);
  void (*kern)(DwFcArgs) = prec == PREC_SPLIT ? ffn_fused_kernel<PREC_SPLIT>
                           : prec == PREC_FP16 ? ffn_fused_kernel<PREC_FP16>
                                               : ffn_fused_kernel<PREC_BF16>;
  set_max_lds(reinterpret_cast<const void*>(kern), (int)LDS_BYTES);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(NTH), LDS_BYTES, s, g);
  return check_launch("ffn_fused");
}

}  // namespace wf
