// gemm_lnw.hip -- the CCF_FFN pwconv of encoder stage 2 (C = 96 -> hidden = 384, 32^3 rows
// per volume; wave_helper.py:281-283: pwconv + LayerNorm(4C) + GELU) as one MFMA GEMM with
// the LayerNorm over the full 384-wide output row in the epilogue:
//
//   h1[m, :] = GELU(LN1(bias + LN_n2(x[m, :]) . Wpw^T))
//
// gemm_kc (the generic K-chunked kernel) gives every wave all 384 columns of 16 rows, so each
// weight fragment staged in LDS feeds one 16-row MFMA per wave and the LDS reads outrun the
// MFMAs.  Here a workgroup owns 64 rows x 384 columns and splits the COLUMNS over its 4 waves
// (96 each): a wave's 4 x 6 tiles reuse every weight fragment 4 times and every A fragment 6
// times.
//   * A (64 rows x K, with the n2 LayerNorm applied from the given row stats) is loaded once,
//     split into bf16 hi / lo and parked in LDS; each K-step a wave reads its 4 row fragments.
//   * the weight never touches LDS: each wave streams its own 96 columns from L2 straight into
//     registers, one K-step ahead, tile by tile (a tile's registers are refilled one tile
//     after its MFMAs issue) -- no barrier inside the K loop.
//   * epilogue: bias, the row's LayerNorm moments reduced over the 4 lanes of a row and the 4
//     waves (two LDS exchanges: mean, then centred squares), LN1 affine + GELU, 16-B stores.
// Bound: HBM (x in, h1 out: 4 + 16 B per row-channel of C / 4C); the bf16x3 MFMA work
// (3 x 2 x 96 x 384 flops per row) runs under it.
#include "gemm_common.hpp"

namespace wf {


// LW_NTW column tiles per wave (N = 16 NWV LW_NTW), LW_RT row tiles of 16 rows per
// workgroup, NWV waves: (6, 4, 4) for N = 384 (stage 2).  (3, 8) for the stage-1 N = 192
// measured slower than gemm_rows (909 vs 974 volumes/s: K = 48 pads to two 32-wide K-steps
// and the A staging is exposed).  Round 5: the wide rows of stages 3 / 4 (N = 768 on 8 waves,
// 1536 on 16) -- the whole row in one workgroup, so the LayerNorm + GELU epilogue replaces
// the K-chunked GEMM + separate ln_act pass (a read and a write of h1)
template <int NWV> struct LnwBounds { static constexpr int MINW = NWV == 4 ? 2 : 1; };
template <int P, int KS, int LW_NTW, int LW_RT, int NWV = 4>
__global__ __launch_bounds__(NWV * 64, LnwBounds<NWV>::MINW) void gemm_lnw_kernel(GemmArgs g) {
  constexpr int NTH = NWV * 64;
  constexpr int LW_N = NWV * LW_NTW * 16;
  constexpr bool SPLIT = P == PREC_SPLIT;
  constexpr int NPL = SPLIT ? 2 : 1;
  constexpr int K32 = KS * 32;
  constexpr int AS = K32 + WF_LDS_KPAD;       // LDS row stride (bf16, gemm_common.hpp)
  constexpr int ROWS = LW_RT * 16;
  __shared__ __attribute__((aligned(16))) uint16_t As[NPL * ROWS * AS];
  __shared__ float red[NWV][ROWS];
  const int K = g.K, N = LW_N;
  const int64_t M = g.M;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g4 = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * ROWS;
  const int cw = wid * LW_NTW * 16;           // first column of this wave

  // ---- weight fragments of K-step 0 (lane: column cw + 16 t + l15, k = 8 g4 .. + 7)
  const uint16_t* wbase = g.w + (int64_t)(cw + l15) * K + 8 * g4;
  bf16x8 wh[LW_NTW], wl[LW_NTW];
  const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
  auto wload = [&](int ks, int t, bf16x8& h, bf16x8& l) {
    const int k = ks * 32 + 8 * g4;
    const int64_t o = (int64_t)t * 16 * K + ks * 32;
    h = k < K ? *reinterpret_cast<const bf16x8*>(wbase + o) : z8;
    if (SPLIT) l = k < K ? *reinterpret_cast<const bf16x8*>(wbase + (int64_t)N * K + o) : z8;
  };
  // ---- A: rows r0 .. r0 + 63, the n2 LayerNorm (LN_GIVEN) applied, split into LDS
  {
    constexpr int Q = K32 / 4;  // f32x4 per row (zero past K)
    for (int i = tid; i < ROWS * Q; i += NTH) {
      const int r = i / Q, q = i - r * Q;
      const int64_t row = min(r0 + r, M - 1);
      const int k = 4 * q;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (k < K) {
        v = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(g.a_src) + row * K + k);
        if (g.a_ln == LN_GIVEN) {
          const float mu = g.a_stats[2 * row], rs = g.a_stats[2 * row + 1];
          const f32x4 lw = *reinterpret_cast<const f32x4*>(g.a_ln_w + k);
          const f32x4 lb = *reinterpret_cast<const f32x4*>(g.a_ln_b + k);
          v = (v - mu) * rs * lw + lb;
        }
      }
      bf16x4 h4, l4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint16_t hb = op_cvt<P>(v[e]);
        h4[e] = (short)hb;
        l4[e] = op_lo<P>(v[e], hb);
      }
      *reinterpret_cast<bf16x4*>(As + r * AS + k) = h4;
      if (SPLIT) *reinterpret_cast<bf16x4*>(As + ROWS * AS + r * AS + k) = l4;
    }
  }
  __syncthreads();
  // the first K-step's weights are loaded here, after the staging.  (Round 2 saw 1-6 wrong
  // rows per launch when they were issued ahead of it; round 3 traced that, and the remaining
  // ~3 % of launches with 1-2 wrong rows, to the gfx950 packed-FP32 hazard the Makefile now
  // avoids: the staging's v_pk_mul_f32 / v_pk_fma_f32 read the n2 statistics' or LayerNorm
  // weights' VGPR pair before the load's last 16-lane group had landed -- DESIGN.md 6.1)
#pragma unroll
  for (int t = 0; t < LW_NTW; ++t) wload(0, t, wh[t], wl[t]);

  f32x4 acc[LW_RT][LW_NTW];
#pragma unroll
  for (int rt = 0; rt < LW_RT; ++rt)
#pragma unroll
    for (int t = 0; t < LW_NTW; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8 ah[LW_RT], al[LW_RT];
#pragma unroll
    for (int rt = 0; rt < LW_RT; ++rt) {
      const uint16_t* p = As + (rt * 16 + l15) * AS + ks * 32 + 8 * g4;
      ah[rt] = *reinterpret_cast<const bf16x8*>(p);
      al[rt] = SPLIT ? *reinterpret_cast<const bf16x8*>(p + ROWS * AS) : z8;
    }
#pragma unroll
    for (int t = 0; t < LW_NTW; ++t) {
      const bf16x8 bh = wh[t], bl = wl[t];
#pragma unroll
      for (int rt = 0; rt < LW_RT; ++rt) {
        if (SPLIT) {
          acc[rt][t] = mma32<P>(bh, al[rt], acc[rt][t]);
          acc[rt][t] = mma32<P>(bl, ah[rt], acc[rt][t]);
        }
        acc[rt][t] = mma32<P>(bh, ah[rt], acc[rt][t]);
      }
      // refill the PREVIOUS tile's registers with the next K-step's fragments: its MFMAs are
      // a whole tile of MFMAs old, so no load lands in a register an issued MFMA still reads
      __builtin_amdgcn_sched_barrier(0);
      if (t > 0 && ks + 1 < KS) wload(ks + 1, t - 1, wh[t - 1], wl[t - 1]);
      if (t == LW_NTW - 1 && ks + 1 < KS) {
        __builtin_amdgcn_sched_barrier(0);
        wload(ks + 1, t, wh[t], wl[t]);
      }
    }
  }

  // ---- epilogue: acc[rt][t][i] = out[row r0 + 16 rt + l15][column cw + 16 t + 4 g4 + i]
  const float* bias = g.bias;
#pragma unroll
  for (int t = 0; t < LW_NTW; ++t) {
    const f32x4 b4 = bias ? *reinterpret_cast<const f32x4*>(bias + cw + 16 * t + 4 * g4)
                          : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int rt = 0; rt < LW_RT; ++rt) acc[rt][t] += b4;
  }
  float mean[LW_RT], rstd[LW_RT];
#pragma unroll
  for (int rt = 0; rt < LW_RT; ++rt) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < LW_NTW; ++t) s += (acc[rt][t].x + acc[rt][t].y) + (acc[rt][t].z + acc[rt][t].w);
    s = xsum16(s);
    s = xsum32(s);
    if (g4 == 0) red[wid][rt * 16 + l15] = s;
  }
  __syncthreads();
  // the waves' partial sums of a row, added in a fixed order
  auto wsum = [&](int r) {
    float t = (red[0][r] + red[1][r]) + (red[2][r] + red[3][r]);
#pragma unroll
    for (int w = 4; w < NWV; w += 4) t += (red[w][r] + red[w + 1][r]) + (red[w + 2][r] + red[w + 3][r]);
    return t;
  };
#pragma unroll
  for (int rt = 0; rt < LW_RT; ++rt) {
    const int r = rt * 16 + l15;
    mean[rt] = wsum(r) * (1.f / LW_N);
  }
  __syncthreads();  // every wave has read the sums
#pragma unroll
  for (int rt = 0; rt < LW_RT; ++rt) {
    float q = 0.f;
#pragma unroll
    for (int t = 0; t < LW_NTW; ++t) {
      const f32x4 d = acc[rt][t] - mean[rt];
      q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
    q = xsum16(q);
    q = xsum32(q);
    if (g4 == 0) red[wid][rt * 16 + l15] = q;
  }
  __syncthreads();
#pragma unroll
  for (int rt = 0; rt < LW_RT; ++rt) {
    const int r = rt * 16 + l15;
    rstd[rt] = rsqrtf(wsum(r) * (1.f / LW_N) + g.e_eps);
  }
#pragma unroll
  for (int t = 0; t < LW_NTW; ++t) {
    const int col = cw + 16 * t + 4 * g4;
    // GELU from half its input (gelu_half4): the 1/2 folded into the LayerNorm affine
    const f32x4 lw = *reinterpret_cast<const f32x4*>(g.e_ln_w + col) * 0.5f;
    const f32x4 lb = *reinterpret_cast<const f32x4*>(g.e_ln_b + col) * 0.5f;
#pragma unroll
    for (int rt = 0; rt < LW_RT; ++rt) {
      const int64_t row = r0 + rt * 16 + l15;
      const f32x4 v = gelu_half4((acc[rt][t] - mean[rt]) * rstd[rt] * lw + lb);
      if (row < M) {
        if (g.out_bf16) {
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (short)f2bf(v[e]);
          *reinterpret_cast<bf16x4*>(reinterpret_cast<uint16_t*>(g.out) + row * g.ldo + col) = o;
        } else {
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(g.out) + row * g.ldo + col) = v;
        }
      }
    }
  }
}

template <int KS, int NTW, int RT, int NWV = 4>
void go_lnw(const GemmArgs& g, hipStream_t s) {
  const dim3 grid((unsigned)cdiv(g.M, RT * 16));
  auto k = g.prec == PREC_SPLIT  ? gemm_lnw_kernel<PREC_SPLIT, KS, NTW, RT, NWV>
           : g.prec == PREC_FP16 ? gemm_lnw_kernel<PREC_FP16, KS, NTW, RT, NWV>
                                 : gemm_lnw_kernel<PREC_BF16, KS, NTW, RT, NWV>;
  hipLaunchKernelGGL(k, grid, dim3(NWV * 64), 0, s, g);
}

// the wide-row shapes this kernel takes: the stage-3 pwconv N = 768 (K <= 192) -- 78.7 us
// against 61.6 + 43.9 for gemm_kc + ln_act_fwd at B = 8 (profiles/r5_lnw_wide_ab.txt).  The
// stage-4 N = 1536 on 16 waves measured 81.9 against 29.3 + 21.2 (256 workgroups of 16 rows
// each streaming the 2.4 MB weight: latency-bound), so it stays on the split path unless
// WF_LNW_WIDE1536=1
bool gemm_lnw_wide_shape(const GemmArgs& g) {
  static const bool off = getenv("WF_FFN_NO_LNW_WIDE") != nullptr;  // A/B switch
  static const bool w1536 = getenv("WF_LNW_WIDE1536") != nullptr;
  const int ks = (g.K + 31) / 32;
  return !off && ((g.N == 768 && ks == 6) || (w1536 && g.N == 1536 && ks == 12));
}

int try_launch_gemm_lnw(const GemmArgs& g, hipStream_t s) {
  static const bool off = getenv("WF_GEMM_NO_LNW") != nullptr;  // A/B switch
  if (off || g.epi != EPI_LN_GELU || g.a_map != MAP_IDENTITY || g.a_bf16 || g.a_gelu ||
      !(g.a_ln == LN_NONE || g.a_ln == LN_GIVEN) || g.a_C != g.K || g.K % 8 != 0 ||
      g.M >= ((int64_t)1 << 31) || g.ldo < g.N || g.ldo % 4 != 0)
    return 0;
  if (try_launch_pw2_resident(g, s)) return 1;
  const int ks = (g.K + 31) / 32;
  static const int wrt = getenv("WF_LNW_WIDE_RT") ? atoi(getenv("WF_LNW_WIDE_RT")) : 4;
  if (gemm_lnw_wide_shape(g)) {
    if (g.N == 768) {
      if (wrt == 2) go_lnw<6, 6, 2, 8>(g, s);
      else go_lnw<6, 6, 4, 8>(g, s);
    } else {
      go_lnw<12, 6, 1, 16>(g, s);
    }
    return 1;
  }
  if (g.N == 384) {
    // WF_LNW384: the stage-2 shape's (column tiles, row tiles, waves) -- 0: (6, 4, 4) (round
    // 2, 200.2-201.1 us at B = 8), 1: (3, 4, 8) (196.0), 2 (default): (3, 8, 8), 128 rows per
    // workgroup, the weight streamed once per 128 rows (194.5; profiles/r5_lnw_wide_ab.txt)
    static const int v384 = getenv("WF_LNW384") ? atoi(getenv("WF_LNW384")) : 2;
    if (ks == 3 && v384 == 1) { go_lnw<3, 3, 4, 8>(g, s); return 1; }
    if (ks == 3 && v384 == 2) { go_lnw<3, 3, 8, 8>(g, s); return 1; }
    switch (ks) {
      case 1: go_lnw<1, 6, 4>(g, s); return 1;
      case 2: go_lnw<2, 6, 4>(g, s); return 1;
      case 3: go_lnw<3, 6, 4>(g, s); return 1;
      case 4: go_lnw<4, 6, 4>(g, s); return 1;
      default: return 0;
    }
  }
  return 0;
}

}  // namespace wf
