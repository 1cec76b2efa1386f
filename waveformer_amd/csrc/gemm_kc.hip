// gemm_kc.hip -- K-chunked MFMA GEMM for the Linear layers whose weight is too large to sit in
// LDS whole (PatchMerging 8C -> 2C, the CCF_FFN fc of stages 2-4, stage 3/4 qkv/pw).
//
// out[m, n] = epilogue( sum_k A[m, k] * Wt[n, k] )
//   * workgroup = 8 waves x one row tile of 16 rows (128 rows) x one column chunk of
//     NC = NT * 16 output channels (grid.y walks the chunks);
//   * the weight chunk streams through LDS 32 k at a time, double buffered: the next k step's
//     [NC][32] bf16 hi (+ lo) slice is loaded into registers while the MFMAs of the current
//     one run, and written to the other buffer behind them (one barrier per k step);
//   * A fragments come straight from global memory into registers (lane l: row l&15,
//     k = 8*(l>>4) .. +7 of the step), one step ahead, through the row gather / LayerNorm /
//     GELU / bf16 hi-lo split of gemm_common.hpp's RowMapper;
//   * transposed MFMA (weight fragment = A operand), so each lane ends with 4 consecutive
//     output channels of one row: 16-byte epilogue loads and stores.
// LayerNorm of A: LN_GIVEN (stats passed in), LN_COMPUTE (one shifted sum / sum-of-squares
// pass over the row before the k loop) or LN_PARTIAL (per-group {mean, M2} of the producer
// combined by Chan's formula).
#include <algorithm>

#include "gemm_common.hpp"

namespace wf {

constexpr int KC_BK = 32;       // k per step (one 16x16x32 MFMA)
constexpr int KC_KP = KC_BK + WF_LDS_KPAD;  // LDS row stride in bf16 (gemm_common.hpp)

template <int NT, int WV = 8>
struct KcCfg {
  // one 16-row tile per wave and 8 waves per workgroup (128 rows): the accumulators stay
  // at NT * 4 VGPRs, so NT <= 8 fits four waves per SIMD to hide the A stream and the
  // per-step barrier (4 waves x 2 tiles: 168-188 VGPRs, two waves per SIMD, ~2x slower)
  static constexpr int RT = 1;
  static constexpr int WAVES = WV, NTHR = 64 * WAVES, ROWS = 16 * RT * WAVES;
  static constexpr int NC = NT * 16;
  static constexpr int WITEMS = NC * (KC_BK / 8);  // 16-byte pieces per plane per k step
  static constexpr int WPT = (WITEMS + NTHR - 1) / NTHR;  // per thread
};

// KR > 0 (K == 32 KR, LN_COMPUTE, one row tile per wave; PatchMerging 1 -> 2 at K = 384):
// the lane's whole A row share (KR k-octets, 8 KR floats) is loaded ONCE into registers before
// the k loop, the LayerNorm moments come from those registers and the (fully unrolled) k loop
// reads them again -- the round-3 statistics pass and the k loop each streamed the rows, and
// with 128-row workgroups the second read missed L2 (PMC 2.2x the input bytes)
// WV = 16 (PatchMerging 1 -> 2, 2048 workgroups of 8 waves): 256-row workgroups, so the weight
// chunk is staged through LDS once per 256 rows instead of per 128 -- at 128 rows the staged
// weight bytes (147 KB per workgroup, 302 MB per launch) were 60 % of the A bytes
template <int NT, int P, int MAP, int EPI, bool ABF16, int KR = 0, int WV = 8>
__global__ __launch_bounds__(64 * WV) void gemm_kc_kernel(GemmArgs g) {
  typedef KcCfg<NT, WV> C;
  constexpr bool SPLIT = P == PREC_SPLIT;  // P: Prec (operand kind)
  constexpr int RT = C::RT, NC = C::NC, NPL = SPLIT ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) uint16_t Wl[];  // [2][NPL][NC][KC_KP]
  const int K = g.K, N = g.N;
  const int M = (int)g.M;
  const int nks = (K + KC_BK - 1) / KC_BK;
  // split-K (g.ksplit > 1, small grids): this workgroup runs k steps [ks0, ks1) and stores its
  // raw fp32 partial sums to g.kpart; gemm_kc_reduce_kernel adds them in split order
  const bool part = g.ksplit > 1;
  int ks0 = 0, ks1 = nks;
  if (part) {
    const int per = (nks + g.ksplit - 1) / g.ksplit;
    ks0 = (int)blockIdx.z * per;
    ks1 = min(nks, ks0 + per);
  }
  const int kend = min(K, ks1 * KC_BK);
  const int c0 = blockIdx.y * NC;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g4 = lane >> 4;
  const int rbase = blockIdx.x * C::ROWS + wid * (16 * RT);

  // ---- weight staging: piece i -> (column i / 4, k-octet i % 4) of the step's slice.  Two
  // register sets: step ks + 2's slice is fetched while step ks runs, and step ks + 1's (fetched
  // a whole step earlier) is written to the other LDS buffer behind its MFMAs -- the round-3
  // loop fetched one step ahead and waited out a full L2 round trip in every step's commit
  typedef bf16x8 WRegs[NPL][C::WPT];
  WRegs wst[2];
  auto wfetch = [&](int ks, WRegs& dst) {
#pragma unroll
    for (int j = 0; j < C::WPT; ++j) {
      const int i = min(j * C::NTHR + tid, C::WITEMS - 1);
      // no zero-select on the loaded slice (a select is a use: it would wait for the load
      // where it is placed): pieces past K re-read the last octet, finite weights that only
      // meet the zeroed A octets (kv below), i.e. exact zero products
      const int n = c0 + (i >> 2), k = ks * KC_BK + 8 * (i & 3);
      const int64_t off = (int64_t)min(n, N - 1) * K + min(k, K - 8);
      dst[0][j] = *reinterpret_cast<const bf16x8*>(g.w + off);
      if (SPLIT) dst[NPL - 1][j] = *reinterpret_cast<const bf16x8*>(g.w + (int64_t)N * K + off);
    }
  };
  auto wcommit = [&](int buf, const WRegs& src) {
#pragma unroll
    for (int j = 0; j < C::WPT; ++j) {
      const int i = j * C::NTHR + tid;
      if (i < C::WITEMS) {
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl)
          *reinterpret_cast<bf16x8*>(Wl + ((size_t)(buf * NPL + pl) * NC + (i >> 2)) * KC_KP +
                                     8 * (i & 3)) = src[pl][j];
      }
    }
  };

  // ---- A rows of this lane (row l15 of each of its RT tiles) and their LayerNorm stats
  int arow[RT];
  float mean[RT], rstd[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    arow[rt] = min(rbase + rt * 16 + l15, M - 1);
    mean[rt] = 0.f;
    rstd[rt] = 1.f;
  }
  if (g.a_ln == LN_GIVEN) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      mean[rt] = g.a_stats[2 * arow[rt]];
      rstd[rt] = g.a_stats[2 * arow[rt] + 1];
    }
  }
  float areg[KR > 0 ? KR : 1][8];
  if constexpr (KR > 0) {
    static_assert(C::RT == 1, "register-resident A: one row tile per wave");
    const RowMapper<MAP> rm(g, arow[0]);
#pragma unroll
    for (int ks = 0; ks < KR; ++ks) load8f<ABF16>(g.a_src, rm.offset(g, ks * KC_BK + 8 * g4), areg[ks]);
    // the same shifted one-pass moments as below, in the same order (octet g4 + 4 ks)
    const float sh = __shfl(areg[0][0], l15, 64);
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int ks = 0; ks < KR; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = areg[ks][j] - sh;
        s += d;
        q += d * d;
      }
    s = xsum16(s);
    s = xsum32(s);
    q = xsum16(q);
    q = xsum32(q);
    const float ms = s / (float)K;
    mean[0] = sh + ms;
    rstd[0] = rsqrtf(fmaxf(q / (float)K - ms * ms, 0.f) + g.a_eps);
  } else if (g.a_ln == LN_COMPUTE) {
    // one pass: sums of x - s and (x - s)^2 with s = the row's first element (keeps the
    // variance free of cancellation when |mean| >> std); the 4 lanes of a row split the k range
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const RowMapper<MAP> rm(g, arow[rt]);
      float v0[8];
      load8f<ABF16>(g.a_src, rm.offset(g, 0), v0);
      const float sh = v0[0];
      float s = 0.f, q = 0.f;
      // four octets per batch, loads first: the round-3 loop waited out one load latency per
      // octet (12 in a row at K = 384); same summation order, the clamped tail octets add 0
      const int noct = K / 8;
      for (int cb = g4; cb < noct; cb += 16) {
        float v[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) load8f<ABF16>(g.a_src, rm.offset(g, min(cb + 4 * u, noct - 1) * 8), v[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float mk = cb + 4 * u < noct ? 1.f : 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float d = (v[u][j] - sh) * mk;
            s += d;
            q += d * d;
          }
        }
      }
      s = xsum16(s);
      s = xsum32(s);
      q = xsum16(q);
      q = xsum32(q);
      const float ms = s / (float)K;
      mean[rt] = sh + ms;
      rstd[rt] = rsqrtf(fmaxf(q / (float)K - ms * ms, 0.f) + g.a_eps);
    }
  } else if (g.a_ln == LN_PARTIAL) {
    const int np = g.a_np;
    const float ng = (float)(K / np);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const float* ps = g.a_stats + (int64_t)arow[rt] * np * 2;
      float s = 0.f;
      for (int c = g4; c < np; c += 4) s += ps[2 * c];
      s = xsum16(s);
      s = xsum32(s);
      const float mu = s / (float)np;
      float q = 0.f;
      for (int c = g4; c < np; c += 4) {
        const float d = ps[2 * c] - mu;
        q += ps[2 * c + 1] + ng * d * d;
      }
      q = xsum16(q);
      q = xsum32(q);
      mean[rt] = mu;
      rstd[rt] = rsqrtf(q / (float)K + g.a_eps);
    }
  }

  f32x4 acc[RT][NT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[rt][t] = f32x4{0, 0, 0, 0};

  typedef float ARegs[RT][8];
  ARegs an[2];
  auto afetch = [&](int ks, ARegs& dst) {
    if constexpr (KR > 0) return;
    const int k = min(ks * KC_BK + 8 * g4, K - 8);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const RowMapper<MAP> rm(g, arow[rt]);
      load8f<ABF16>(g.a_src, rm.offset(g, k), dst[rt]);
    }
  };

  // the loader's LayerNorm gamma/beta in LDS (a global load inside the k loop would queue on
  // the in-order vmcnt behind the prefetches and drain them every step)
  // (sized for an even step count: the unrolled loop's extra step of an odd count reads
  // lnw / lnb at k >= K, zeros here, discarded by its kv select)
  const int nks2 = part ? ((nks + 2) & ~1) : ((nks + 1) & ~1);  // kc_ln_steps
  float* lnw = reinterpret_cast<float*>(Wl + (size_t)2 * NPL * NC * KC_KP);
  float* lnb = lnw + nks2 * KC_BK;
  if (g.a_ln != LN_NONE) {
    for (int i = tid; i < nks2 * KC_BK; i += C::NTHR) {
      lnw[i] = i < K ? g.a_ln_w[i] : 0.f;
      lnb[i] = i < K ? g.a_ln_b[i] : 0.f;
    }
  }
  wfetch(ks0, wst[0]);
  afetch(ks0, an[0]);
  wfetch(min(ks0 + 1, ks1 - 1), wst[1]);
  afetch(min(ks0 + 1, ks1 - 1), an[1]);
  wcommit(0, wst[0]);
  __syncthreads();
  // step ks runs on LDS buffer / register set S = ks & 1 (a compile-time slot: the k loop is
  // unrolled by two)
  auto kbody = [&](int ks, auto slot, const ARegs& vin) {
    constexpr int S = decltype(slot)::value;
    const int buf = S;
    const int k = ks * KC_BK + 8 * g4;
    const bool kv = k < kend;
    float v[RT][8];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int j = 0; j < 8; ++j) v[rt][j] = vin[rt][j];
    wfetch(min(ks + 2, ks1 - 1), wst[S]);  // two steps ahead (tail steps: unused re-reads)
    bf16x8 ah[RT], al[RT];
    {
      float wv[8], bv[8];
      if (g.a_ln != LN_NONE) {
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(lnw + k);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(lnw + k + 4);
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(lnb + k);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(lnb + k + 4);
        wv[0] = w0.x; wv[1] = w0.y; wv[2] = w0.z; wv[3] = w0.w;
        wv[4] = w1.x; wv[5] = w1.y; wv[6] = w1.z; wv[7] = w1.w;
        bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w;
        bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        if (g.a_ln != LN_NONE) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[rt][j] = (v[rt][j] - mean[rt]) * rstd[rt] * wv[j] + bv[j];
        }
        if (g.a_gelu) {
          gelu_erf8(v[rt]);
        }
        {
          float xs[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) xs[j] = kv ? v[rt][j] : 0.f;
          split8<P>(xs, ah[rt], al[rt]);
        }
      }
    }
    // the A set of this slot is consumed (split) before its next load is issued, so the load
    // can reuse its registers: no loop-carried copies (and load waits) at the barrier
    afetch(min(ks + 2, ks1 - 1), an[S]);
    const uint16_t* Wb = Wl + (size_t)buf * NPL * NC * KC_KP;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int wo = (t * 16 + l15) * KC_KP + 8 * g4;
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Wb + wo);
      if (SPLIT) {
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Wb + NC * KC_KP + wo);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          acc[rt][t] = mma32<P>(bh, al[rt], acc[rt][t]);
          acc[rt][t] = mma32<P>(bl, ah[rt], acc[rt][t]);
        }
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        acc[rt][t] = mma32<P>(bh, ah[rt], acc[rt][t]);
      if (t % 4 == 3) __builtin_amdgcn_sched_barrier(0);
    }
    wcommit(buf ^ 1, wst[S ^ 1]);  // step ks + 1's slice, fetched during step ks - 1
    __syncthreads();
  };
  typedef std::integral_constant<int, 0> Slot0;
  typedef std::integral_constant<int, 1> Slot1;
  if constexpr (KR > 0) {
#pragma unroll
    for (int ks = 0; ks < KR; ks += 2) {
      ARegs vin;
#pragma unroll
      for (int j = 0; j < 8; ++j) vin[0][j] = areg[ks][j];
      kbody(ks, Slot0{}, vin);
      if (ks + 1 < KR) {
#pragma unroll
        for (int j = 0; j < 8; ++j) vin[0][j] = areg[ks + 1][j];
        kbody(ks + 1, Slot1{}, vin);
      }
    }
  } else {
    // both halves unconditional (a conditional second half makes the loop-carried register
    // sets phis, and their copies wait for the prefetches at every barrier): an odd step
    // count runs one extra step whose A operands are zeroed (k >= K: the kv select) against a
    // weight slice re-reading the last octet (finite), adding exact zeros
#pragma unroll 1
    for (int ks = ks0; ks < ks1; ks += 2) {
      kbody(ks, Slot0{}, an[0]);
      kbody(ks + 1, Slot1{}, an[1]);
    }
  }

  if (part) {  // raw partials (M, N) of split blockIdx.z; bias and epilogue in the reduce
    float* pz = g.kpart + (int64_t)blockIdx.z * M * N;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int row = rbase + rt * 16 + l15;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int col = c0 + t * 16 + 4 * g4;
        if (row < M && col < N) *reinterpret_cast<f32x4*>(pz + (int64_t)row * N + col) = acc[rt][t];
      }
    }
    return;
  }
  // ---- epilogue: acc[rt][t][i] = out[row rbase + 16 rt + l15][channel c0 + 16 t + 4 g4 + i]
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int row = rbase + rt * 16 + l15;
    const bool rv = row < M;
    const int rowc = min(row, M - 1);
    if (g.bias) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[rt][t] += *reinterpret_cast<const f32x4*>(g.bias + min(c0 + t * 16 + 4 * g4, N - 4));
    }
    float rm_ = 0.f, rs_ = 1.f, bs = 1.f;
    if (EPI == EPI_LN_GELU) {  // NC == N: the 4 lanes of a row hold the full row
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) s += (acc[rt][t].x + acc[rt][t].y) + (acc[rt][t].z + acc[rt][t].w);
      s = xsum16(s);
      s = xsum32(s);
      rm_ = s / (float)N;
      float q = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f32x4 d = acc[rt][t] - rm_;
        q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
      }
      q = xsum16(q);
      q = xsum32(q);
      rs_ = rsqrtf(q / (float)N + g.e_eps);
    } else if (EPI == EPI_RESID) {
      if (g.r_stats) {
        rm_ = g.r_stats[2 * rowc];
        rs_ = g.r_stats[2 * rowc + 1];
      }
      if (g.r_scale) bs = g.r_scale[rowc / (int)g.rows_per_sample];
    } else if (EPI == EPI_STORE && !ABF16) {
      // LayerNorm partials of this row's NC stored columns (fp32 stores only: the statistics
      // are those of the stored values): {mean, M2} over the 4 lanes of the row
      if (g.o_pstats) {
        float sm = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) sm += (acc[rt][t].x + acc[rt][t].y) + (acc[rt][t].z + acc[rt][t].w);
        sm = xsum16(sm);
        sm = xsum32(sm);
        const float mu = sm * (1.f / NC);
        float q = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const f32x4 d = acc[rt][t] - mu;
          q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
        }
        q = xsum16(q);
        q = xsum32(q);
        if (rv && g4 == 0)
          *reinterpret_cast<float2*>(g.o_pstats + ((int64_t)row * gridDim.y + blockIdx.y) * 2) =
              float2{mu, q};
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = c0 + t * 16 + 4 * g4;
      const int colc = min(col, N - 4);
      f32x4 v = acc[rt][t];
      if (EPI == EPI_LN_GELU) {
        const f32x4 lw = *reinterpret_cast<const f32x4*>(g.e_ln_w + colc);
        const f32x4 lb = *reinterpret_cast<const f32x4*>(g.e_ln_b + colc);
        v = (v - rm_) * rs_ * lw + lb;
        v = gelu_erf4(v);
      } else if (EPI == EPI_RESID) {
        const f32x4 xr = *reinterpret_cast<const f32x4*>(g.r_x + (int64_t)rowc * N + colc);
        if (g.r_stats) {
          const f32x4 lw = *reinterpret_cast<const f32x4*>(g.r_ln_w + colc);
          const f32x4 lb = *reinterpret_cast<const f32x4*>(g.r_ln_b + colc);
          const f32x4 n2 = (xr - rm_) * rs_ * lw + lb;
          v = xr + (n2 + v) * bs;  // attn_fused + drop_path(n2 + ffn(n2)), quirk Q4
        } else {
          v = xr + v * bs;
        }
      }
      if (rv && col < N) {
        if (g.out_bf16) {
          bf16x4 o;
          o[0] = (short)f2bf(v.x);
          o[1] = (short)f2bf(v.y);
          o[2] = (short)f2bf(v.z);
          o[3] = (short)f2bf(v.w);
          *reinterpret_cast<bf16x4*>(reinterpret_cast<uint16_t*>(g.out) + (int64_t)row * g.ldo + col) = o;
        } else {
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(g.out) + (int64_t)row * g.ldo + col) = v;
        }
      }
      if (t % 2 == 1) __builtin_amdgcn_sched_barrier(0);
    }
  }
}

constexpr int KC_MAX_SPLIT = 4;
// split-K reduction: out = epilogue(sum over splits z = 0, 1, .. in order + bias), one thread
// per 4 columns of a row (EPI_STORE without LayerNorm partials, EPI_RESID)
template <int EPI>
__global__ __launch_bounds__(256) void gemm_kc_reduce_kernel(GemmArgs g) {
  const int N = g.N, n4 = N / 4, M = (int)g.M;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= M * n4) return;
  const int row = i / n4, col = (i - row * n4) * 4;
  const int64_t MN = (int64_t)M * N;
  const float* p = g.kpart + (int64_t)row * N + col;
  f32x4 q[KC_MAX_SPLIT];  // all partial loads in flight before the in-order sum
#pragma unroll
  for (int z = 0; z < KC_MAX_SPLIT; ++z)
    if (z < g.ksplit) q[z] = *reinterpret_cast<const f32x4*>(p + z * MN);
  f32x4 v = q[0];
#pragma unroll
  for (int z = 1; z < KC_MAX_SPLIT; ++z)
    if (z < g.ksplit) v += q[z];
  if (g.bias) v += *reinterpret_cast<const f32x4*>(g.bias + col);
  if (EPI == EPI_RESID) {
    const f32x4 xr = *reinterpret_cast<const f32x4*>(g.r_x + (int64_t)row * N + col);
    const float bs = g.r_scale ? g.r_scale[row / (int)g.rows_per_sample] : 1.f;
    if (g.r_stats) {
      const float rm_ = g.r_stats[2 * row], rs_ = g.r_stats[2 * row + 1];
      const f32x4 lw = *reinterpret_cast<const f32x4*>(g.r_ln_w + col);
      const f32x4 lb = *reinterpret_cast<const f32x4*>(g.r_ln_b + col);
      const f32x4 n2 = (xr - rm_) * rs_ * lw + lb;
      v = xr + (n2 + v) * bs;  // as gemm_kc_kernel's EPI_RESID
    } else {
      v = xr + v * bs;
    }
  }
  if (g.out_bf16) {
    bf16x4 o;
    o[0] = (short)f2bf(v.x);
    o[1] = (short)f2bf(v.y);
    o[2] = (short)f2bf(v.z);
    o[3] = (short)f2bf(v.w);
    *reinterpret_cast<bf16x4*>(reinterpret_cast<uint16_t*>(g.out) + (int64_t)row * g.ldo + col) = o;
  } else {
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(g.out) + (int64_t)row * g.ldo + col) = v;
  }
}

// k splits for g (1 = none).  Only the GELU-loader fc of CCF_FFN at K >= 1536 (stage 4, 128
// workgroups at B = 8), with a caller scratch: 64.6 -> 54 us per B = 8 launch incl. the reduce;
// at stage 3 (K = 768, 512 workgroups) a split of 2 measured 71 -> 94 us, and the merging / qkv
// loaders gain nothing (profiles/r6/r6ks*_ab.txt).  The split count is a function of K, N and the
// precision only -- never of M -- so a row's sum order does not change with the batch (the B = 8
// graph replay equals per-volume B = 1 forwards, test_gpu_bench_config.py).
// (WF_KC_SPLIT: the largest split, A/B; 1 disables)
static int kc_ksplit(const GemmArgs& g, bool areg) {
  static const int maxs = getenv("WF_KC_SPLIT") ? std::max(1, atoi(getenv("WF_KC_SPLIT"))) : 4;
  if (!g.kpart || areg || g.o_pstats || !g.a_gelu || (g.epi != EPI_STORE && g.epi != EPI_RESID))
    return 1;
  if (g.M * (int64_t)(g.N / 4) >= ((int64_t)1 << 31) || g.N % 4 != 0 || g.K < 1536) return 1;
  const int nks = (g.K + KC_BK - 1) / KC_BK;
  // scratch: the caller's kpart_bytes is a multiple of M (the fc's dead h1 = M x hidden), so the
  // fit test below does not depend on M either
  int s = 1;
  while (2 * s <= std::min(maxs, KC_MAX_SPLIT) && nks / (2 * s) >= 6 &&
         (int64_t)(2 * s) * g.M * g.N * 4 <= g.kpart_bytes)
    s *= 2;
  if (s == 1) return 1;
  const int per = (nks + s - 1) / s;
  return (nks + per - 1) / per;  // every split non-empty
}

template <int NT, int MAP, int EPI>
static void go_kc(const GemmArgs& g, hipStream_t s) {
  typedef KcCfg<NT> C;
  const bool split = g.prec == PREC_SPLIT;
  void (*kern)(GemmArgs);
  // PatchMerging 1 -> 2 (K = 8 x 48): A rows register-resident, opt-in WF_KC_AREG=1 -- one
  // read of A, but 170 VGPRs (one 8-wave workgroup per CU instead of two) and it measured
  // 207-210 us against 204 us for the statistics pass + streaming k loop (round 4)
  static const bool no_areg = getenv("WF_KC_AREG") == nullptr || getenv("WF_KC_AREG")[0] == '0';
  constexpr bool areg_ok = MAP == MAP_MERGE && EPI == EPI_STORE && NT <= 8;
  const bool areg = areg_ok && !no_areg && g.K == 12 * KC_BK && g.a_ln == LN_COMPUTE && !g.a_bf16;
  if (areg)
    kern = split ? gemm_kc_kernel<NT, PREC_SPLIT, MAP, EPI, false, areg_ok ? 12 : 0>
                 : (g.prec == PREC_FP16 ? gemm_kc_kernel<NT, PREC_FP16, MAP, EPI, false, areg_ok ? 12 : 0>
                                        : gemm_kc_kernel<NT, PREC_BF16, MAP, EPI, false, areg_ok ? 12 : 0>);
  else if (g.a_bf16)  // bf16 activations only exist in PREC_BF16
    kern = gemm_kc_kernel<NT, PREC_BF16, MAP, EPI, true>;
  else if (split)
    kern = gemm_kc_kernel<NT, PREC_SPLIT, MAP, EPI, false>;
  else if (g.prec == PREC_FP16)
    kern = gemm_kc_kernel<NT, PREC_FP16, MAP, EPI, false>;
  else
    kern = gemm_kc_kernel<NT, PREC_BF16, MAP, EPI, false>;
  // 16-wave workgroups for every grid of >= 1024 8-wave workgroups (default, WF_KC_WV16=1),
  // PatchMerging only (=2) or none (=0): stage-1 merge 209.8 -> 201.9 us, stage-3 pwconv
  // 64.2 -> 61.4, config 5 45.6-45.8 -> 46.0 volumes/s (profiles/r4_gemm/)
  static const int wv16 = getenv("WF_KC_WV16") ? atoi(getenv("WF_KC_WV16")) : 1;
  int rows = C::ROWS, nthr = C::NTHR;
  if constexpr (NT <= 8 && EPI != EPI_LN_GELU) {
    const bool want = wv16 == 1 || (wv16 == 2 && MAP == MAP_MERGE);
    if (want && !areg && !g.a_bf16 && cdiv(g.M, C::ROWS) * (g.N / C::NC) >= 1024 &&
        (split || g.prec == PREC_FP16)) {
      kern = split ? gemm_kc_kernel<NT, PREC_SPLIT, MAP, EPI, false, 0, 16>
                   : gemm_kc_kernel<NT, PREC_FP16, MAP, EPI, false, 0, 16>;
      rows = KcCfg<NT, 16>::ROWS;
      nthr = KcCfg<NT, 16>::NTHR;
    }
  }
  GemmArgs gk = g;
  gk.ksplit = 1;
  if constexpr (EPI == EPI_STORE || EPI == EPI_RESID)
    gk.ksplit = kc_ksplit(g, areg);
  const int nks = (int)cdiv(g.K, KC_BK);
  const int nks2 = gk.ksplit > 1 ? ((nks + 2) & ~1) : ((nks + 1) & ~1);  // as the kernel's
  const size_t lds = (size_t)2 * (split ? 2 : 1) * C::NC * KC_KP * 2 +
                     (g.a_ln != LN_NONE ? (size_t)2 * nks2 * KC_BK * 4 : 0);
  if (lds > 64 * 1024)
    set_max_lds(reinterpret_cast<const void*>(kern), (int)lds);
  const dim3 grid((unsigned)cdiv(g.M, rows), (unsigned)(g.N / C::NC), (unsigned)gk.ksplit);
  hipLaunchKernelGGL(kern, grid, dim3(nthr), lds, s, gk);
  if constexpr (EPI == EPI_STORE || EPI == EPI_RESID) {
    if (gk.ksplit > 1) {
      const int64_t n = g.M * (g.N / 4);
      hipLaunchKernelGGL(gemm_kc_reduce_kernel<EPI>, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, gk);
    }
  }
}

template <int MAP, int EPI>
static void dispatch_kc(int nt, const GemmArgs& g, hipStream_t s) {
  switch (nt) {
    case 24: go_kc<24, MAP, EPI>(g, s); break;
    case 12: go_kc<12, MAP, EPI>(g, s); break;
    case 8: go_kc<8, MAP, EPI>(g, s); break;
    case 6: go_kc<6, MAP, EPI>(g, s); break;
    case 4: go_kc<4, MAP, EPI>(g, s); break;
    case 3: go_kc<3, MAP, EPI>(g, s); break;
    case 2: go_kc<2, MAP, EPI>(g, s); break;
    default: go_kc<1, MAP, EPI>(g, s); break;
  }
}

// column tiles per workgroup gemm_kc would use for g (0: it does not take the shape)
int gemm_kc_pick_nt(const GemmArgs& g) {
  if (g.N % 32 != 0 || g.K < 8 || g.M >= ((int64_t)1 << 31)) return 0;
  const bool known = (g.a_map == MAP_WINDOW && g.epi == EPI_STORE) ||
                     (g.a_map == MAP_IDENTITY) || (g.a_map == MAP_MERGE && g.epi == EPI_STORE);
  if (!known) return 0;
  const int tiles = g.N / 16;
  static const int cand[] = {24, 12, 8, 6, 4, 3, 2, 1};
  // narrowest chunk the small-M search may go down to (WF_KC_MINNT, A/B; round 1-4: 3)
  static const char* env_minnt = getenv("WF_KC_MINNT");
  int minnt = env_minnt ? std::max(1, atoi(env_minnt)) : 3;
  // loaders with a costly A transform (the fc's LayerNorm + GELU, the window gather + LN of qkv)
  // redo it per column chunk: at N >= 384 (8+ chunks of 3 tiles) 6-tile chunks halve that work
  // (stage-4 qkv 52.3 -> 39.0 us, the 576-column qkv 16.1 -> 13.4 us; plain loaders measured
  // slower with fewer chunks, profiles/r6/r6ks2_ab.txt)
  if (!env_minnt && (g.a_gelu || g.a_map == MAP_WINDOW) && g.N >= 384) minnt = 6;
  // the split-K fc (kc_ksplit: GELU loader, K >= 1536, caller scratch): the widest chunk up to
  // 12 tiles -- 2 chunks of 192 at stage 4, 256 workgroups with the 4 k splits: 55.5 -> 48.0 us
  // per B = 8 launch against 6 tiles; at stage 3 (no split) one 12-tile chunk measured 71 -> 73.5
  // (profiles/r6/r6ks4_ab.txt)
  const bool fc_wide = g.a_gelu && g.kpart && g.K >= 1536 && store32(g.prec) && !g.a_bf16;
  // widest column chunk that divides N (fewest re-reads of A); then, for small M, narrower
  // chunks until the grid has ~2 workgroups per CU (the K loop is a serial chain per workgroup)
  auto blocks = [&](int c) { return cdiv(g.M, 128) * (tiles / c); };
  int nt = 0;
  // with fp32 activations (PREC_SPLIT / PREC_FP16) NT = 12 / 24 need 150-210 VGPRs (two or
  // three waves per SIMD) -- at most 8 column tiles (<= 136 VGPRs) and the A rows re-read per
  // chunk from L2 instead
  const int ntmax = fc_wide ? 12 : (g.epi != EPI_LN_GELU && store32(g.prec) && !g.a_bf16) ? 8 : 24;
  for (int c : cand) {
    if (tiles % c != 0 || c > ntmax) continue;
    if (g.epi == EPI_LN_GELU && c != tiles) continue;  // LayerNorm needs the full row
    if (nt == 0 || (g.epi != EPI_LN_GELU && !fc_wide && blocks(nt) < 512 &&
                    c >= minnt))
      nt = c;
    if (blocks(nt) >= 512) break;
  }
  return nt;
}

int try_launch_gemm_kc(const GemmArgs& g, hipStream_t s) {
  const int nt = gemm_kc_pick_nt(g);
  if (nt == 0) return 0;
  if (g.a_map == MAP_WINDOW) dispatch_kc<MAP_WINDOW, EPI_STORE>(nt, g, s);
  else if (g.a_map == MAP_MERGE) dispatch_kc<MAP_MERGE, EPI_STORE>(nt, g, s);
  else if (g.epi == EPI_LN_GELU) dispatch_kc<MAP_IDENTITY, EPI_LN_GELU>(nt, g, s);
  else if (g.epi == EPI_RESID) dispatch_kc<MAP_IDENTITY, EPI_RESID>(nt, g, s);
  else dispatch_kc<MAP_IDENTITY, EPI_STORE>(nt, g, s);
  return 1;
}

}  // namespace wf
