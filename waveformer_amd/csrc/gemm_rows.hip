// gemm_rows.hip -- streaming MFMA GEMM for the large-M, small-K/N Linear layers of the path.
//
// out[m, n] = epilogue( sum_k A[m, k] * Wt[n, k] ),   M = positions (up to B * 64^3),
// K, N <= a few hundred.  The weights are tiny and the rows are many, so the kernel is built
// around streaming A exactly once from HBM:
//   * a 512-thread workgroup stages one column chunk of Wt (bf16 hi [+ lo] planes, NT*16
//     columns x K) in LDS once, then its 8 waves walk 16-row tiles of A persistently;
//   * a wave loads its A fragments straight from global memory into registers (lane l: row
//     l&15, k = 8*(l>>4) .. +7 of each 32-deep k step), applies the row gather / LayerNorm /
//     bf16 hi-lo split on the fly, and issues NT v_mfma_f32_16x16x32_bf16 (x3 for PREC_SPLIT; the _f16 form for PREC_FP16)
//     per k step against B fragments read from LDS with ds_read_b128;
//   * the epilogue runs on the accumulators in registers (C layout: lane l holds rows
//     4*(l>>4)+i, column l&15 of each 16-wide tile): bias, LayerNorm over the full row
//     (16-lane xor shuffles) + GELU, or the Block residual; stores go straight to HBM.
// Every load in the hot loops is unconditional (clamped address, then a select): a branch
// around a load makes hipcc wait vmcnt(0) for it and serialises the stream.  The row map
// (identity / window gather / PatchMerging gather) and the epilogue are template parameters
// so each call site compiles to straight-line code with 32-bit index math.
#include "gemm_common.hpp"
// cache policy of the staged (1-KB-per-instruction) output stores: 0 default, 2 nt (A/B)
#ifndef WF_ROWS_STORE_POLICY
#define WF_ROWS_STORE_POLICY 0
#endif

#ifndef WF_ROWS_DBG  // 1: timing-experiment build (GemmArgs::dbg phase skips; never the shipped library)
#define WF_ROWS_DBG 0
#endif

namespace wf {

// NTH = 768 (LN + GELU epilogue with fp32 output; WF_GEMM_ROWS_12W=0 for the 8-wave one): 12 waves per
// workgroup, three per SIMD -- the epilogue's LayerNorm / GELU VALU work needs three waves to
// reach the SIMD's issue rate (tools/ubench_valu.hip); the output restaging then goes through
// LDS 8 rows at a time so 12 waves' staging buffers fit next to the weight chunk
template <int NT, int P, int MAP, int EPI, bool ABF16, int NTH = 512>
__global__ __launch_bounds__(NTH) void gemm_rows_kernel(GemmArgs g) {
  constexpr bool SPLIT = P == PREC_SPLIT;  // P: Prec (operand kind)
  extern __shared__ __attribute__((aligned(16))) uint16_t Wl[];  // [NB][NT*16][KP]
  const int K = g.K, N = g.N;
  const int M = (int)g.M;
  // LN+GELU epilogue call sites (CCF_FFN pwconv) load with given stats or none
  const int a_ln = EPI == EPI_LN_GELU ? (g.a_ln == LN_GIVEN ? LN_GIVEN : LN_NONE) : g.a_ln;
  const int a_gelu = EPI == EPI_LN_GELU ? 0 : g.a_gelu;
  const int K32 = (K + 31) & ~31;
  const int KP = K32 + WF_LDS_KPAD;
  constexpr int NCOL = NT * 16;
  const int c0 = blockIdx.y * NCOL;  // first column of this chunk
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g4 = lane >> 4;

  // ---- stage the weight chunk (zero-padded rows >= N and k >= K)
  {
    const int kc = K32 / 8;
    for (int it = tid; it < NCOL * kc; it += blockDim.x) {
      const int r = it / kc, ch = it - r * kc;
      const int n = c0 + r;
      const bool ok = n < N && ch * 8 < K;
      const int64_t off = (int64_t)min(n, N - 1) * K + min(ch * 8, K - 8);
      const bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      const bf16x8 hv = *reinterpret_cast<const bf16x8*>(g.w + off);
      *reinterpret_cast<bf16x8*>(Wl + r * KP + ch * 8) = ok ? hv : z;
      if (SPLIT) {
        const bf16x8 lv = *reinterpret_cast<const bf16x8*>(g.w + (int64_t)N * K + off);
        *reinterpret_cast<bf16x8*>(Wl + (NCOL + r) * KP + ch * 8) = ok ? lv : z;
      }
    }
  }
  // the loader's LayerNorm gamma/beta [K32] and the epilogue's bias / LN gamma / LN beta
  // [NCOL] live in LDS: read from global inside the loops they would sit on the in-order
  // vmcnt behind the A prefetch and drain it at every k step
  float* lnw = reinterpret_cast<float*>(Wl + (SPLIT ? 2 : 1) * NCOL * KP);
  float* lnb = lnw + K32;
  float* ebias = lnb + K32;
  float* elw = ebias + NCOL;
  float* elb = elw + NCOL;
  // fp32 W2 output restaged per wave in LDS so each store instruction writes 1 KB of the
  // tile's 16 contiguous rows (the accumulator layout writes 16 rows x 64 B per instruction)
  constexpr bool STAGE = EPI == EPI_LN_GELU && P != PREC_BF16;
  constexpr int OST = NCOL + 4;  // staged row stride in floats (16-B pad)
  constexpr int SROWS = NTH > 512 ? 8 : 16;  // rows staged per pass
  float* ostg = elb + NCOL + (STAGE ? (threadIdx.x >> 6) * SROWS * OST : 0);
  for (int i = tid; i < K32; i += blockDim.x) {
    const bool ok = a_ln != LN_NONE && i < K;
    lnw[i] = ok ? g.a_ln_w[i] : 0.f;
    lnb[i] = ok ? g.a_ln_b[i] : 0.f;
  }
  for (int i = tid; i < NCOL; i += blockDim.x) {
    const int n = c0 + i;
    const int nb = EPI == EPI_SUBVOXEL ? n % (N >> 3) : n;  // sub-voxel columns share a bias
    ebias[i] = (g.bias && n < N) ? g.bias[nb] : 0.f;
    const bool e = EPI == EPI_LN_GELU && n < N;
    elw[i] = e ? 0.5f * g.e_ln_w[n] : 0.f;  // half: the epilogue feeds gelu_half2
    elb[i] = e ? 0.5f * g.e_ln_b[n] : 0.f;
  }
  __syncthreads();

  const int ntiles = (M + 15) >> 4;
  const int nwaves = blockDim.x >> 6;
  const int stride = gridDim.x * nwaves;
  // the first A fragment (and LN_GIVEN stats) of a wave's NEXT tile are loaded during the
  // current tile's last k step, so they are in flight through its epilogue
  int tile = blockIdx.x * nwaves + wid;
  int arow_c = min(tile * 16 + l15, M - 1);
  // EPI_SUBVOXEL: position offset (dz, dy, dx) and channel of each of this lane's 4-column
  // groups -- tile-invariant, so the column -> sub-voxel division runs once per kernel
  int sv_off[NT], sv_col[NT];
  if constexpr (EPI == EPI_SUBVOXEL) {
    const int Cs = N >> 3, W2 = 2 * g.mW, H2 = 2 * g.mH;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = c0 + t * 16 + 4 * g4;
      const int s = col / Cs;
      sv_col[t] = col - s * Cs;
      sv_off[t] = ((s >> 2) * H2 + ((s >> 1) & 1)) * W2 + (s & 1);
    }
  }
  RowMapper<MAP> rm(g, arow_c);
  // LN + GELU (CCF_FFN pwconv, K <= 64): BOTH k steps of the next tile are loaded at the top of
  // the current one, ahead of its epilogue stores.  vmcnt counts stores too and retires in
  // order, so a load issued after a tile's 12 stores could only be waited for together with
  // them: the one-step prefetch made every tile wait out the previous tile's write latency
  // (without the stores the kernel ran 341 instead of 567 us at B = 8)
  constexpr bool W2 = EPI == EPI_LN_GELU;
  // output descriptor of the W2 stores: M rows of ldo elements (host: < 2^31 bytes)
  const bool obf_ = EPI == EPI_LN_GELU ? P == PREC_BF16 : false;
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
      g.out, 0, W2 ? (int)((int64_t)M * g.ldo * (obf_ ? 2 : 4)) : 0, 0x00020000);
  float vn[8], vn1[8];
  load8f<ABF16>(g.a_src, rm.offset(g, min(8 * g4, K - 8)), vn);
  if (W2) load8f<ABF16>(g.a_src, rm.offset(g, min(32 + 8 * g4, K - 8)), vn1);
  float gmean = 0.f, grstd = 1.f;
  if (a_ln == LN_GIVEN) {
    gmean = g.a_stats[2 * arow_c];
    grstd = g.a_stats[2 * arow_c + 1];
  }
  for (; tile < ntiles; tile += stride) {
    // ---- A rows of this lane: row l15 of the tile (and of the next one)
    const int arow_n = min((tile + stride) * 16 + l15, M - 1);
    const RowMapper<MAP> rmn(g, arow_n);
    float mean = gmean, rstd = grstd;
    if (a_ln == LN_COMPUTE) {  // lanes l15, l15+16, l15+32, l15+48 share the row
      // two passes, each issuing its loads four octets at a time (a load per iteration waited
      // out one latency per octet); same summation order, clamped tail octets add 0
      const int noct = K / 8;
      float s = 0.f;
      for (int cb = g4; cb < noct; cb += 16) {
        float v[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) load8f<ABF16>(g.a_src, rm.offset(g, min(cb + 4 * u, noct - 1) * 8), v[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float mk = cb + 4 * u < noct ? 1.f : 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) s += v[u][j] * mk;
        }
      }
      s = xsum16(s);
      s = xsum32(s);
      mean = s / (float)K;
      float q = 0.f;
      for (int cb = g4; cb < noct; cb += 16) {
        float v[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) load8f<ABF16>(g.a_src, rm.offset(g, min(cb + 4 * u, noct - 1) * 8), v[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float mk = cb + 4 * u < noct ? 1.f : 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float d = (v[u][j] - mean) * mk;
            q += d * d;
          }
        }
      }
      q = xsum16(q);
      q = xsum32(q);
      rstd = rsqrtf(q / (float)K + g.a_eps);
    } else if (a_ln == LN_PARTIAL) {  // combine the producer's per-group {mean, M2}
      const int np = g.a_np;
      const float* ps = g.a_stats + (int64_t)arow_c * np * 2;
      float s = 0.f;
      for (int c = g4; c < np; c += 4) s += ps[2 * c];
      s = xsum16(s);
      s = xsum32(s);
      mean = s / (float)np;
      const float ng = (float)(K / np);
      float q = 0.f;
      for (int c = g4; c < np; c += 4) {
        const float d = ps[2 * c] - mean;
        q += ps[2 * c + 1] + ng * d * d;
      }
      q = xsum16(q);
      q = xsum32(q);
      rstd = rsqrtf(q / (float)K + g.a_eps);
    }

    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0, 0, 0, 0};

    // one 32-deep k step on the A fragment v (LayerNorm / GELU / split in the loader)
    auto kstep = [&](int k0, float* v) {
      const int k = k0 + 8 * g4;
      const bool kv = k < K;
      if (a_ln != LN_NONE) {
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(lnw + k);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(lnw + k + 4);
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(lnb + k);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(lnb + k + 4);
        const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (v[j] - mean) * rstd * wv[j] + bv[j];
      }
      if (a_gelu) {
        gelu_erf8(v);
      }
      bf16x8 ah, al;
      {
        float xs[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) xs[j] = kv ? v[j] : 0.f;
        split8<P>(xs, ah, al);
      }
      // transposed product C^T = Wt . A^T: the weight fragment is the A operand (rows =
      // output channels), the activation fragment the B operand (columns = positions), so
      // the accumulator gives each lane 4 CONSECUTIVE channels of one position.
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int wo = (t * 16 + l15) * KP + k0 + 8 * g4;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Wl + wo);
        if (SPLIT) {
          const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Wl + NCOL * KP + wo);
          acc[t] = mma32<P>(bh, al, acc[t]);
          acc[t] = mma32<P>(bl, ah, acc[t]);
        }
        acc[t] = mma32<P>(bh, ah, acc[t]);
        // keep the LDS fragment reads from being hoisted all at once (VGPR pressure ->
        // occupancy): a scheduling fence every 3 tiles
        if (t % 3 == 2) __builtin_amdgcn_sched_barrier(0);
      }
    };

    if constexpr (W2) {
      float v0[8], v1[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v0[j] = vn[j];
        v1[j] = vn1[j];
      }
      load8f<ABF16>(g.a_src, rmn.offset(g, min(8 * g4, K - 8)), vn);
      load8f<ABF16>(g.a_src, rmn.offset(g, min(32 + 8 * g4, K - 8)), vn1);
      if (a_ln == LN_GIVEN) {
        gmean = g.a_stats[2 * arow_n];
        grstd = g.a_stats[2 * arow_n + 1];
      }
#if WF_ROWS_DBG
      if (!(g.dbg & 4)) {
#endif
      kstep(0, v0);
      if (K32 > 32) kstep(32, v1);
#if WF_ROWS_DBG
      }
#endif
    } else {
      // k loop with a one-step register prefetch of the A fragment (last step: the next tile's)
#pragma unroll 1
      for (int k0 = 0; k0 < K32; k0 += 32) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = vn[j];
        const int64_t noff = k0 + 32 < K32 ? rm.offset(g, min(k0 + 32 + 8 * g4, K - 8))
                                           : rmn.offset(g, min(8 * g4, K - 8));
        load8f<ABF16>(g.a_src, noff, vn);
        kstep(k0, v);
      }
    }

    if (!W2 && a_ln == LN_GIVEN) {  // next tile's stats, in flight through the epilogue
      gmean = g.a_stats[2 * arow_n];
      grstd = g.a_stats[2 * arow_n + 1];
    }

    // ---- epilogue: acc[t][i] = out[position tile*16 + l15][channel c0 + t*16 + 4*g4 + i]
    const int row = tile * 16 + l15;
    const bool rv = row < M;
    const int rowc = min(row, M - 1);
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] += *reinterpret_cast<const f32x4*>(ebias + t * 16 + 4 * g4);
    float rm_ = 0.f, rs_ = 1.f, bs = 1.f;
    int64_t sv_p0 = 0;  // EPI_SUBVOXEL: output position of sub-voxel (0, 0, 0) of this row
    if (EPI == EPI_SUBVOXEL) {
      int r = rowc;
      const int x = r % g.mW;
      r /= g.mW;
      const int y = r % g.mH;
      r /= g.mH;
      const int z = r % g.mD, b = r / g.mD;
      sv_p0 = (((int64_t)b * 2 * g.mD + 2 * z) * (2 * g.mH) + 2 * y) * (2 * g.mW) + 2 * x;
    }
    if (EPI == EPI_LN_GELU) {  // full row in this wave (NCOL == N): the 4 lanes of a position
      // moments on f32x2 pairs straight off the accumulator registers (.xy / .zw: no
      // repacking moves; scalar v_add / v_fma pairs in this build)
      f32x2 s2 = {0.f, 0.f};
#pragma unroll
      for (int t = 0; t < NT; ++t) s2 += lo2(acc[t]) + hi2(acc[t]);
      float s = s2.x + s2.y;
      s = xsum16(s);
      s = xsum32(s);
      rm_ = s / (float)N;
      f32x2 q2 = {0.f, 0.f};
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f32x2 d0 = lo2(acc[t]) - rm_, d1 = hi2(acc[t]) - rm_;
        q2 = d0 * d0 + q2;
        q2 = d1 * d1 + q2;
      }
      float q = q2.x + q2.y;
      q = xsum16(q);
      q = xsum32(q);
      rs_ = rsqrtf(q / (float)N + g.e_eps);
    } else if (EPI == EPI_RESID) {
      if (g.r_stats) {
        rm_ = g.r_stats[2 * rowc];
        rs_ = g.r_stats[2 * rowc + 1];
      }
      if (g.r_scale) bs = g.r_scale[rowc / (int)g.rows_per_sample];
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = c0 + t * 16 + 4 * g4;
      const int colc = min(col, N - 4);
      f32x4 v = acc[t];
#if WF_ROWS_DBG
      if (EPI == EPI_LN_GELU && !(g.dbg & 2)) {
#else
      if (EPI == EPI_LN_GELU) {
#endif
        // elw / elb hold HALF the LayerNorm affine (staged x 0.5, exact): the normalised
        // value comes out as GELU's half input; (v - mean) * rstd as one FMA per pair
        const f32x4 lw = *reinterpret_cast<const f32x4*>(elw + t * 16 + 4 * g4);
        const f32x4 lb = *reinterpret_cast<const f32x4*>(elb + t * 16 + 4 * g4);
        const float nb = -rm_ * rs_;
        const f32x2 u0 = lo2(v) * rs_ + nb, u1 = hi2(v) * rs_ + nb;
        const f32x2 h0 = gelu_half2(u0 * lo2(lw) + lo2(lb));
        const f32x2 h1 = gelu_half2(u1 * hi2(lw) + hi2(lb));
        v = f32x4{h0.x, h0.y, h1.x, h1.y};
      } else if (EPI == EPI_RESID) {
        const f32x4 xr = *reinterpret_cast<const f32x4*>(g.r_x + (int64_t)rowc * N + colc);
        if (g.r_stats) {
          const f32x4 lw = *reinterpret_cast<const f32x4*>(g.r_ln_w + colc);
          const f32x4 lb = *reinterpret_cast<const f32x4*>(g.r_ln_b + colc);
          const f32x4 n2 = (xr - rm_) * rs_ * lw + lb;
          v = xr + (n2 + v) * bs;  // attn_fused + drop_path(n2 + ffn(n2)), quirk Q4
        } else {
          v = xr + v * bs;         // bare CCF_FFN.forward: x + x_out
        }
      }
      // LN+GELU (CCF_FFN pwconv): the chunk is the whole row and the storage type follows
      // the precision, so the store needs no column test and no runtime type branch
      const bool cv = EPI == EPI_LN_GELU ? true : col < N;
      const bool obf = EPI == EPI_LN_GELU ? P == PREC_BF16 : g.out_bf16 != 0;
      if constexpr (W2) {
        // range-checked buffer store (rows >= M dropped by the descriptor): no exec branch,
        // so the compiler can count these stores and wait for the next tile's loads only
        if (obf) {
          bf16x4 o;
          o[0] = (short)f2bf(v.x);
          o[1] = (short)f2bf(v.y);
          o[2] = (short)f2bf(v.z);
          o[3] = (short)f2bf(v.w);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), orsrc,
                                                (int)((row * g.ldo + col) * 2), 0, 0);
        } else if (STAGE) {
          if constexpr (SROWS == 16)
            *reinterpret_cast<f32x4*>(ostg + l15 * OST + t * 16 + 4 * g4) = v;
          else
            acc[t] = v;  // staged below, 8 rows per pass
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), orsrc,
                                                 (int)((row * g.ldo + col) * 4), 0, 0);
        }
      } else if (EPI == EPI_SUBVOXEL) {
        if (rv)
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(g.out) +
                                    (sv_p0 + sv_off[t]) * g.ldo + sv_col[t]) = v;
      } else if (rv && cv) {
        if (obf) {
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
      if (t % 2 == 1) __builtin_amdgcn_sched_barrier(0);  // bound load hoisting (VGPRs)
    }
    if constexpr (STAGE) {
      // one wave's LDS operations complete in issue order; the fences only keep the compiler
      // from moving the lanes' exchange
      constexpr int RC = NCOL / 4;  // 16-B chunks per row
#pragma unroll
      for (int half = 0; half < 16 / SROWS; ++half) {
        if constexpr (SROWS < 16) {
          if ((l15 >> 3) == half) {
#pragma unroll
            for (int t = 0; t < NT; ++t)
              *reinterpret_cast<f32x4*>(ostg + (l15 & 7) * OST + t * 16 + 4 * g4) = acc[t];
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int j = 0; j < SROWS * RC / 64; ++j) {
          const int c = j * 64 + lane, r = c / RC, c4 = c - r * RC;
          const f32x4 v = *reinterpret_cast<const f32x4*>(ostg + r * OST + 4 * c4);
#if WF_ROWS_DBG
          const int doff = (g.dbg & 1) ? 0x7fffff00 : 0;  // past the descriptor: dropped
#else
          constexpr int doff = 0;
#endif
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(u32x4, v), orsrc,
              doff + (int)(((tile * 16 + half * SROWS + r) * g.ldo + 4 * c4) * 4), 0,
              WF_ROWS_STORE_POLICY);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
    arow_c = arow_n;
    rm = rmn;
  }
}

// the 12-wave LN + GELU variant (fp32 output, identity rows): default since round 4 (446 vs
// 452-453 us per stage-1 launch at B = 8); WF_GEMM_ROWS_12W=0 for the 8-wave one
static bool rows_w12(const GemmArgs& g) {
  static const bool w12 = getenv("WF_GEMM_ROWS_12W") == nullptr || getenv("WF_GEMM_ROWS_12W")[0] != '0';
  return w12 && g.epi == EPI_LN_GELU && g.a_map == MAP_IDENTITY && !g.a_bf16 && g.prec != PREC_BF16;
}

template <int NT, int MAP, int EPI>
static void go_rows(const GemmArgs& g0, dim3 grid, size_t lds, hipStream_t s) {
  GemmArgs g = g0;
  g.dbg = WF_ROWS_DBG && getenv("WF_ROWS_DBG") ? atoi(getenv("WF_ROWS_DBG")) : 0;
  void (*kern)(GemmArgs);
  if constexpr (EPI == EPI_LN_GELU && MAP == MAP_IDENTITY) {
    if (rows_w12(g)) {  // lds already holds the 12 x 8-row output staging (host below)
      kern = g.prec == PREC_SPLIT ? gemm_rows_kernel<NT, PREC_SPLIT, MAP, EPI, false, 768>
                                  : gemm_rows_kernel<NT, PREC_FP16, MAP, EPI, false, 768>;
      set_max_lds(reinterpret_cast<const void*>(kern), (int)lds);
      const unsigned gx = (unsigned)std::min<int64_t>(cdiv((g.M + 15) / 16, 12), 256);
      hipLaunchKernelGGL(kern, dim3(gx, grid.y), dim3(768), lds, s, g);
      return;
    }
  }
  if (g.a_bf16)  // bf16 activations only exist in PREC_BF16
    kern = gemm_rows_kernel<NT, PREC_BF16, MAP, EPI, true>;
  else if (g.prec == PREC_SPLIT)
    kern = gemm_rows_kernel<NT, PREC_SPLIT, MAP, EPI, false>;
  else if (g.prec == PREC_FP16)
    kern = gemm_rows_kernel<NT, PREC_FP16, MAP, EPI, false>;
  else
    kern = gemm_rows_kernel<NT, PREC_BF16, MAP, EPI, false>;
  if (lds > 64 * 1024)
    set_max_lds(reinterpret_cast<const void*>(kern), (int)lds);
  hipLaunchKernelGGL(kern, grid, dim3(512), lds, s, g);
}

template <int MAP, int EPI>
static void dispatch_nt(int nt, const GemmArgs& g, dim3 grid, size_t lds, hipStream_t s) {
  switch (nt) {
    case 12: go_rows<12, MAP, EPI>(g, grid, lds, s); break;
    case 9: go_rows<9, MAP, EPI>(g, grid, lds, s); break;
    case 8: go_rows<8, MAP, EPI>(g, grid, lds, s); break;
    case 6: go_rows<6, MAP, EPI>(g, grid, lds, s); break;
    case 4: go_rows<4, MAP, EPI>(g, grid, lds, s); break;
    case 3: go_rows<3, MAP, EPI>(g, grid, lds, s); break;
    case 2: go_rows<2, MAP, EPI>(g, grid, lds, s); break;
    default: go_rows<1, MAP, EPI>(g, grid, lds, s); break;
  }
}

int try_launch_gemm_rows(const GemmArgs& g, hipStream_t s, bool single_chunk_only) {
  if (g.N % 16 != 0 || g.K < 8 || g.M >= ((int64_t)1 << 31)) return 0;
  // call-site shapes (the others fall back to gemm_ares): window qkv, identity store/LN/resid,
  // PatchMerging gather
  const bool known = (g.a_map == MAP_WINDOW && g.epi == EPI_STORE) ||
                     (g.a_map == MAP_IDENTITY) || (g.a_map == MAP_MERGE && g.epi == EPI_STORE);
  if (!known) return 0;
  // the LN+GELU instantiations are specialised to the CCF_FFN pwconv's loader and storage
  const int64_t out_bytes = g.M * g.ldo * ((g.prec == PREC_BF16 || g.a_bf16) ? 2 : 4);
  if (g.epi == EPI_LN_GELU && (g.K > 64 || out_bytes >= ((int64_t)1 << 31) || (g.a_ln != LN_GIVEN && g.a_ln != LN_NONE) || g.a_gelu ||
                               (g.out_bf16 != 0) != (g.prec == PREC_BF16 || g.a_bf16 != 0)))
    return 0;
  if (g.epi == EPI_SUBVOXEL && (g.out_bf16 || (g.N / 8) % 4 != 0 || g.a_map != MAP_IDENTITY))
    return 0;
  const bool split = g.prec == PREC_SPLIT;
  const int K32 = (g.K + 31) & ~31;
  const size_t per_col = (size_t)(split ? 2 : 1) * (K32 + WF_LDS_KPAD) * 2;
  const int tiles = g.N / 16;
  static const int cand[] = {12, 9, 8, 6, 4, 3, 2, 1};
  // the transposed conv's N = 8 Cout is wide: one workgroup per CU holding half the columns
  // reads A twice instead of six times at 64 KB
  // WF_ROWS_WIDE=1 (A/B): PatchMerging's whole 8C -> 2C weight (150 KB at 1 -> 2) resident in
  // one workgroup per CU, persistent over row tiles, no barrier in the k loop (gemm_kc streams
  // the weight through LDS a k-step at a time)
  static const bool wide = getenv("WF_ROWS_WIDE") && getenv("WF_ROWS_WIDE")[0] == '1';
  const size_t wbudget = g.epi == EPI_SUBVOXEL ? 136 * 1024
                         : (wide && g.a_map == MAP_MERGE) ? 152 * 1024 : 64 * 1024;
  int nt = 0;
  for (int c : cand) {
    if (tiles % c != 0) continue;
    if (g.epi == EPI_LN_GELU && c != tiles) continue;  // LayerNorm needs the full row
    if ((size_t)c * 16 * per_col <= wbudget) {
      nt = c;
      break;
    }
  }
  if (nt == 0) return 0;
  size_t lds = (size_t)nt * 16 * per_col + (size_t)(2 * K32 + 3 * nt * 16) * 4;
  if (g.epi == EPI_LN_GELU && g.prec != PREC_BF16 && !g.a_bf16)  // output staging per wave
    lds += (size_t)(rows_w12(g) ? 12 * 8 : 8 * 16) * (nt * 16 + 4) * 4;
  if (lds > 160 * 1024) return 0;
  const int chunks = tiles / nt;
  if (single_chunk_only && chunks > 1) return 0;
  const int64_t ntiles = (g.M + 15) / 16;
  int64_t gx = cdiv(ntiles, 8);
  // ~2 workgroups of 8 waves per CU; one per CU when the weight chunk fills the LDS
  const int64_t cap = lds > 80 * 1024 ? 256 : (512 + chunks - 1) / chunks;
  if (gx > cap) gx = cap;
  if (gx < 1) gx = 1;
  dim3 grid((unsigned)gx, (unsigned)chunks);
  if (g.a_map == MAP_WINDOW) dispatch_nt<MAP_WINDOW, EPI_STORE>(nt, g, grid, lds, s);
  else if (g.a_map == MAP_MERGE) dispatch_nt<MAP_MERGE, EPI_STORE>(nt, g, grid, lds, s);
  else if (g.epi == EPI_LN_GELU) dispatch_nt<MAP_IDENTITY, EPI_LN_GELU>(nt, g, grid, lds, s);
  else if (g.epi == EPI_RESID) dispatch_nt<MAP_IDENTITY, EPI_RESID>(nt, g, grid, lds, s);
  else if (g.epi == EPI_SUBVOXEL) dispatch_nt<MAP_IDENTITY, EPI_SUBVOXEL>(nt, g, grid, lds, s);
  else dispatch_nt<MAP_IDENTITY, EPI_STORE>(nt, g, grid, lds, s);
  return 1;
}

}  // namespace wf
