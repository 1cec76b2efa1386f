// gemm.hip -- the A-resident bf16 MFMA GEMM behind every Linear / 1x1x1 Conv3d of the path.
//
//   qkv   (attention.py:87, with window_partition wave_helper.py:450-461 and norm1 folded in)
//   proj  (attention.py:102)
//   pwconv (wave_helper.py:278) + LN(4C) + GELU (:279) folded into the epilogue
//   fc    (wave_helper.py:289) + the Block's double residual (:293 and :509, quirk Q4)
//   PatchMerging gather + LN(8C) + reduction (wave_helper.py:183-193, quirk Q3)
//
// Structure (one 256-thread workgroup = BM rows x all N columns):
//   1. loader: the BM source rows (gathered, optionally LayerNorm'ed in fp32) are rounded to
//      bf16 into an LDS tile A[BM][KP] (plus the residual tile A_lo for PREC_SPLIT) -- A is
//      read from HBM exactly once.
//   2. MFMA: each wave owns 16 columns of a 64-column chunk; per 32-deep k step it loads its
//      Wt[n][k..k+8] fragment(s) straight from L2 (the weights are at most 1.2 MB) and issues
//      BM/16 v_mfma_f32_16x16x32_bf16 (x3 for PREC_SPLIT: hi*hi + lo*hi + hi*lo) against A
//      fragments read by ds_read_b128.
//   3. the fp32 accumulators land in an LDS row buffer R[BM][N]; the epilogue then walks rows
//      (bias, LayerNorm+GELU or residual) and writes whole rows with 16-B stores.
// Roofline: for every call site K, N <= 1536 and the arithmetic intensity is far below the
// bf16 ridge point, so the kernel is HBM-bound on reading A and writing the output.
#include "kernels.hpp"

namespace wf {

__device__ __forceinline__ void load8(const void* src, int is_bf16, int64_t off, float (&v)[8]) {
  if (is_bf16) {
    bf16x8 u = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const uint16_t*>(src) + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f((uint16_t)u[j]);
  } else {
    const f32x4* p = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(src) + off);
    f32x4 a = p[0], b = p[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}

// Element offset of element k of logical row m in the source.
struct RowSource {
  const GemmArgs& g;
  int64_t pos;  // MAP_WINDOW: raster row; MAP_MERGE: (b, 2z, 2y, 2x) raster row
  __device__ RowSource(const GemmArgs& g_, int64_t m) : g(g_), pos(0) {
    if (g.a_map == MAP_WINDOW) {
      const int ws = g.mws;
      const int N = ws * ws * ws;
      const int nWd = g.mD / ws, nWh = g.mH / ws, nWw = g.mW / ws;
      const int64_t bw = m / N;
      const int t = (int)(m - bw * N);
      const int nW = nWd * nWh * nWw;
      const int b = (int)(bw / nW);
      int wi = (int)(bw - (int64_t)b * nW);
      const int wx = wi % nWw;
      wi /= nWw;
      const int wy = wi % nWh;
      const int wz = wi / nWh;
      const int tx = t % ws, ty = (t / ws) % ws, tz = t / (ws * ws);
      pos = (((int64_t)b * g.mD + wz * ws + tz) * g.mH + wy * ws + ty) * g.mW + wx * ws + tx;
    } else if (g.a_map == MAP_MERGE) {
      const int d = g.mD >> 1, h = g.mH >> 1, w = g.mW >> 1;
      int64_t r = m;
      const int x = (int)(r % w);
      r /= w;
      const int y = (int)(r % h);
      r /= h;
      const int z = (int)(r % d);
      const int b = (int)(r / d);
      pos = (((int64_t)b * g.mD + 2 * z) * g.mH + 2 * y) * g.mW + 2 * x;
    } else {
      pos = m;
    }
  }
  __device__ int64_t offset(int k) const {
    if (g.a_map == MAP_MERGE) {
      // sub-lattice order from merge_code (see wf_patch_merging_fwd)
      const int seg = k / g.a_C;
      const int c = k - seg * g.a_C;
      const int o = (g.merge_code >> (4 * seg)) & 0xF;  // bit2: d, bit1: h, bit0: w
      const int64_t p = pos + (((int64_t)((o >> 2) & 1) * g.mH + ((o >> 1) & 1)) * g.mW) +
                        (o & 1);
      return p * g.a_C + c;
    }
    return pos * (int64_t)(g.a_C * g.a_nseg) + k;
  }
};

template <int TPR>
__device__ __forceinline__ float tpr_sum(float v) {
#pragma unroll
  for (int o = TPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int BM, int P>
__global__ __launch_bounds__(256) void gemm_ares_kernel(GemmArgs g) {
  constexpr bool SPLIT = P == PREC_SPLIT;  // P: Prec (operand kind)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TPR = 256 / BM;  // threads per row in row-assigned phases
  constexpr int MT = BM / 16;
  const int K = g.K, N = g.N;
  const int K32 = (K + 31) & ~31;
  const int KP = K32 + 8;        // bf16 row stride of A (16 B pad vs bank conflicts)
  const int NP = N + 4;          // fp32 row stride of R
  const size_t abytes = ((size_t)BM * KP * 2 + 15) & ~(size_t)15;
  uint16_t* A = reinterpret_cast<uint16_t*>(smem);
  uint16_t* Alo = reinterpret_cast<uint16_t*>(smem + abytes);  // PREC_SPLIT only
  float* R = reinterpret_cast<float*>(smem + (SPLIT ? 2 : 1) * abytes);
  float* st = R + (size_t)BM * NP;  // [BM][2]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * BM;

  // ---------------- 1. A loader ----------------
  {
    const int r = tid / TPR, q = tid % TPR;
    const int64_t m = m0 + r;
    const bool mv = m < g.M;
    float mean = 0.f, rstd = 1.f;
    if (g.a_ln == LN_GIVEN) {
      if (mv) {
        mean = g.a_stats[2 * m];
        rstd = g.a_stats[2 * m + 1];
      }
    } else if (g.a_ln == LN_COMPUTE) {
      RowSource rs(g, mv ? m : 0);
      float s = 0.f;
      for (int ch = q; ch < K / 8; ch += TPR) {
        float v[8];
        load8(g.a_src, g.a_bf16, rs.offset(ch * 8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[j];
      }
      mean = tpr_sum<TPR>(s) / (float)K;
      float sq = 0.f;
      for (int ch = q; ch < K / 8; ch += TPR) {
        float v[8];
        load8(g.a_src, g.a_bf16, rs.offset(ch * 8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float dlt = v[j] - mean;
          sq += dlt * dlt;
        }
      }
      rstd = rsqrtf(tpr_sum<TPR>(sq) / (float)K + g.a_eps);
    } else if (g.a_ln == LN_PARTIAL) {  // combine the producer's per-group {mean, M2}
      const int np = g.a_np;
      const float* ps = g.a_stats + (mv ? m : 0) * np * 2;
      float s = 0.f;
      for (int c = q; c < np; c += TPR) s += ps[2 * c];
      mean = tpr_sum<TPR>(s) / (float)np;
      const float ng = (float)(K / np);
      float sq = 0.f;
      for (int c = q; c < np; c += TPR) {
        const float d = ps[2 * c] - mean;
        sq += ps[2 * c + 1] + ng * d * d;
      }
      rstd = rsqrtf(tpr_sum<TPR>(sq) / (float)K + g.a_eps);
    }
    if (q == 0) {
      st[2 * r] = mean;
      st[2 * r + 1] = rstd;
    }
  }
  __syncthreads();
  {
    const int KC = K32 / 8;  // 8-element chunks per LDS row (incl. zero tail)
    for (int item = tid; item < BM * KC; item += 256) {
      const int r = item / KC, ch = item - r * KC;
      const int64_t m = m0 + r;
      bf16x8 o = {0, 0, 0, 0, 0, 0, 0, 0}, olo = {0, 0, 0, 0, 0, 0, 0, 0};
      if (m < g.M && ch * 8 < K) {
        RowSource rs(g, m);
        float v[8];
        load8(g.a_src, g.a_bf16, rs.offset(ch * 8), v);
        if (g.a_ln != LN_NONE) {
          const float mean = st[2 * r], rstd = st[2 * r + 1];
          const f32x4* gw = reinterpret_cast<const f32x4*>(g.a_ln_w + ch * 8);
          const f32x4* gb = reinterpret_cast<const f32x4*>(g.a_ln_b + ch * 8);
          const f32x4 w0 = gw[0], w1 = gw[1], b0 = gb[0], b1 = gb[1];
          const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
          const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (v[j] - mean) * rstd * wv[j] + bv[j];
        }
        if (g.a_gelu) {
          gelu_erf8(v);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint16_t hi = op_cvt<P>(v[j]);
          o[j] = (short)hi;
          if (SPLIT) olo[j] = op_lo<P>(v[j], hi);
        }
      }
      *reinterpret_cast<bf16x8*>(A + (size_t)r * KP + ch * 8) = o;
      if (SPLIT) *reinterpret_cast<bf16x8*>(Alo + (size_t)r * KP + ch * 8) = olo;
    }
  }
  __syncthreads();

  // ---------------- 2. MFMA over 64-column chunks ----------------
  const int kq = 8 * (lane >> 4);
  for (int n0 = 0; n0 < N; n0 += 64) {
    const int n = n0 + wid * 16 + (lane & 15);
    const bool nv = n < N;
    const uint16_t* wrow = g.w + (int64_t)(nv ? n : 0) * K;
    const uint16_t* wlo = wrow + (int64_t)N * K;  // lo plane (PREC_SPLIT)
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0, 0, 0, 0};
    const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    bf16x8 bnext = z8, blnext = z8;
    if (nv && kq < K) {
      bnext = *reinterpret_cast<const bf16x8*>(wrow + kq);
      if (SPLIT) blnext = *reinterpret_cast<const bf16x8*>(wlo + kq);
    }
    for (int k0 = 0; k0 < K32; k0 += 32) {
      const bf16x8 b = bnext, bl = blnext;
      bnext = z8;
      blnext = z8;
      if (nv && k0 + 32 + kq < K) {
        bnext = *reinterpret_cast<const bf16x8*>(wrow + k0 + 32 + kq);
        if (SPLIT) blnext = *reinterpret_cast<const bf16x8*>(wlo + k0 + 32 + kq);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const size_t aoff = (size_t)(mt * 16 + (lane & 15)) * KP + k0 + kq;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + aoff);
        if (SPLIT) {
          const bf16x8 al = *reinterpret_cast<const bf16x8*>(Alo + aoff);
          acc[mt] = mma32<P>(al, b, acc[mt]);
          acc[mt] = mma32<P>(a, bl, acc[mt]);
        }
        acc[mt] = mma32<P>(a, b, acc[mt]);
      }
    }
    if (nv) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) R[(size_t)(mt * 16 + 4 * (lane >> 4) + i) * NP + n] = acc[mt][i];
    }
  }
  __syncthreads();

  // ---------------- 3. epilogue ----------------
  const int N4 = N >> 2;
  if (g.epi == EPI_LN_GELU) {  // row statistics of (acc + bias), two-pass from LDS
    const int r = tid / TPR, q = tid % TPR;
    float s = 0.f;
    for (int c4 = q; c4 < N4; c4 += TPR) {
      f32x4 v = *reinterpret_cast<const f32x4*>(R + (size_t)r * NP + 4 * c4);
      if (g.bias) v += reinterpret_cast<const f32x4*>(g.bias)[c4];
      s += (v.x + v.y) + (v.z + v.w);
    }
    const float mean = tpr_sum<TPR>(s) / (float)N;
    float sq = 0.f;
    for (int c4 = q; c4 < N4; c4 += TPR) {
      f32x4 v = *reinterpret_cast<const f32x4*>(R + (size_t)r * NP + 4 * c4);
      if (g.bias) v += reinterpret_cast<const f32x4*>(g.bias)[c4];
      v -= mean;
      sq += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
    }
    const float rstd = rsqrtf(tpr_sum<TPR>(sq) / (float)N + g.e_eps);
    __syncthreads();  // st[] may still be read by nobody, but keep phases ordered
    if (q == 0) {
      st[2 * r] = mean;
      st[2 * r + 1] = rstd;
    }
    __syncthreads();
  }
  for (int item = tid; item < BM * N4; item += 256) {
    const int r = item / N4, c4 = item - r * N4;
    const int64_t m = m0 + r;
    if (m >= g.M) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(R + (size_t)r * NP + 4 * c4);
    if (g.bias) v += reinterpret_cast<const f32x4*>(g.bias)[c4];
    if (g.epi == EPI_LN_GELU) {
      const f32x4 lw = reinterpret_cast<const f32x4*>(g.e_ln_w)[c4];
      const f32x4 lb = reinterpret_cast<const f32x4*>(g.e_ln_b)[c4];
      v = (v - st[2 * r]) * st[2 * r + 1] * lw + lb;
      v = gelu_erf4(v);
    } else if (g.epi == EPI_RESID) {
      const f32x4 xr = reinterpret_cast<const f32x4*>(g.r_x + m * (int64_t)N)[c4];
      const float bs = g.r_scale ? g.r_scale[m / g.rows_per_sample] : 1.f;
      if (g.r_stats) {
        const float mean = g.r_stats[2 * m], rstd = g.r_stats[2 * m + 1];
        const f32x4 lw = reinterpret_cast<const f32x4*>(g.r_ln_w)[c4];
        const f32x4 lb = reinterpret_cast<const f32x4*>(g.r_ln_b)[c4];
        const f32x4 n2 = (xr - mean) * rstd * lw + lb;
        v = xr + (n2 + v) * bs;  // attn_fused + drop_path(n2 + ffn(n2)), quirk Q4
      } else {
        v = xr + v * bs;         // bare CCF_FFN.forward: x + x_out (wave_helper.py:293)
      }
    }
    if (g.out_bf16) {
      bf16x4 o;
      o[0] = (short)f2bf(v.x);
      o[1] = (short)f2bf(v.y);
      o[2] = (short)f2bf(v.z);
      o[3] = (short)f2bf(v.w);
      *reinterpret_cast<bf16x4*>(reinterpret_cast<uint16_t*>(g.out) + m * g.ldo + 4 * c4) = o;
    } else {
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(g.out) + m * g.ldo + 4 * c4) = v;
    }
  }
}

static size_t gemm_lds_bytes(int BM, int K, int N, bool split) {
  const size_t K32 = (size_t)((K + 31) & ~31);
  const size_t a = ((size_t)BM * (K32 + 8) * 2 + 15) & ~(size_t)15;
  return (split ? 2 : 1) * a + (size_t)BM * (N + 4) * 4 + (size_t)BM * 2 * 4;
}

int launch_gemm(const GemmArgs& g, hipStream_t s, const char* who) {
  if (g.K <= 0 || g.K % 8 != 0) return fail(WF_E_SHAPE, std::string(who) + ": K must be a positive multiple of 8");
  if (g.N <= 0 || g.N % 4 != 0) return fail(WF_E_SHAPE, std::string(who) + ": N must be a positive multiple of 4");
  if (g.a_C % 8 != 0) return fail(WF_E_SHAPE, std::string(who) + ": channels must be a multiple of 8");
  if (g.M <= 0) return WF_OK;
  // streaming kernels first: gemm_rows when one LDS-resident weight chunk covers all N,
  // else the K-chunked gemm_kc (WF_GEMM_NO_KC: gemm_rows over several column chunks); the A-resident
  // gemm_ares takes the remaining shapes.  (WF_GEMM_ARES_ONLY / WF_GEMM_NO_KC: A/B switches)
  static const bool ares_only = getenv("WF_GEMM_ARES_ONLY") != nullptr;
  static const bool no_kc = getenv("WF_GEMM_NO_KC") != nullptr;
  if (g.o_pstats) {  // LayerNorm partials in the epilogue: gemm_kc only
    if (g.epi == EPI_STORE && !g.out_bf16 && !g.a_bf16 && try_launch_gemm_kc(g, s))
      return check_launch(who);
    return fail(WF_E_SHAPE, std::string(who) + ": LN-partial epilogue needs the gemm_kc shape");
  }
  if (!ares_only) {
    if (try_launch_gemm_lnw(g, s)) return check_launch(who);
    if (try_launch_gemm_rows(g, s, !no_kc)) return check_launch(who);
    if (!no_kc && try_launch_gemm_kc(g, s)) return check_launch(who);
  }
  const bool split = g.prec == PREC_SPLIT;
  int BM = 64;
  while (BM > 16 && gemm_lds_bytes(BM, g.K, g.N, split) > 80 * 1024) BM >>= 1;
  const size_t lds = gemm_lds_bytes(BM, g.K, g.N, split);
  if (lds > 160 * 1024) return fail(WF_E_SHAPE, std::string(who) + ": K/N too large for the LDS tile");
  const unsigned blocks = (unsigned)cdiv(g.M, BM);
  auto go = [&](auto kern) {
    if (lds > 64 * 1024)
      set_max_lds(reinterpret_cast<const void*>(kern), (int)lds);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, s, g);
  };
  if (split) {
    switch (BM) {
      case 64: go(gemm_ares_kernel<64, PREC_SPLIT>); break;
      case 32: go(gemm_ares_kernel<32, PREC_SPLIT>); break;
      default: go(gemm_ares_kernel<16, PREC_SPLIT>); break;
    }
  } else if (g.prec == PREC_FP16) {
    switch (BM) {
      case 64: go(gemm_ares_kernel<64, PREC_FP16>); break;
      case 32: go(gemm_ares_kernel<32, PREC_FP16>); break;
      default: go(gemm_ares_kernel<16, PREC_FP16>); break;
    }
  } else {
    switch (BM) {
      case 64: go(gemm_ares_kernel<64, PREC_BF16>); break;
      case 32: go(gemm_ares_kernel<32, PREC_BF16>); break;
      default: go(gemm_ares_kernel<16, PREC_BF16>); break;
    }
  }
  return check_launch(who);
}

}  // namespace wf
