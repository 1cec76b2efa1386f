// gemm_rows.hip -- streaming MFMA GEMM for the large-M, small-K/N Linear layers of the path.
//
// out[m, n] = epilogue( sum_k A[m, k] * Wt[n, k] ),   M = positions (up to B * 64^3),
// K, N <= a few hundred.  The weights are tiny and the rows are many, so the kernel is built
// around streaming A exactly once from HBM:
//   * a 512-thread workgroup stages one column chunk of Wt (bf16 hi [+ lo] planes, NT*16
//     columns x K) in LDS once, then its 8 waves walk 16-row tiles of A persistently;
//   * a wave loads its A fragments straight from global memory into registers (lane l: row
//     l&15, k = 8*(l>>4) .. +7 of each 32-deep k step), applies the row gather / LayerNorm /
//     bf16 hi-lo split on the fly, and issues NT v_mfma_f32_16x16x32_bf16 (x3 for PREC_SPLIT)
//     per k step against B fragments read from LDS with ds_read_b128;
//   * the epilogue runs on the accumulators in registers (C layout: lane l holds rows
//     4*(l>>4)+i, column l&15 of each 16-wide tile): bias, LayerNorm over the full row
//     (16-lane xor shuffles) + GELU, or the Block residual; stores go straight to HBM.
// Every load in the hot loops is unconditional (clamped address, then a select): a branch
// around a load makes hipcc wait vmcnt(0) for it and serialises the stream.  The row map
// (identity / window gather / PatchMerging gather) and the epilogue are template parameters
// so each call site compiles to straight-line code with 32-bit index math.
#include "kernels.hpp"

namespace wf {

template <bool BF16>
__device__ __forceinline__ void load8f(const void* src, int64_t off, float (&v)[8]) {
  if (BF16) {
    const bf16x8 u = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const uint16_t*>(src) + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f((uint16_t)u[j]);
  } else {
    const f32x4* p = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(src) + off);
    const f32x4 a = p[0], b = p[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}

// Source element offset of logical (row m, column k).
template <int MAP>
struct RowMapper {
  int pos;  // source raster row (MAP_MERGE: the (2z, 2y, 2x) corner)
  __device__ __forceinline__ RowMapper(const GemmArgs& g, int m) {
    if (MAP == MAP_WINDOW) {
      const int ws = g.mws;
      const int N = ws * ws * ws;
      const int nWh = g.mH / ws, nWw = g.mW / ws, nW = (g.mD / ws) * nWh * nWw;
      const int bw = m / N;
      const int t = m - bw * N;
      const int b = bw / nW;
      int wi = bw - b * nW;
      const int wx = wi % nWw;
      wi /= nWw;
      const int wy = wi % nWh, wz = wi / nWh;
      const int tx = t % ws, ty = (t / ws) % ws, tz = t / (ws * ws);
      pos = ((b * g.mD + wz * ws + tz) * g.mH + wy * ws + ty) * g.mW + wx * ws + tx;
    } else if (MAP == MAP_MERGE) {
      const int d = g.mD >> 1, h = g.mH >> 1, w = g.mW >> 1;
      int r = m;
      const int x = r % w;
      r /= w;
      const int y = r % h;
      r /= h;
      const int z = r % d;
      const int b = r / d;
      pos = ((b * g.mD + 2 * z) * g.mH + 2 * y) * g.mW + 2 * x;
    } else {
      pos = m;
    }
  }
  __device__ __forceinline__ int64_t offset(const GemmArgs& g, int k) const {
    if (MAP == MAP_MERGE) {
      const int seg = k / g.a_C;
      const int c = k - seg * g.a_C;
      const int o = (g.merge_code >> (4 * seg)) & 0xF;  // bit2: d, bit1: h, bit0: w
      const int p = pos + (((o >> 2) & 1) * g.mH + ((o >> 1) & 1)) * g.mW + (o & 1);
      return (int64_t)p * g.a_C + c;
    }
    return (int64_t)pos * g.K + k;
  }
};

template <int NT, bool SPLIT, int MAP, int EPI, bool ABF16>
__global__ __launch_bounds__(512) void gemm_rows_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t Wl[];  // [NB][NT*16][KP]
  const int K = g.K, N = g.N;
  const int M = (int)g.M;
  const int K32 = (K + 31) & ~31;
  const int KP = K32 + 8;
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
  __syncthreads();

  const int ntiles = (M + 15) >> 4;
  const int nwaves = blockDim.x >> 6;
  for (int tile = blockIdx.x * nwaves + wid; tile < ntiles; tile += gridDim.x * nwaves) {
    // ---- A rows of this lane: row l15 of the tile
    const int arow_c = min(tile * 16 + l15, M - 1);
    const RowMapper<MAP> rm(g, arow_c);
    float mean = 0.f, rstd = 1.f;
    if (g.a_ln == LN_GIVEN) {
      mean = g.a_stats[2 * arow_c];
      rstd = g.a_stats[2 * arow_c + 1];
    } else if (g.a_ln == LN_COMPUTE) {  // lanes l15, l15+16, l15+32, l15+48 share the row
      float s = 0.f;
      for (int ch = g4; ch < K / 8; ch += 4) {
        float v[8];
        load8f<ABF16>(g.a_src, rm.offset(g, ch * 8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[j];
      }
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      mean = s / (float)K;
      float q = 0.f;
      for (int ch = g4; ch < K / 8; ch += 4) {
        float v[8];
        load8f<ABF16>(g.a_src, rm.offset(g, ch * 8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[j] - mean;
          q += d * d;
        }
      }
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      rstd = rsqrtf(q / (float)K + g.a_eps);
    }

    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0, 0, 0, 0};

    // k loop with a one-step register prefetch of the A fragment
    float vn[8];
    load8f<ABF16>(g.a_src, rm.offset(g, min(8 * g4, K - 8)), vn);
#pragma unroll 1
    for (int k0 = 0; k0 < K32; k0 += 32) {
      const int k = k0 + 8 * g4;
      const bool kv = k < K;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = vn[j];
      load8f<ABF16>(g.a_src, rm.offset(g, min(k + 32, K - 8)), vn);  // (last: unused)
      if (g.a_ln != LN_NONE) {
        const int kk = min(k, K - 8);
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(g.a_ln_w + kk);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(g.a_ln_w + kk + 4);
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(g.a_ln_b + kk);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(g.a_ln_b + kk + 4);
        const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (v[j] - mean) * rstd * wv[j] + bv[j];
      }
      bf16x8 ah, al;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = kv ? v[j] : 0.f;
        const uint16_t h = f2bf(x);
        ah[j] = (short)h;
        al[j] = SPLIT ? (short)f2bf(x - bf2f(h)) : (short)0;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int wo = (t * 16 + l15) * KP + k0 + 8 * g4;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Wl + wo);
        if (SPLIT) {
          const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Wl + NCOL * KP + wo);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc[t], 0, 0, 0);
        }
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc[t], 0, 0, 0);
      }
    }

    // ---- epilogue on the accumulators: acc[t][i] = C[row 4*g4+i][col c0 + t*16 + l15]
    if (g.bias) {
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] += g.bias[min(c0 + t * 16 + l15, N - 1)];
    }
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
      const int row = tile * 16 + 4 * g4 + i;
      const bool rv = row < M;
      const int rowc = min(row, M - 1);
      float rm_ = 0.f, rs_ = 1.f, bs = 1.f;
      if (EPI == EPI_LN_GELU) {  // full row in this wave (NCOL == N): 16-lane reductions
        float s = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) s += acc[t][i];
        rm_ = group_sum<16>(s) / (float)N;
        float q = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const float d = acc[t][i] - rm_;
          q += d * d;
        }
        rs_ = rsqrtf(group_sum<16>(q) / (float)N + g.e_eps);
      } else if (EPI == EPI_RESID) {
        if (g.r_stats) {
          rm_ = g.r_stats[2 * rowc];
          rs_ = g.r_stats[2 * rowc + 1];
        }
        if (g.r_scale) bs = g.r_scale[rowc / (int)g.rows_per_sample];
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int col = c0 + t * 16 + l15;
        const int colc = min(col, N - 1);
        float v = acc[t][i];
        if (EPI == EPI_LN_GELU) {
          v = gelu_erf((v - rm_) * rs_ * g.e_ln_w[colc] + g.e_ln_b[colc]);
        } else if (EPI == EPI_RESID) {
          const float xr = g.r_x[(int64_t)rowc * N + colc];
          if (g.r_stats) {
            const float n2 = (xr - rm_) * rs_ * g.r_ln_w[colc] + g.r_ln_b[colc];
            v = xr + (n2 + v) * bs;  // attn_fused + drop_path(n2 + ffn(n2)), quirk Q4
          } else {
            v = xr + v * bs;         // bare CCF_FFN.forward: x + x_out
          }
        }
        if (rv && col < N) {
          if (g.out_bf16)
            reinterpret_cast<uint16_t*>(g.out)[(int64_t)row * g.ldo + col] = f2bf(v);
          else
            reinterpret_cast<float*>(g.out)[(int64_t)row * g.ldo + col] = v;
        }
      }
    }
  }
}

template <int NT, int MAP, int EPI>
static void go_rows(const GemmArgs& g, dim3 grid, size_t lds, hipStream_t s) {
  const bool split = g.prec == PREC_SPLIT;
  void (*kern)(GemmArgs);
  if (g.a_bf16)
    kern = split ? gemm_rows_kernel<NT, true, MAP, EPI, true> : gemm_rows_kernel<NT, false, MAP, EPI, true>;
  else
    kern = split ? gemm_rows_kernel<NT, true, MAP, EPI, false> : gemm_rows_kernel<NT, false, MAP, EPI, false>;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
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

int try_launch_gemm_rows(const GemmArgs& g, hipStream_t s) {
  if (g.N % 16 != 0 || g.K < 8 || g.M >= ((int64_t)1 << 31)) return 0;
  // call-site shapes (the others fall back to gemm_ares): window qkv, identity store/LN/resid,
  // PatchMerging gather
  const bool known = (g.a_map == MAP_WINDOW && g.epi == EPI_STORE) ||
                     (g.a_map == MAP_IDENTITY) || (g.a_map == MAP_MERGE && g.epi == EPI_STORE);
  if (!known) return 0;
  const bool split = g.prec == PREC_SPLIT;
  const int K32 = (g.K + 31) & ~31;
  const size_t per_col = (size_t)(split ? 2 : 1) * (K32 + 8) * 2;
  const int tiles = g.N / 16;
  static const int cand[] = {12, 9, 8, 6, 4, 3, 2, 1};
  int nt = 0;
  for (int c : cand) {
    if (tiles % c != 0) continue;
    if (g.epi == EPI_LN_GELU && c != tiles) continue;  // LayerNorm needs the full row
    if ((size_t)c * 16 * per_col <= 64 * 1024) {
      nt = c;
      break;
    }
  }
  if (nt == 0) return 0;
  const size_t lds = (size_t)nt * 16 * per_col;
  const int chunks = tiles / nt;
  const int64_t ntiles = (g.M + 15) / 16;
  int64_t gx = cdiv(ntiles, 8);
  const int64_t cap = (512 + chunks - 1) / chunks;  // ~2 workgroups of 8 waves per CU
  if (gx > cap) gx = cap;
  if (gx < 1) gx = 1;
  dim3 grid((unsigned)gx, (unsigned)chunks);
  if (g.a_map == MAP_WINDOW) dispatch_nt<MAP_WINDOW, EPI_STORE>(nt, g, grid, lds, s);
  else if (g.a_map == MAP_MERGE) dispatch_nt<MAP_MERGE, EPI_STORE>(nt, g, grid, lds, s);
  else if (g.epi == EPI_LN_GELU) dispatch_nt<MAP_IDENTITY, EPI_LN_GELU>(nt, g, grid, lds, s);
  else if (g.epi == EPI_RESID) dispatch_nt<MAP_IDENTITY, EPI_RESID>(nt, g, grid, lds, s);
  else dispatch_nt<MAP_IDENTITY, EPI_STORE>(nt, g, grid, lds, s);
  return 1;
}

}  // namespace wf
