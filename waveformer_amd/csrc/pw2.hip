// pw2.hip -- the CCF_FFN pwconv of encoder stage 2 (C = 96 -> hidden = 384 with LayerNorm(4C)
// + GELU, wave_helper.py:281-283) on persistent workgroups with the whole weight resident:
//
//   h1[m, :] = GELU(LN1(bias + LN_n2(x[m, :]) . Wpw^T))
//
// gemm_lnw (the one-shot kernel it replaces by default) splits the 384 columns over 8 waves of a
// 128-row workgroup and streams the 147 KB weight through registers once per workgroup: 2048
// workgroups read 302 MB of weight from L2 for 100 MB of input rows, and every workgroup pays a
// staging phase, two LDS reductions and three barriers (194.5 us per B = 8 launch).  Here one
// workgroup per CU stages the weight ONCE (384 x 96 bf16 hi + lo = 147 KB, XOR-swizzled so the
// fragment reads are conflict-free without padding), and each wave then owns whole 16-row
// tiles -- all 384 columns, 24 accumulator tiles -- so the LayerNorm moments are a reduction
// over the wave's own lanes: no barrier after the staging.  A wave loads its next tile's rows
// (with the n2 LayerNorm statistics) while it computes the current one.
//
// Bit-identical to gemm_lnw<3, 3, 8, 8> (the same split products in the same order per column
// tile; the row moments summed as its 8 waves' 48-column partials, in its fixed tree order).
// Bound: HBM (x in: 384 B, h1 out: 1536 B per row).
#include <algorithm>

#include "gemm_common.hpp"

namespace wf {

namespace pw2 {
constexpr int K = 96, N = 384, KS = K / 32, NT = N / 16;  // 3 k steps, 24 column tiles
constexpr int RB = K * 2;                                  // weight row bytes (one plane)
constexpr int PLANE = N * RB;                              // 73,728 B
}  // namespace pw2

// chunk (16 B) position of k-octet o of weight row n: XOR within aligned groups of 4 chunks by
// f((n >> 2) & 3), f = {0, 2, 3, 1} -- the 16 reads of each ds_read_b128 lane group (rows
// {0-3, 12-15} at one octet, rows {4-11} at the next, MI355X_MICROARCH.md LDS) then fall on 16
// distinct 4-bank slots with the 192-B row stride
__device__ __forceinline__ int pw2_chunk(int n, int o) {
  const int f = (0x1E >> (2 * ((n >> 2) & 3))) & 3;  // {0, 2, 3, 1}
  return (o & ~3) | ((o & 3) ^ f);
}

template <int P, int NW>
__global__ __launch_bounds__(64 * NW, 1) void pw2_res_kernel(GemmArgs g) {
  using namespace pw2;
  constexpr bool SPLIT = P == PREC_SPLIT;  // P: Prec (operand kind)
  constexpr int NPL = SPLIT ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* ew = reinterpret_cast<float*>(smem + NPL * PLANE);  // [N] LN1 gamma / 2
  float* eb = ew + N;                                        // [N] LN1 beta / 2
  float* bs = eb + N;                                        // [N] bias
  float* aw = bs + N;                                        // [K] n2 gamma
  float* ab = aw + K;                                        // [K] n2 beta
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g4 = lane >> 4;

  // ---- the weight (global [2][N][K] bf16) into the swizzled image, once per workgroup
  for (int it = tid; it < NPL * N * (K / 8); it += 64 * NW) {
    const int pr = it / (K / 8), o = it - pr * (K / 8);  // pr = plane * N + n
    const int n = pr % N;
    *reinterpret_cast<bf16x8*>(smem + pr * RB + 16 * pw2_chunk(n, o)) =
        *reinterpret_cast<const bf16x8*>(g.w + (int64_t)pr * K + 8 * o);
  }
  for (int i = tid; i < N; i += 64 * NW) {
    ew[i] = 0.5f * g.e_ln_w[i];  // GELU from half its input (gelu_half4)
    eb[i] = 0.5f * g.e_ln_b[i];
    bs[i] = g.bias ? g.bias[i] : 0.f;
  }
  const bool aln = g.a_ln == LN_GIVEN;
  for (int i = tid; i < K; i += 64 * NW) {
    aw[i] = aln ? g.a_ln_w[i] : 1.f;
    ab[i] = aln ? g.a_ln_b[i] : 0.f;
  }
  __syncthreads();

  const int M = (int)g.M;
  const int ntiles = (M + 15) >> 4;
  const float* xa = reinterpret_cast<const float*>(g.a_src);
  // this lane's rows of A: row l15 of the tile, k = 32 ks + 8 g4 .. + 7 (two f32x4 per step)
  f32x4 an[KS][2];
  float mn = 0.f, rn = 1.f;
  auto aload = [&](int tile) {
    const int row = min(tile * 16 + l15, M - 1);
    const float* p = xa + (int64_t)row * K + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      an[ks][0] = *reinterpret_cast<const f32x4*>(p + 32 * ks);
      an[ks][1] = *reinterpret_cast<const f32x4*>(p + 32 * ks + 4);
    }
    if (aln) {
      mn = g.a_stats[2 * row];
      rn = g.a_stats[2 * row + 1];
    }
  };
  int tile = blockIdx.x * NW + wid;
  const int stride = gridDim.x * NW;
  if (tile < ntiles) aload(tile);
  // fragment base of this lane in the swizzled image: row 16 t + l15, octet 4 ks + g4
  const int wlane = l15 * RB + 16 * ((g4 ^ ((0x1E >> (2 * ((l15 >> 2) & 3))) & 3)));
  for (; tile < ntiles; tile += stride) {
    // ---- this tile's A: n2 LayerNorm + bf16 hi / lo split (gemm_lnw's staging arithmetic)
    bf16x8 ah[KS], al[KS];
    const float mu = mn, rs = rn;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = 32 * ks + 8 * g4;
#pragma unroll
      for (int hq = 0; hq < 2; ++hq) {
        f32x4 v = an[ks][hq];
        if (aln) {
          const f32x4 lw = *reinterpret_cast<const f32x4*>(aw + k + 4 * hq);
          const f32x4 lb = *reinterpret_cast<const f32x4*>(ab + k + 4 * hq);
          v = (v - mu) * rs * lw + lb;
        }
        uint32_t h0, h1, l0, l1;
        split_pair<P>(v[0], v[1], h0, l0);
        split_pair<P>(v[2], v[3], h1, l1);
        ah[ks][4 * hq] = (short)(h0 & 0xFFFF);
        ah[ks][4 * hq + 1] = (short)(h0 >> 16);
        ah[ks][4 * hq + 2] = (short)(h1 & 0xFFFF);
        ah[ks][4 * hq + 3] = (short)(h1 >> 16);
        al[ks][4 * hq] = (short)(l0 & 0xFFFF);
        al[ks][4 * hq + 1] = (short)(l0 >> 16);
        al[ks][4 * hq + 2] = (short)(l1 & 0xFFFF);
        al[ks][4 * hq + 3] = (short)(l1 >> 16);
      }
    }
    // the next tile's rows, in flight across this tile's MFMAs and epilogue
    if (tile + stride < ntiles) aload(tile + stride);

    // opaque LDS base per tile: the 3 x 24 fragment addresses fold into ds_read offsets
    int wb = wlane;
    asm volatile("" : "+v"(wb));
    const unsigned char* Wb = smem + wb;
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int wo = t * 16 * RB + 64 * ks;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Wb + wo);
        if (SPLIT) {
          const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Wb + PLANE + wo);
          acc[t] = mma32<P>(bh, al[ks], acc[t]);
          acc[t] = mma32<P>(bl, ah[ks], acc[t]);
        }
        acc[t] = mma32<P>(bh, ah[ks], acc[t]);
        if (t % 4 == 3) __builtin_amdgcn_sched_barrier(0);  // bound the fragment-read hoisting
      }
    }

    // ---- epilogue: acc[t][i] = h1[row 16 tile + l15][column 16 t + 4 g4 + i]
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] += *reinterpret_cast<const f32x4*>(bs + 16 * t + 4 * g4);
    // row moments as gemm_lnw<3, 3, 8, 8> forms them: 8 partials of 3 column tiles (its waves),
    // each reduced over the row's 4 lanes, then a fixed tree
    float part[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      float s = 0.f;
#pragma unroll
      for (int t = 3 * w; t < 3 * w + 3; ++t) s += (acc[t].x + acc[t].y) + (acc[t].z + acc[t].w);
      s = xsum16(s);
      part[w] = xsum32(s);
    }
    const float mean =
        (((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]))) *
        (1.f / N);
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      float q = 0.f;
#pragma unroll
      for (int t = 3 * w; t < 3 * w + 3; ++t) {
        const f32x4 d = acc[t] - mean;
        q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
      }
      q = xsum16(q);
      part[w] = xsum32(q);
    }
    const float rstd = rsqrtf(
        (((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]))) *
            (1.f / N) + g.e_eps);
    const int row = tile * 16 + l15;
    float* o = reinterpret_cast<float*>(g.out) + (int64_t)min(row, M - 1) * g.ldo + 4 * g4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f32x4 lw = *reinterpret_cast<const f32x4*>(ew + 16 * t + 4 * g4);
      const f32x4 lb = *reinterpret_cast<const f32x4*>(eb + 16 * t + 4 * g4);
      const f32x4 v = gelu_half4((acc[t] - mean) * rstd * lw + lb);
      if (row < M) *reinterpret_cast<f32x4*>(o + 16 * t) = v;
      if (t % 4 == 3) __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// the stage-2 pwconv shape (K = 96, N = 384, LN + GELU epilogue, fp32 rows in and out) on the
// resident-weight kernel; 0 if g is not that shape.  WF_PW2_RES=0 keeps gemm_lnw (A/B).
int try_launch_pw2_resident(const GemmArgs& g, hipStream_t s) {
  using namespace pw2;
  static const bool off = getenv("WF_PW2_RES") != nullptr && getenv("WF_PW2_RES")[0] == '0';
  if (off || g.epi != EPI_LN_GELU || g.a_map != MAP_IDENTITY || g.a_bf16 || g.a_gelu ||
      !(g.a_ln == LN_NONE || g.a_ln == LN_GIVEN) || g.K != K || g.N != N || g.a_C != K ||
      g.out_bf16 || g.ldo < N || g.ldo % 4 != 0 || (g.prec != PREC_SPLIT && g.prec != PREC_FP16) ||
      g.M < 1 || g.M >= ((int64_t)1 << 31) - 16)
    return 0;
  constexpr int NW = 8;
  const bool split = g.prec == PREC_SPLIT;
  const size_t lds = (size_t)(split ? 2 : 1) * PLANE + (size_t)(3 * N + 2 * K) * 4;
  void (*kern)(GemmArgs) = split ? pw2_res_kernel<PREC_SPLIT, NW> : pw2_res_kernel<PREC_FP16, NW>;
  set_max_lds(reinterpret_cast<const void*>(kern), (int)lds);
  const int64_t ntiles = (g.M + 15) / 16;
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(ntiles, NW), 256);
  hipLaunchKernelGGL(kern, dim3(gx), dim3(64 * NW), lds, s, g);
  return 1;
}

}  // namespace wf
