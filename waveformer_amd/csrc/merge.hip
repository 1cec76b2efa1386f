// merge.hip -- PatchMerging 1 -> 2 (a9: wave_helper.py:173-194, quirk Q3; the 8C -> 2C
// Linear after the LayerNorm over the 8 gathered sub-lattices) at C = 48, the one merge whose
// whole reduction weight fits the LDS: 96 x 384 bf16 hi + lo = 150 KB.
//
// gemm_kc (the general K-chunked path) streams the weight through LDS one 32-deep k slice at a
// time behind a workgroup barrier per k step, so its waves run in lockstep: every wave's A
// loads, then every wave's MFMAs -- one 16-wave workgroup per CU, load and compute phases never
// overlapping (202-210 us per B = 8 launch, 2.4 TB/s).  Here one persistent workgroup per CU
// stages the whole weight ONCE, and its 12 waves (three per SIMD) walk 16-row tiles with no
// barrier at all: a wave loads its tile's 8 x 48 gathered inputs into registers (12 octets per
// lane, 24 KB per wave in flight), takes the LayerNorm moments from those registers, and runs
// the 12 k steps x 6 column tiles of MFMAs against the resident weight while the other waves
// of its SIMD wait on their loads.  A is read from HBM exactly once.
//
// Same arithmetic as gemm_kc's LN_COMPUTE path, in the same order (shifted one-pass moments
// over octets g4, g4 + 4, ..., MFMA accumulation k step by k step, hi.lo + lo.hi + hi.hi per
// tile): the outputs are bit-identical (tests/test_gpu_parity.py).
#include <algorithm>

#include "gemm_common.hpp"

namespace wf {

constexpr int MR_C = 48;
constexpr int MR_K = 8 * MR_C;                // 384
constexpr int MR_N = 2 * MR_C;                // 96
constexpr int MR_NT = MR_N / 16;              // 6 column tiles
constexpr int MR_KS = MR_K / 32;              // 12 k steps
constexpr int MR_KP = MR_K + WF_LDS_KPAD;     // LDS row stride in bf16: 200 dwords, 8 mod 16
#ifndef WF_MR_WAVES  // waves per merge_res workgroup: 8 measured 135.5-139.3 us against 141.8-143.8
#define WF_MR_WAVES 8  // (12), 149.9-151.0 (6), 154.8-155.6 (4); 16 spills (r6/r6ap_merge_res_waves_ab.txt)
#endif
constexpr int MR_WAVES = WF_MR_WAVES;

template <int P>
__global__ __launch_bounds__(64 * MR_WAVES, 1) void merge_res_kernel(GemmArgs g) {
  constexpr bool SPLIT = P == PREC_SPLIT;  // P: Prec (operand kind)
  constexpr int NPL = SPLIT ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) uint16_t Wl[];  // [NPL][96][MR_KP]
  float* lnw = reinterpret_cast<float*>(Wl + NPL * MR_N * MR_KP);
  float* lnb = lnw + MR_K;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g4 = lane >> 4;

  // ---- the weight ([2][N][K] bf16 planes) and the LayerNorm affine, once per workgroup
  constexpr int OCT = MR_K / 8;
  for (int it = tid; it < NPL * MR_N * OCT; it += 64 * MR_WAVES) {
    const int pr = it / OCT, ch = it - pr * OCT;  // pr = plane * 96 + n
    *reinterpret_cast<bf16x8*>(Wl + pr * MR_KP + 8 * ch) =
        *reinterpret_cast<const bf16x8*>(g.w + (int64_t)pr * MR_K + 8 * ch);
  }
  for (int i = tid; i < MR_K; i += 64 * MR_WAVES) {
    lnw[i] = g.a_ln_w[i];
    lnb[i] = g.a_ln_b[i];
  }
  __syncthreads();

  const int M = (int)g.M;
  const int ntiles = (M + 15) >> 4;
  const int hd = g.mD >> 1, hh = g.mH >> 1, hw = g.mW >> 1;
  for (int tile = blockIdx.x * MR_WAVES + wid; tile < ntiles; tile += gridDim.x * MR_WAVES) {
    const int row = tile * 16 + l15;
    int r = min(row, M - 1);
    const int x = r % hw;
    r /= hw;
    const int y = r % hh;
    r /= hh;
    const int z = r % hd, b = r / hd;
    const float* src = reinterpret_cast<const float*>(g.a_src) +
                       (int64_t)(((b * g.mD + 2 * z) * g.mH + 2 * y) * g.mW + 2 * x) * MR_C;
    // this lane's source offset of k octet g4 + 4 ks relative to the row's (2z, 2y, 2x) corner,
    // in floats: sub-lattice (k / 48) -> (dz, dy, dx) from merge_code (RowMapper<MAP_MERGE>)
    int g4o = g4;  // opaque: the 12 offsets are recomputed per tile, not held across tiles
    asm volatile("" : "+v"(g4o));
    int koff[MR_KS];
#pragma unroll
    for (int ks = 0; ks < MR_KS; ++ks) {
      const int k = ks * 32 + 8 * g4o;
      const int seg = k / MR_C, c = k - seg * MR_C;
      const int o = (g.merge_code >> (4 * seg)) & 0xF;  // bit2: d, bit1: h, bit0: w
      koff[ks] = ((((o >> 2) & 1) * g.mH + ((o >> 1) & 1)) * g.mW + (o & 1)) * MR_C + c;
    }
    // lane (l15, g4): octets g4 + 4 ks of row l15 -- the k-step fragments of every step
    float a[MR_KS][8];
#pragma unroll
    for (int ks = 0; ks < MR_KS; ++ks) {
      const f32x4* p = reinterpret_cast<const f32x4*>(src + koff[ks]);
      const f32x4 u0 = p[0], u1 = p[1];
      a[ks][0] = u0.x; a[ks][1] = u0.y; a[ks][2] = u0.z; a[ks][3] = u0.w;
      a[ks][4] = u1.x; a[ks][5] = u1.y; a[ks][6] = u1.z; a[ks][7] = u1.w;
    }
    // shifted one-pass moments, shift = the row's first element (gemm_kc LN_COMPUTE's order)
    const float sh = __shfl(a[0][0], l15, 64);
    float s = 0.f, q = 0.f;
    // an opaque zero: with a literal one the compiler folds the first d * d + 0 into a multiply
    // and may then fuse the SECOND square into the add instead of the first (a different last
    // bit than gemm_kc's loop, whose accumulator starts in a register)
    asm volatile("" : "+v"(q));
#pragma unroll
    for (int ks = 0; ks < MR_KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = a[ks][j] - sh;
        s += d;
        q += d * d;
      }
    s = xsum16(s);
    s = xsum32(s);
    q = xsum16(q);
    q = xsum32(q);
    const float kf = (float)g.K;  // the runtime K, as gemm_kc divides by
    const float ms = s / kf;
    const float mean = sh + ms;
    const float rstd = rsqrtf(fmaxf(q / kf - ms * ms, 0.f) + g.a_eps);

    // LDS bases re-derived per tile (opaque to the compiler): hoisted out of the tile loop, the
    // 12 x 6 fragment addresses would be loop invariants held in (spilled) VGPRs; per tile they
    // fold into the ds_read offset fields
    uint32_t wb = (uint32_t)((l15 * MR_KP + 8 * g4) * 2), lb = (uint32_t)(8 * g4 * 4);
    asm volatile("" : "+v"(wb), "+v"(lb));
    const char* Wb = reinterpret_cast<const char*>(Wl) + wb;
    const char* Lw = reinterpret_cast<const char*>(lnw) + lb;
    const char* Lb = reinterpret_cast<const char*>(lnb) + lb;
    f32x4 acc[MR_NT];
#pragma unroll
    for (int t = 0; t < MR_NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < MR_KS; ++ks) {
      __builtin_amdgcn_sched_barrier(0);
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(Lw + ks * 128);
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(Lw + ks * 128 + 16);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(Lb + ks * 128);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(Lb + ks * 128 + 16);
      const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      bf16x8 ah, al;
      {
        float xs[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float xv = (a[ks][j] - mean) * rstd * wv[j] + bv[j];
          // fp16: the fp32 value first (gemm_kc's double rounding), not a v_fma_mix straight
          // to fp16, so the two paths stay bit-identical
          if (!SPLIT) asm volatile("" : "+v"(xv));
          xs[j] = xv;
        }
        split8<P>(xs, ah, al);
      }
#pragma unroll
      for (int t = 0; t < MR_NT; ++t) {
        const int wo = (t * 16 * MR_KP + ks * 32) * 2;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Wb + wo);
        if (SPLIT) {
          const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Wb + MR_N * MR_KP * 2 + wo);
          acc[t] = mma32<P>(bh, al, acc[t]);
          acc[t] = mma32<P>(bl, ah, acc[t]);
        }
        acc[t] = mma32<P>(bh, ah, acc[t]);
        // bound the hoisting of the weight-fragment reads (VGPRs: three waves per SIMD)
        if (t % 3 == 2) __builtin_amdgcn_sched_barrier(0);
      }
    }
    // acc[t][i] = out[row][16 t + 4 g4 + i]: the 6 tiles of a row leave back to back, so its
    // 384-B line pair is complete in L2 before it is written back
    if (row < M) {
      float* o = reinterpret_cast<float*>(g.out) + (int64_t)row * g.ldo + 4 * g4;
#pragma unroll
      for (int t = 0; t < MR_NT; ++t) *reinterpret_cast<f32x4*>(o + 16 * t) = acc[t];
    }
  }
}

// PatchMerging 1 -> 2 (C = 48, fp32 in / out, bf16x3 or fp16 operands) on the resident-weight
// kernel; 0 if g is not that shape (the caller falls back to launch_gemm).  WF_MERGE_RES=0
// keeps gemm_kc (A/B).
int try_launch_merge_resident(const GemmArgs& g, hipStream_t s) {
  static const bool off = getenv("WF_MERGE_RES") != nullptr && getenv("WF_MERGE_RES")[0] == '0';
  if (off || g.a_map != MAP_MERGE || g.a_C != MR_C || g.K != MR_K || g.N != MR_N ||
      g.a_ln != LN_COMPUTE || g.a_bf16 || g.out_bf16 || g.epi != EPI_STORE || g.bias ||
      g.o_pstats || g.ldo < MR_N || (g.prec != PREC_SPLIT && g.prec != PREC_FP16) || g.M < 1 ||
      g.M >= ((int64_t)1 << 31) - 16)
    return 0;
  const bool split = g.prec == PREC_SPLIT;
  const size_t lds = (size_t)(split ? 2 : 1) * MR_N * MR_KP * 2 + (size_t)2 * MR_K * 4;
  void (*kern)(GemmArgs) = split ? merge_res_kernel<PREC_SPLIT> : merge_res_kernel<PREC_FP16>;
  set_max_lds(reinterpret_cast<const void*>(kern), (int)lds);
  const int64_t ntiles = (g.M + 15) / 16;
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(ntiles, MR_WAVES), 256);
  hipLaunchKernelGGL(kern, dim3(gx), dim3(64 * MR_WAVES), lds, s, g);
  return 1;
}

}  // namespace wf
