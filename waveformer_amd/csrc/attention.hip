// attention.hip -- windowed multi-head self-attention.
//
// Reference: network_models/attention.py:83-104 (Attention.forward), driven by
// Block.multi_scale_forward (wave_helper.py:482-499): window_partition -> qkv -> q*scale ->
// q@k^T + relative_position_bias -> softmax -> @v -> proj, then the window "reverse" that is
// a plain reshape (quirk Q1).  Here:
//   qkv  : gemm_ares with the window gather (and norm1 for level-0 blocks) in its loader
//   core : one workgroup = (window b_, head h, 64 queries); flash-style loop over key tiles
//          staged in LDS.  S^T = K.Q^T is computed "swapped" (keys on the MFMA rows, queries
//          on the lanes) so the fp32 accumulator of S^T is, register for register, the B
//          operand of O^T = V^T.P^T after bf16 rounding -- P never leaves registers and the
//          softmax column reductions are 2 lane shuffles.  v_mfma_f32_16x16x16_bf16 covers
//          head_dim in 16-wide steps (head_dim is 16 at the default widths).  PREC_SPLIT
//          carries Q, K, V and P as bf16 hi + lo pairs (3 MFMAs per product).
//   proj : gemm_ares; rows stay in window-major order, which is exactly the reference's
//          reshaped raster (Q1).
#include "kernels.hpp"

namespace wf {

constexpr int kQB = 64;  // queries per workgroup (16 per wave)

// XCD-aware decode of the 1-D grid.  Workgroups are dealt round-robin over the 8 XCDs (linear
// id L runs on XCD L % 8), so the query tiles of one (window, head) -- which all stage the same
// K / V rows -- would land on 8 different XCDs and each XCD's L2 would fetch those rows again.
// Logical id t = the L-th slot of XCD L % 8 in a contiguous split keeps consecutive t (the
// query tiles of one (window, head)) on one XCD.
__device__ __forceinline__ void attn_block(int gx, int heads, int& qb, int& h, int64_t& bw) {
  const int64_t L = blockIdx.x, nb = gridDim.x;
  const int64_t xcd = L & 7, q8 = nb >> 3, r8 = nb & 7;
  int64_t t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
  qb = (int)(t % gx);
  t /= gx;
  h = (int)(t % heads);
  bw = t / heads;
}

// 8 consecutive values of an activation row as MFMA operands: fp32 storage (PREC_SPLIT,
// PREC_FP16) converted to the operand kind (+ the split's lo part), or bf16 storage as-is
template <int P>
__device__ __forceinline__ void load8_split(const void* base, int64_t off, bf16x8& hi,
                                            bf16x8& lo) {
  if (store32(P)) {
    const f32x4* p = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(base) + off);
    const f32x4 a = p[0], b = p[1];
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint16_t h = op_cvt<P>(v[j]);
      hi[j] = (short)h;
      lo[j] = op_lo<P>(v[j], h);
    }
  } else {
    hi = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const uint16_t*>(base) + off);
  }
}

// WS == 0: `bias` is the dense (heads, N, N) relative-position bias.  WS == 8 (ws % 4 == 0
// in general): `bias` is the (T, heads) relative_position_bias_table itself; its column h is
// staged in LDS (pre-scaled by log2 e) and each score's row is the reference's index formula
// (attention.py:40-56, with the Q2 depth stride 3 ws - 1) evaluated from the query / key
// coordinates -- the (heads, N, N) tensor (805 MB of L2 reads per stage-1 launch) is never
// touched.  The 4 keys a lane holds share (z, y) and have consecutive x, so their indices are
// i0, i0 - 1, i0 - 2, i0 - 3.
template <int HD, int KT, int P, int WS = 0>
__global__ __launch_bounds__(256) void attn_core_kernel(const void* __restrict__ qkv,
                                                        const float* __restrict__ bias,
                                                        void* __restrict__ out,
                                                        float* __restrict__ lse, int N,
                                                        int heads, float scale_log2) {
  constexpr bool SPLIT = P == PREC_SPLIT;  // P: Prec (operand kind)
  constexpr int TBLN = WS ? (2 * WS - 2) * (3 * WS - 1) + (2 * WS - 2) * (2 * WS - 1) + 2 * WS - 1
                          : 1;  // reachable table rows (Q2 collapses the (2ws-1)^3 table)
  __shared__ float tb[TBLN];
  constexpr int NC = HD / 16;  // 16-wide head_dim chunks
  constexpr int NKT = KT / 16; // 16-key sub-tiles per tile
  constexpr int KS = HD + 4, VS = KT + 4;
  constexpr int NB = SPLIT ? 2 : 1;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[NB][KT * KS];  // [key][hd]
  __shared__ __attribute__((aligned(16))) uint16_t Vt[NB][HD * VS];  // [hd][key]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int qb, h;
  int64_t bw;
  attn_block((N + kQB - 1) / kQB, heads, qb, h, bw);
  const int C = heads * HD;
  const int64_t row0 = bw * N;  // first token row of this window
  const int ld = 3 * C;
  const int q = qb * kQB + wid * 16 + (lane & 15);  // this lane's query (column)
  const bool qv = q < N;
  const int g4 = 4 * (lane >> 4);

  // Q^T fragments (B operand): lane holds Q[q][c*16 + g4 + j], j < 4
  bf16x4 qf[NC], qfl[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    qf[c] = bf16x4{0, 0, 0, 0};
    qfl[c] = bf16x4{0, 0, 0, 0};
    if (!qv) continue;
    const int64_t off = (row0 + q) * ld + h * HD + c * 16 + g4;
    if (store32(P)) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(qkv) + off);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint16_t hh = op_cvt<P>(v[j]);
        qf[c][j] = (short)hh;
        qfl[c][j] = op_lo<P>(v[j], hh);
      }
    } else {
      qf[c] = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const uint16_t*>(qkv) + off);
    }
  }
  f32x4 o[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) o[c] = f32x4{0, 0, 0, 0};
  float mrun = -INFINITY, lrun = 0.f;
  const float* brow = bias + ((int64_t)h * N + (qv ? q : 0)) * (WS ? 0 : N);
  int qbase = 0;
  if (WS) {
    for (int i = tid; i < TBLN; i += 256) tb[i] = bias[(int64_t)i * heads + h] * 1.4426950408889634f;
    const int qq = qv ? q : 0;
    const int qz = qq / (WS * WS), qy = (qq / WS) % WS, qx = qq % WS;
    qbase = (qz + WS - 1) * (3 * WS - 1) + (qy + WS - 1) * (2 * WS - 1) + (qx + WS - 1);
  }

  for (int k0 = 0; k0 < N; k0 += KT) {
    __syncthreads();
    // stage K rows and V^T for keys k0..k0+KT-1 (chunks of 8 head_dim values)
    for (int it = tid; it < KT * (HD / 8); it += 256) {
      const int kr = it / (HD / 8), ch = it % (HD / 8);
      const int key = k0 + kr;
      bf16x8 kh = {0, 0, 0, 0, 0, 0, 0, 0}, kl = kh, vh = kh, vl = kh;
      if (key < N) {
        const int64_t off = (row0 + key) * ld + h * HD + ch * 8;
        load8_split<P>(qkv, off + C, kh, kl);
        load8_split<P>(qkv, off + 2 * C, vh, vl);
      }
      *reinterpret_cast<bf16x8*>(&Ks[0][kr * KS + ch * 8]) = kh;
      if (SPLIT) *reinterpret_cast<bf16x8*>(&Ks[NB - 1][kr * KS + ch * 8]) = kl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        Vt[0][(ch * 8 + j) * VS + kr] = (uint16_t)vh[j];
        if (SPLIT) Vt[NB - 1][(ch * 8 + j) * VS + kr] = (uint16_t)vl[j];
      }
    }
    __syncthreads();

    // S^T for NKT sub-tiles of 16 keys: rows key = k0 + kt*16 + g4 + i, column = query
    f32x4 s[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      s[kt] = f32x4{0, 0, 0, 0};
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ko = (kt * 16 + (lane & 15)) * KS + c * 16 + g4;
        const bf16x4 a = *reinterpret_cast<const bf16x4*>(&Ks[0][ko]);
        if (SPLIT) {
          const bf16x4 al = *reinterpret_cast<const bf16x4*>(&Ks[NB - 1][ko]);
          s[kt] = mma16<P>(al, qf[c], s[kt]);
          s[kt] = mma16<P>(a, qfl[c], s[kt]);
        }
        s[kt] = mma16<P>(a, qf[c], s[kt]);
      }
    }
    // scale + relative-position bias (log2 domain), key mask
    float tmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const int kb = k0 + kt * 16 + g4;
      f32x4 bv;
      if (WS) {  // already scaled by log2 e
        const int kz = kb / (WS * WS), ky = (kb / WS) % WS, kx = kb % WS;
        const int i0 = min(max(qbase - (kz * (3 * WS - 1) + ky * (2 * WS - 1) + kx), 3), TBLN - 1);
        bv = f32x4{tb[i0], tb[i0 - 1], tb[i0 - 2], tb[i0 - 3]};
      } else if (kb + 3 < N) {
        bv = *reinterpret_cast<const f32x4*>(brow + kb) * 1.4426950408889634f;
      } else {
        bv.x = kb + 0 < N ? brow[kb + 0] : 0.f;
        bv.y = kb + 1 < N ? brow[kb + 1] : 0.f;
        bv.z = kb + 2 < N ? brow[kb + 2] : 0.f;
        bv.w = kb + 3 < N ? brow[kb + 3] : 0.f;
        bv *= 1.4426950408889634f;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float t = s[kt][i] * scale_log2 + bv[i];
        t = (kb + i < N) ? t : -INFINITY;
        s[kt][i] = t;
        tmax = fmaxf(tmax, t);
      }
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(mrun, tmax);
    const float alpha = __builtin_amdgcn_exp2f(mrun - mnew);  // mrun = -inf on the first tile -> 0
    mrun = mnew;
    float psum = 0.f;
    bf16x4 pf[NKT], pfl[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = __builtin_amdgcn_exp2f(s[kt][i] - mnew);
        psum += p;
        const uint16_t ph = op_cvt<P>(p);
        pf[kt][i] = (short)ph;
        pfl[kt][i] = op_lo<P>(p, ph);
      }
    }
    lrun = lrun * alpha + psum;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      o[c] *= alpha;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const int vo = (c * 16 + (lane & 15)) * VS + kt * 16 + g4;
        const bf16x4 a = *reinterpret_cast<const bf16x4*>(&Vt[0][vo]);
        if (SPLIT) {
          const bf16x4 al = *reinterpret_cast<const bf16x4*>(&Vt[NB - 1][vo]);
          o[c] = mma16<P>(al, pf[kt], o[c]);
          o[c] = mma16<P>(a, pfl[kt], o[c]);
        }
        o[c] = mma16<P>(a, pf[kt], o[c]);
      }
    }
  }
  // full column sums: the 4 lane groups hold disjoint key subsets
  lrun = xsum16(lrun);
  lrun = xsum32(lrun);
  // training: the row log-sum-exp (log2 domain) that the backward recomputes P from
  if (lse && qv && lane < 16) lse[(bw * heads + h) * N + q] = mrun + __log2f(lrun);
  if (qv) {
    const float inv = 1.f / lrun;
    const int64_t off = (row0 + q) * C + h * HD + g4;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (store32(P)) {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(out) + off + c * 16) = o[c] * inv;
      } else {
        bf16x4 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = (short)f2bf(o[c][i] * inv);
        *reinterpret_cast<bf16x4*>(reinterpret_cast<uint16_t*>(out) + off + c * 16) = r;
      }
    }
  }
}

// Whole-window variant (N <= 512, the 8^3 windows of the default config): all N keys' K rows
// and V^T are staged into LDS ONCE per workgroup (one barrier), then each wave runs the flash
// loop over 64-key tiles with no barriers, prefetching the next tile's relative-position bias
// rows into registers while the current tile's MFMAs and softmax run (the per-tile staging +
// 2 barriers + exposed bias loads of attn_core_kernel left the waves waiting on memory 57% of
// their cycles).  V is stored [key/4][hd][4 keys], so the staging writes 4 keys per
// ds_write_b64 and the PV A fragment (4 consecutive keys of one hd) is one ds_read_b64.
template <int HD, int P>
__global__ __launch_bounds__(256, 2) void attn_win_kernel(const void* __restrict__ qkv,
                                                          const float* __restrict__ bias,
                                                          void* __restrict__ out,
                                                          float* __restrict__ lse, int N,
                                                          int heads, float scale_log2) {
  constexpr bool SPLIT = P == PREC_SPLIT;  // P: Prec (operand kind)
  constexpr int NC = HD / 16;
  constexpr int KT = 64, NKT = KT / 16;
  constexpr int KS = HD + 4;
  constexpr int NB = SPLIT ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds_attn[];
  const int NP = (N + KT - 1) / KT * KT;  // keys padded to whole tiles (zero K / V rows)
  uint16_t* Ks = lds_attn;                           // [NB][NP][KS]
  uint16_t* Vq = lds_attn + (size_t)NB * NP * KS;    // [NB][NP/4][HD][4]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int qb, h;
  int64_t bw;
  attn_block((N + kQB - 1) / kQB, heads, qb, h, bw);
  const int C = heads * HD;
  const int64_t row0 = bw * N;
  const int ld = 3 * C;
  const int q = qb * kQB + wid * 16 + (lane & 15);
  const bool qv = q < N;
  const int g4 = 4 * (lane >> 4);

  // ---- stage K [key][hd] and V [key/4][hd][4] for all keys (zero past N)
  for (int it = tid; it < NP * (HD / 8); it += 256) {
    const int kr = it / (HD / 8), ch = it % (HD / 8);
    bf16x8 kh = {0, 0, 0, 0, 0, 0, 0, 0}, kl = kh;
    if (kr < N) load8_split<P>(qkv, (row0 + kr) * ld + C + h * HD + ch * 8, kh, kl);
    *reinterpret_cast<bf16x8*>(Ks + (size_t)kr * KS + ch * 8) = kh;
    if (SPLIT) *reinterpret_cast<bf16x8*>(Ks + (size_t)(NP + kr) * KS + ch * 8) = kl;
  }
  for (int it = tid; it < (NP / 4) * (HD / 8); it += 256) {
    const int k4 = it / (HD / 8), ch = it % (HD / 8);
    bf16x8 vh[4], vl[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      vh[r] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      vl[r] = vh[r];
      const int key = 4 * k4 + r;
      if (key < N) load8_split<P>(qkv, (row0 + key) * ld + 2 * C + h * HD + ch * 8, vh[r], vl[r]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const size_t o = ((size_t)k4 * HD + ch * 8 + j) * 4;
      *reinterpret_cast<bf16x4*>(Vq + o) = bf16x4{vh[0][j], vh[1][j], vh[2][j], vh[3][j]};
      if (SPLIT)
        *reinterpret_cast<bf16x4*>(Vq + (size_t)NP * HD + o) =
            bf16x4{vl[0][j], vl[1][j], vl[2][j], vl[3][j]};
    }
  }

  // Q^T fragments (B operand): lane holds Q[q][c*16 + g4 + j], j < 4
  bf16x4 qf[NC], qfl[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    qf[c] = bf16x4{0, 0, 0, 0};
    qfl[c] = bf16x4{0, 0, 0, 0};
    if (!qv) continue;
    const int64_t off = (row0 + q) * ld + h * HD + c * 16 + g4;
    if (store32(P)) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(qkv) + off);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint16_t hh = op_cvt<P>(v[j]);
        qf[c][j] = (short)hh;
        qfl[c][j] = op_lo<P>(v[j], hh);
      }
    } else {
      qf[c] = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const uint16_t*>(qkv) + off);
    }
  }
  f32x4 o[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) o[c] = f32x4{0, 0, 0, 0};
  float mrun = -INFINITY, lrun = 0.f;
  const float* brow = bias + ((int64_t)h * N + (qv ? q : 0)) * N;
  // bias of key kb .. kb+3 (zero past N; kb is a multiple of 4 and N of 4 or not -- guarded)
  auto load_bias = [&](int kb) -> f32x4 {
    if (kb + 3 < N) return *reinterpret_cast<const f32x4*>(brow + kb);
    f32x4 r;
    r.x = kb + 0 < N ? brow[kb + 0] : 0.f;
    r.y = kb + 1 < N ? brow[kb + 1] : 0.f;
    r.z = kb + 2 < N ? brow[kb + 2] : 0.f;
    r.w = kb + 3 < N ? brow[kb + 3] : 0.f;
    return r;
  };
  f32x4 bnext[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) bnext[kt] = load_bias(kt * 16 + g4);
  __syncthreads();

  for (int k0 = 0; k0 < N; k0 += KT) {
    f32x4 bv[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) bv[kt] = bnext[kt];
    if (k0 + KT < N) {
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) bnext[kt] = load_bias(k0 + KT + kt * 16 + g4);
    }
    f32x4 s[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      s[kt] = f32x4{0, 0, 0, 0};
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ko = (k0 + kt * 16 + (lane & 15)) * KS + c * 16 + g4;
        const bf16x4 a = *reinterpret_cast<const bf16x4*>(Ks + ko);
        if (SPLIT) {
          const bf16x4 al = *reinterpret_cast<const bf16x4*>(Ks + (size_t)NP * KS + ko);
          s[kt] = mma16<P>(al, qf[c], s[kt]);
          s[kt] = mma16<P>(a, qfl[c], s[kt]);
        }
        s[kt] = mma16<P>(a, qf[c], s[kt]);
      }
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const int kb = k0 + kt * 16 + g4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float t = s[kt][i] * scale_log2 + bv[kt][i] * 1.4426950408889634f;
        t = (kb + i < N) ? t : -INFINITY;
        s[kt][i] = t;
        tmax = fmaxf(tmax, t);
      }
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(mrun, tmax);
    const float alpha = __builtin_amdgcn_exp2f(mrun - mnew);
    mrun = mnew;
    float psum = 0.f;
    bf16x4 pf[NKT], pfl[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = __builtin_amdgcn_exp2f(s[kt][i] - mnew);
        psum += p;
        const uint16_t ph = op_cvt<P>(p);
        pf[kt][i] = (short)ph;
        pfl[kt][i] = op_lo<P>(p, ph);
      }
    }
    lrun = lrun * alpha + psum;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      o[c] *= alpha;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const size_t vo = ((size_t)((k0 + kt * 16 + g4) >> 2) * HD + c * 16 + (lane & 15)) * 4;
        const bf16x4 a = *reinterpret_cast<const bf16x4*>(Vq + vo);
        if (SPLIT) {
          const bf16x4 al = *reinterpret_cast<const bf16x4*>(Vq + (size_t)NP * HD + vo);
          o[c] = mma16<P>(al, pf[kt], o[c]);
          o[c] = mma16<P>(a, pfl[kt], o[c]);
        }
        o[c] = mma16<P>(a, pf[kt], o[c]);
      }
    }
  }
  lrun = xsum16(lrun);
  lrun = xsum32(lrun);
  if (lse && qv && lane < 16) lse[(bw * heads + h) * N + q] = mrun + __log2f(lrun);
  if (qv) {
    const float inv = 1.f / lrun;
    const int64_t off = (row0 + q) * C + h * HD + g4;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (store32(P)) {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(out) + off + c * 16) = o[c] * inv;
      } else {
        bf16x4 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = (short)f2bf(o[c][i] * inv);
        *reinterpret_cast<bf16x4*>(reinterpret_cast<uint16_t*>(out) + off + c * 16) = r;
      }
    }
  }
}

// Table-bias attention for the default window (ws 8: N = 512 tokens, head_dim 16), one
// workgroup per (window, head) -- or per 1/2 or 1/4 of its queries when there are too few
// windows to fill the chip.  K and V are split into bf16 hi / lo ONCE per (window, head) and
// staged in LDS (68 KB: two workgroups per CU), instead of once per 64-query workgroup.  Every
// product runs on v_mfma_f32_16x16x32_bf16:
//   S^T = K Q'^T + B : the K = 32 reduction packs [Kh | Kl] against [Q'h | Q'h] (Kh Q'h + Kl Q'h
//                 in one MFMA), a second MFMA adds Kh Q'l ([Kh | Kl] against [Q'l | 0]).  Q' is
//                 Q pre-scaled by scale * log2 e, and the accumulator STARTS at the bias
//                 (log2 e-scaled table entries), so the MFMA output is already the exp2-domain
//                 logit: no scale / bias pass on the VALU;
//   O^T = V^T P^T : 32 keys per MFMA, the B operand is the lane's two 4-key score quads of two
//                 16-key sub-tiles as they come out of the S MFMAs (the K-slot order is matched
//                 by reading V at the same keys), x3 for the split;
//   l   = 1^T P^T : the softmax row sums on the same B operands (a ones A operand, hi + lo),
//                 instead of an add per score on the VALU; every accumulator row holds the sum.
// The bias index is the reference's formula (attention.py:40-56, Q2 depth stride 3 ws - 1)
// with the key part reduced to per-tile constants: a 64-key tile is one z slice of the window.
// The table is staged REVERSED, so a lane's 16 bias values of a tile are 4 ascending runs of 4
// at one per-tile base + compile-time offsets 30 kt + i (ds_read2_b32 immediate offsets).
// K rows are 64 B (hi 16 | lo 16) with the four 16-B chunks XOR-swizzled by (row / 4) & 3
// through {0, 2, 3, 1}: every 16-lane group of a ds_read_b128 (gfx950 groups lanes
// {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) then hits 16 distinct 4-bank sets -- the
// round-2 80-B padded rows were 2-way conflicted (SQ_LDS_BANK_CONFLICT ~ SQ_INSTS_LDS).
template <int P>
__device__ __forceinline__ void load8_split_scaled(const void* base, int64_t off, float sc,
                                                   bf16x8& hi, bf16x8& lo) {
  if (store32(P)) {
    const f32x4* p = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(base) + off);
    const f32x4 a = p[0] * sc, b = p[1] * sc;
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint16_t h = op_cvt<P>(v[j]);
      hi[j] = (short)h;
      lo[j] = op_lo<P>(v[j], h);
    }
  } else {
    const bf16x8 r = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const uint16_t*>(base) + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) hi[j] = (short)f2bf(bf2f((uint16_t)r[j]) * sc);
  }
}

__device__ __forceinline__ int kswz(int row) {  // 16-B chunk XOR of a K row (see above)
  return (0x78 >> (2 * ((row >> 2) & 3))) & 3;  // {0, 2, 3, 1}[(row >> 2) & 3]
}

// WF_ATTN_MFMA_SUM=0: the softmax row sums as fp32 VALU adds instead of the ones-operand
// MFMAs (4 of the 18 MFMAs per 64-key tile); measured slower -- 191 vs 171 us per B = 8
// stage-1 launch (profiles/r4_attention_rowsum_ab.txt): the kernel's VALU, not its MFMA
// pipe, is the tighter resource, so the default keeps the sums on the MFMA.
#ifndef WF_ATTN_MFMA_SUM
#define WF_ATTN_MFMA_SUM 1
#endif
// WF_ATTN_BPERMUTE: the per-tile max exchange across the 4 key groups of a query column as
// __shfl_xor (ds_bpermute, LDS crossbar; default) or as v_permlane16/32_swap (VALU, 0).  The
// round-5 kernel-trace A/B (profiles/r5_attention_ab.txt) has the bpermute form 162.8 vs
// 169.1 us per B = 8 stage-1 launch: the kernel's VALU is its tighter resource, and the swap
// form adds VALU work.  A software-pipelined variant (tile t + 1's score MFMAs issued before
// tile t's softmax) measured 174.8 us and was dropped.
#ifndef WF_ATTN_BPERMUTE
#define WF_ATTN_BPERMUTE 1
#endif
#ifndef WF_ATTN_T4  // 1: bias quads as single ds_read_b128 (A/B; 0: four scalar reads)
#define WF_ATTN_T4 1
#endif
// WF_ATTN_LAZY (round 6): the running max is kept while no score of a 64-key tile exceeds it
// by more than 2^WF_ATTN_TAU in the exp2 domain (a lane-local max + one wave ballot); only then
// does the tile pay the cross-group max exchange (two ds_bpermute round trips on the
// critical path), the alpha exponential and the o / l rescale.  The exponentials of a kept tile
// are at most 2^TAU; the normalisation o / l is the same quotient, so this changes only fp32
// rounding.  0: the max is exchanged and the rescale applied on every tile (round 5).
#ifndef WF_ATTN_LAZY
#define WF_ATTN_LAZY 1
#endif
#ifndef WF_ATTN_TAU
#define WF_ATTN_TAU 16.0f
#endif
// WF_ATTN_DOT2 (round 6, bf16x3): the split's lo part of a pair of probabilities is
// bf16(p - hi) with p - hi from one v_dot2c_f32_bf16 per value (the packed hi pair against
// (-1, 0) / (0, -1), accumulated onto p) instead of unpacking hi back to fp32 and subtracting
// (two VALU ops per value).  p - hi is exact in fp32, so the operands are bitwise the same.
#ifndef WF_ATTN_DOT2
#define WF_ATTN_DOT2 1
#endif
// WF_ATTN_QP (round 6): two 16-query sub-tiles per wave in one loop (see the kernel); 0: one
#ifndef WF_ATTN_QP_VSUM
#define WF_ATTN_QP_VSUM 1
#endif
#ifndef WF_ATTN_QP
#define WF_ATTN_QP 1
#endif
template <int P>
__global__ __launch_bounds__(512, 2) void attn_tbl_kernel(const void* __restrict__ qkv,
                                                          const float* __restrict__ table,
                                                          void* __restrict__ out, int heads,
                                                          int qsplit, float scale_log2) {
  constexpr bool SPLIT = P == PREC_SPLIT;  // P: Prec (operand kind)
  constexpr int N = 512, HD = 16;
  constexpr int TBLN = 547;      // reachable rows of the (15^3, heads) table under Q2
  constexpr int KS = 32;         // K row: hi[16] | lo[16], chunks swizzled (kswz)
  // V: [hi, lo][key/4][hd][4 keys], each key-quad block padded to 136 B so the staging
  // stores (lanes 64 / 128 B apart) spread over the banks; the loop's 16-lane reads stay
  // contiguous inside one block
  constexpr int VB = HD * 4 + 4;
  constexpr int VQ = (N / 4) * VB;
  // one LDS block, the table first: its quads then sit below the 64-KiB reach of the ds_read
  // offset field, so a tile's 4 bias reads are one base register + immediates (separate
  // __shared__ arrays were placed table-last, 72 KB up: one address add per read)
#if WF_ATTN_T4
  // the reversed table as overlapping quads: tq[i] = {tbr[i], tbr[i+1], tbr[i+2], tbr[i+3]},
  // so a lane's 4 consecutive bias values are one aligned ds_read_b128
  constexpr int TQ_BYTES = TBLN * 16;
#else
  constexpr int TQ_BYTES = ((TBLN + 1) * 4 + 15) / 16 * 16;
#endif
  __shared__ __attribute__((aligned(16))) uint8_t lds_tbl[TQ_BYTES + N * KS * 2 + 2 * VQ * 2];
#if WF_ATTN_T4
  f32x4* tq = reinterpret_cast<f32x4*>(lds_tbl);
#else
  float* tbr = reinterpret_cast<float*>(lds_tbl);  // reversed, x log2 e
#endif
  uint16_t* Ks = reinterpret_cast<uint16_t*>(lds_tbl + TQ_BYTES);
  uint16_t* Vq = Ks + N * KS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int qs, h;
  int64_t bw;
  attn_block(qsplit, heads, qs, h, bw);
  const int C = heads * HD, ld = 3 * C;
  const int64_t row0 = bw * N;
  const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};

  for (int i = tid; i < TBLN; i += 512)
#if WF_ATTN_T4
  {
    // tq[j].c = tbr[j + c] = table[TBLN - 1 - j - c] (0 past the end: never read)
    const float v = table[(int64_t)i * heads + h] * 1.4426950408889634f;
    const int j = TBLN - 1 - i;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (j - c >= 0) reinterpret_cast<float*>(&tq[j - c])[c] = v;
    if (j >= TBLN - 3)
      for (int c = TBLN - j; c < 4; ++c) reinterpret_cast<float*>(&tq[j])[c] = 0.f;
  }
#else
    tbr[TBLN - 1 - i] = table[(int64_t)i * heads + h] * 1.4426950408889634f;
#endif
  for (int it = tid; it < N * 2; it += 512) {  // K: (key, 8-value chunk)
    const int key = it >> 1, ch = it & 1, sw = kswz(key);
    bf16x8 hi = z8, lo = z8;
    load8_split<P>(qkv, (row0 + key) * ld + C + h * HD + ch * 8, hi, lo);
    *reinterpret_cast<bf16x8*>(&Ks[key * KS + 8 * (ch ^ sw)]) = hi;
    *reinterpret_cast<bf16x8*>(&Ks[key * KS + 8 * ((2 + ch) ^ sw)]) = SPLIT ? lo : z8;
  }
  for (int it = tid; it < (N / 4) * 2; it += 512) {  // V: (key quad, 8-value chunk)
    const int k4 = it >> 1, ch = it & 1;
    bf16x8 vh[4], vl[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      vh[r] = z8;
      vl[r] = z8;
      load8_split<P>(qkv, (row0 + 4 * k4 + r) * ld + 2 * C + h * HD + ch * 8, vh[r], vl[r]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = k4 * VB + (ch * 8 + j) * 4;
      *reinterpret_cast<bf16x4*>(&Vq[o]) = bf16x4{vh[0][j], vh[1][j], vh[2][j], vh[3][j]};
      if (SPLIT) *reinterpret_cast<bf16x4*>(&Vq[VQ + o]) = bf16x4{vl[0][j], vl[1][j], vl[2][j], vl[3][j]};
    }
  }
  __syncthreads();

  const int l15 = lane & 15, g4 = lane >> 4;
  const int kch = 8 * (g4 ^ kswz(l15));  // this lane's K chunk (rows t*64 + kt*16 + l15)
  const short one = (short)op_cvt<P>(1.0f);
  const bf16x8 ones = bf16x8{one, one, one, one, one, one, one, one};
  const int nsub = N / 16 / qsplit;  // 16-query sub-tiles of this workgroup
#if WF_ATTN_QP
  static_assert(WF_ATTN_LAZY && WF_ATTN_MFMA_SUM && WF_ATTN_T4 && WF_ATTN_BPERMUTE,
                "the query-pair loop implements the default options only");
  // WF_ATTN_QP_VSUM (split operands): the row sums as fp32 VALU adds of the exponentials (each
  // lane's partial over its 4 keys per 16-key block, the 4 lanes of a query reduced once at
  // the end) instead of the ones-operand MFMAs (4 of 18 per tile and sub-tile): 157.0 vs
  // 159.6 us per B = 8 stage-1 launch, interleaved (profiles/r6/r6n_attn_vsum_ab.txt).  The
  // sum is then of the fp32 exponentials rather than of their hi + lo splits (closer to exact
  // by the split's 2^-16 residual).  Plain bf16 / fp16 keep the MFMA sums: their l must be
  // the sum of the same rounded P the numerator uses.
  constexpr bool VSUM = WF_ATTN_QP_VSUM && SPLIT;
  if (nsub >= 16) {
    // two independent 16-query sub-tiles per wave (st and st + 8): every K / V fragment read
    // from LDS feeds both, and the two sub-tiles' dependency chains (scores -> max -> exp ->
    // PV) interleave -- the single-sub-tile loop left the SIMDs waiting on those chains with
    // four waves each (LDS caps the workgroups at two per CU)
    constexpr int NQ = 2;
    for (int st = wid; st < nsub; st += 8 * NQ) {
      int qq[NQ], rbq[NQ];
      bf16x8 b1[NQ], b2[NQ];
      f32x4 o[NQ], l4[NQ];
      float mrun[NQ];
#pragma unroll
      for (int u = 0; u < NQ; ++u) {
        const int q = qs * (N / qsplit) + (st + 8 * u) * 16 + l15;
        qq[u] = q;
        bf16x8 hi = z8, lo = z8;
        load8_split_scaled<P>(qkv, (row0 + q) * ld + h * HD + 8 * (g4 & 1), scale_log2, hi, lo);
        b1[u] = hi;
        b2[u] = (SPLIT && g4 < 2) ? lo : z8;
        const int qz = q >> 6, qy = (q >> 3) & 7, qx = q & 7;
        rbq[u] = (TBLN - 1) - ((qz + 7) * 23 + (qy + 7) * 15 + (qx + 7)) +
                 ((g4 >> 1) * 15 + 4 * (g4 & 1));
        o[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        l4[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        mrun[u] = -INFINITY;
      }
      for (int t = 0; t < 8; ++t) {
        f32x4 s[NQ][4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(&Ks[(t * 64 + kt * 16 + l15) * KS + kch]);
#pragma unroll
          for (int u = 0; u < NQ; ++u) {
            s[u][kt] = mma32<P>(a, b1[u], tq[rbq[u] + 23 * t + 30 * kt]);
            if (SPLIT) s[u][kt] = mma32<P>(a, b2[u], s[u][kt]);
          }
        }
        float lmax[NQ];
        bool big = false;
#pragma unroll
        for (int u = 0; u < NQ; ++u) {
          lmax[u] = s[u][0][0];
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int i = (kt == 0 ? 1 : 0); i < 4; ++i) lmax[u] = fmaxf(lmax[u], s[u][kt][i]);
          big = big || lmax[u] > mrun[u] + WF_ATTN_TAU;
        }
        if (__builtin_amdgcn_ballot_w64(big) != 0) {  // wave-uniform
#pragma unroll
          for (int u = 0; u < NQ; ++u) {
            float tmax = fmaxf(mrun[u], lmax[u]);
            tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
            tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
            const float alpha = __builtin_amdgcn_exp2f(mrun[u] - tmax);  // 0 on the first tile
            mrun[u] = tmax;
            o[u] *= alpha;
            l4[u] *= alpha;
          }
        }
        uint32_t ph[NQ][4][2], pl[NQ][4][2];
#pragma unroll
        for (int u = 0; u < NQ; ++u)
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int i = 0; i < 4; i += 2) {
              const float e0 = __builtin_amdgcn_exp2f(s[u][kt][i] - mrun[u]);
              const float e1 = __builtin_amdgcn_exp2f(s[u][kt][i + 1] - mrun[u]);
              if (VSUM) l4[u][0] += e0 + e1;
              split_pair<P>(e0, e1, ph[u][kt][i >> 1], pl[u][kt][i >> 1]);
            }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int o1 = (16 * t + 8 * j + g4) * VB + l15 * 4;
          const int o2 = (16 * t + 8 * j + 4 + g4) * VB + l15 * 4;
          const bf16x4 v1 = *reinterpret_cast<const bf16x4*>(&Vq[o1]);
          const bf16x4 v2 = *reinterpret_cast<const bf16x4*>(&Vq[o2]);
          const bf16x8 vh = bf16x8{v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
          bf16x8 vl = z8;
          if (SPLIT) {
            const bf16x4 w1 = *reinterpret_cast<const bf16x4*>(&Vq[VQ + o1]);
            const bf16x4 w2 = *reinterpret_cast<const bf16x4*>(&Vq[VQ + o2]);
            vl = bf16x8{w1[0], w1[1], w1[2], w1[3], w2[0], w2[1], w2[2], w2[3]};
          }
#pragma unroll
          for (int u = 0; u < NQ; ++u) {
            const bf16x8 pb = __builtin_bit_cast(
                bf16x8, u32x4{ph[u][2 * j][0], ph[u][2 * j][1], ph[u][2 * j + 1][0], ph[u][2 * j + 1][1]});
            if (SPLIT) {
              const bf16x8 plb = __builtin_bit_cast(
                  bf16x8, u32x4{pl[u][2 * j][0], pl[u][2 * j][1], pl[u][2 * j + 1][0], pl[u][2 * j + 1][1]});
              o[u] = mma32<P>(vl, pb, o[u]);
              o[u] = mma32<P>(vh, plb, o[u]);
              if (!VSUM) l4[u] = mma32<P>(ones, plb, l4[u]);
            }
            o[u] = mma32<P>(vh, pb, o[u]);
            if (!VSUM) l4[u] = mma32<P>(ones, pb, l4[u]);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < NQ; ++u) {
        if (VSUM) {  // the 4 lanes (g4) of query l15
          l4[u][0] += __shfl_xor(l4[u][0], 16, 64);
          l4[u][0] += __shfl_xor(l4[u][0], 32, 64);
        }
        const float inv = 1.f / l4[u][0];
        const int64_t off = (row0 + qq[u]) * C + h * HD + 4 * g4;
        if (store32(P)) {
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(out) + off) = o[u] * inv;
        } else {
          bf16x4 r;
#pragma unroll
          for (int i = 0; i < 4; ++i) r[i] = (short)f2bf(o[u][i] * inv);
          *reinterpret_cast<bf16x4*>(reinterpret_cast<uint16_t*>(out) + off) = r;
        }
      }
    }
    return;
  }
#endif
  // the query-pair loop's VALU row sums, in the same order, wherever it runs (the qsplit = 4
  // launches of small grids take this loop: a volume's result must not depend on the batch)
  constexpr bool VSUM1 = WF_ATTN_QP && WF_ATTN_QP_VSUM && SPLIT && WF_ATTN_MFMA_SUM && WF_ATTN_LAZY;
  for (int st = wid; st < nsub; st += 8) {
    const int q = qs * (N / qsplit) + st * 16 + l15;
    // B operands of S: slots 8 g4 .. +7 <- Q'[q][8 (g4 & 1) ..]: [Q'h | Q'h] and [Q'l | 0]
    bf16x8 b1 = z8, b2 = z8;
    {
      bf16x8 hi = z8, lo = z8;
      load8_split_scaled<P>(qkv, (row0 + q) * ld + h * HD + 8 * (g4 & 1), scale_log2, hi, lo);
      b1 = hi;
      b2 = (SPLIT && g4 < 2) ? lo : z8;
    }
    const int qz = q >> 6, qy = (q >> 3) & 7, qx = q & 7;
    // reversed-table base of tile 0: (TBLN - 1) - index(q, key (0, 2 (g4 >> 1), 4 (g4 & 1)))
    const int rb = (TBLN - 1) - ((qz + 7) * 23 + (qy + 7) * 15 + (qx + 7)) +
                   ((g4 >> 1) * 15 + 4 * (g4 & 1));
    f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#if WF_ATTN_MFMA_SUM
    f32x4 l4 = f32x4{0.f, 0.f, 0.f, 0.f};
#else
    float lsum = 0.f;  // this lane's 16 keys of each tile; the 4 key groups are summed at the end
#endif
    float mrun = -INFINITY;
    // S^T of 64-key tile t: 4 sub-tiles of 16 keys, the accumulator starting at the bias
    auto scores = [&](int t, f32x4 (&s)[4]) {
#if WF_ATTN_T4
      const f32x4* bq = tq + rb + 23 * t;
#else
      const float* bt = tbr + rb + 23 * t;
#endif
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&Ks[(t * 64 + kt * 16 + l15) * KS + kch]);
#if WF_ATTN_T4
        const f32x4 bias = bq[30 * kt];
#else
        const f32x4 bias = f32x4{bt[30 * kt], bt[30 * kt + 1], bt[30 * kt + 2], bt[30 * kt + 3]};
#endif
        s[kt] = mma32<P>(a, b1, bias);
        if (SPLIT) s[kt] = mma32<P>(a, b2, s[kt]);
      }
    };
#pragma unroll 2
    for (int t = 0; t < 8; ++t) {  // 64-key tiles (one z slice of the window each)
      f32x4 s[4];
      scores(t, s);
#if WF_ATTN_LAZY
      float lmax = s[0][0];  // a chain, so the compiler pairs it into v_max3_f32
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = (kt == 0 ? 1 : 0); i < 4; ++i) lmax = fmaxf(lmax, s[kt][i]);
      if (__builtin_amdgcn_ballot_w64(lmax > mrun + WF_ATTN_TAU) != 0) {  // wave-uniform
        float tmax = fmaxf(mrun, lmax);
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float alpha = __builtin_amdgcn_exp2f(mrun - tmax);  // 0 on the first tile
        mrun = tmax;
        o *= alpha;
#if WF_ATTN_MFMA_SUM
        l4 *= alpha;
#else
        lsum *= alpha;
#endif
      }
      const float mnew = mrun;
#else
      float tmax = mrun;  // a chain, so the compiler pairs it into v_max3_f32
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) tmax = fmaxf(tmax, s[kt][i]);
#if WF_ATTN_BPERMUTE
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
#else
      // the 4 key groups of a query column (lanes l15 + 16 g4): xor 16 / xor 32 exchanges on
      // v_permlane16_swap / v_permlane32_swap (VALU) instead of two ds_bpermute round trips
      // on every tile's max -> exp chain
      {
        const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(tmax),
                                                          __float_as_uint(tmax), false, false);
        tmax = fmaxf(__uint_as_float(r16[0]), __uint_as_float(r16[1]));
        const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(tmax),
                                                          __float_as_uint(tmax), false, false);
        tmax = fmaxf(__uint_as_float(r32[0]), __uint_as_float(r32[1]));
      }
#endif
      const float mnew = tmax;
      const float alpha = __builtin_amdgcn_exp2f(mrun - mnew);
      mrun = mnew;
      o *= alpha;
#if WF_ATTN_MFMA_SUM
      l4 *= alpha;
#else
      lsum *= alpha;
#endif
#endif  // WF_ATTN_LAZY
      // P^T operand words: pairs of 16-bit values, hi and (bf16x3) lo parts
      uint32_t ph[4][2], pl[4][2];
#if !WF_ATTN_MFMA_SUM
      float ps[4];
#endif
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const float p0 = __builtin_amdgcn_exp2f(s[kt][i] - mnew);
          const float p1 = __builtin_amdgcn_exp2f(s[kt][i + 1] - mnew);
#if WF_ATTN_MFMA_SUM
          if (VSUM1) l4[0] += p0 + p1;
#endif
          if (WF_ATTN_DOT2) {
            split_pair<P>(p0, p1, ph[kt][i >> 1], pl[kt][i >> 1]);
          } else {
            const uint16_t hb0 = op_cvt<P>(p0), hb1 = op_cvt<P>(p1);
            ph[kt][i >> 1] = (uint32_t)hb0 | ((uint32_t)hb1 << 16);
            pl[kt][i >> 1] = (uint32_t)(uint16_t)op_lo<P>(p0, hb0) |
                             ((uint32_t)(uint16_t)op_lo<P>(p1, hb1) << 16);
          }
#if !WF_ATTN_MFMA_SUM
          ps[i] = kt == 0 ? p0 : ps[i] + p0;  // 4 chains over the key sub-tiles
          ps[i + 1] = kt == 0 ? p1 : ps[i + 1] + p1;
#endif
        }
      }
#if !WF_ATTN_MFMA_SUM
      lsum += (ps[0] + ps[1]) + (ps[2] + ps[3]);
#endif
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16x8 pb = __builtin_bit_cast(
            bf16x8, u32x4{ph[2 * j][0], ph[2 * j][1], ph[2 * j + 1][0], ph[2 * j + 1][1]});
        const int o1 = (16 * t + 8 * j + g4) * VB + l15 * 4;
        const int o2 = (16 * t + 8 * j + 4 + g4) * VB + l15 * 4;
        const bf16x4 v1 = *reinterpret_cast<const bf16x4*>(&Vq[o1]);
        const bf16x4 v2 = *reinterpret_cast<const bf16x4*>(&Vq[o2]);
        const bf16x8 vh = bf16x8{v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
        if (SPLIT) {
          const bf16x8 plb = __builtin_bit_cast(
              bf16x8, u32x4{pl[2 * j][0], pl[2 * j][1], pl[2 * j + 1][0], pl[2 * j + 1][1]});
          const bf16x4 w1 = *reinterpret_cast<const bf16x4*>(&Vq[VQ + o1]);
          const bf16x4 w2 = *reinterpret_cast<const bf16x4*>(&Vq[VQ + o2]);
          const bf16x8 vl = bf16x8{w1[0], w1[1], w1[2], w1[3], w2[0], w2[1], w2[2], w2[3]};
          o = mma32<P>(vl, pb, o);
          o = mma32<P>(vh, plb, o);
#if WF_ATTN_MFMA_SUM
          if (!VSUM1) l4 = mma32<P>(ones, plb, l4);
#endif
        }
        o = mma32<P>(vh, pb, o);
#if WF_ATTN_MFMA_SUM
        if (!VSUM1) l4 = mma32<P>(ones, pb, l4);
#endif
      }
    }
#if WF_ATTN_MFMA_SUM
    if (VSUM1) {  // the 4 lanes (g4) of query l15, as in the query-pair loop
      l4[0] += __shfl_xor(l4[0], 16, 64);
      l4[0] += __shfl_xor(l4[0], 32, 64);
    }
    const float inv = 1.f / l4[0];
#else
    lsum = xsum16(lsum);
    lsum = xsum32(lsum);
    const float inv = 1.f / lsum;
#endif
    const int64_t off = (row0 + q) * C + h * HD + 4 * g4;
    if (store32(P)) {
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(out) + off) = o * inv;
    } else {
      bf16x4 r;
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = (short)f2bf(o[i] * inv);
      *reinterpret_cast<bf16x4*>(reinterpret_cast<uint16_t*>(out) + off) = r;
    }
  }
}

static size_t attn_win_lds(int N, int hd, bool split) {
  const size_t NP = (size_t)(N + 63) / 64 * 64;
  return (split ? 2 : 1) * (NP * (hd + 4) + NP * hd) * sizeof(uint16_t);
}

int launch_attn_core(const void* qkv, const float* bias, void* out, float* lse, int64_t Bw,
                     int N, int heads, int hd, float scale, int prec, hipStream_t s,
                     int table_ws) {
  if (Bw <= 0) return WF_OK;
  const int64_t nblk = cdiv(N, kQB) * heads * Bw;
  if (nblk > 0x7fffffff) return fail(WF_E_SHAPE, "attention: too many (window, head) tiles");
  dim3 grid((unsigned)nblk);  // 1-D, decoded XCD-aware by attn_block
  const float sl2 = scale * 1.4426950408889634f;
  const bool split = prec == PREC_SPLIT;
  const bool f16 = prec == PREC_FP16;
  if (!valid_prec(prec)) return fail(WF_E_SHAPE, "attention: unknown precision");
  if (table_ws) {  // bias = the (T, heads) table; index from the coordinates
    if (table_ws != 8 || hd != 16 || N != 512)
      return fail(WF_E_SHAPE, "attention (table bias): implemented for ws = 8, head_dim = 16");
    static const bool tiled = getenv("WF_ATTN_TILED") != nullptr;  // the r1 kernel, for A/B
    if (!lse && !tiled) {
      // queries of one (window, head) split over 1, 2 or 4 workgroups: enough workgroups for
      // two per CU, each staging the window's K / V once
      const int64_t wh = Bw * heads;
      const int qsplit = wh >= 512 ? 1 : (wh >= 256 ? 2 : 4);
      const dim3 g1((unsigned)(wh * qsplit));
      auto k = split ? attn_tbl_kernel<PREC_SPLIT>
                     : (f16 ? attn_tbl_kernel<PREC_FP16> : attn_tbl_kernel<PREC_BF16>);
      hipLaunchKernelGGL(k, g1, dim3(512), 0, s, qkv, bias, out, heads, qsplit, sl2);
      return check_launch("attention core (table bias, window per workgroup)");
    }
    auto k = split ? attn_core_kernel<16, 64, PREC_SPLIT, 8>
                   : (f16 ? attn_core_kernel<16, 64, PREC_FP16, 8>
                          : attn_core_kernel<16, 64, PREC_BF16, 8>);
    hipLaunchKernelGGL(k, grid, dim3(256), 0, s, qkv, bias, out, lse, N, heads, sl2);
    return check_launch("attention core (table bias)");
  }
  // the window-resident variant measured slower (236 vs 186 us on the stage-1 launch: its
  // 74 KB of LDS leaves 2 workgroups per CU, the tiled kernel's occupancy hides more latency;
  // hoisting the tiled kernel's bias loads over its staging cost occupancy too: 206 us); opt-in
  static const bool use_win = getenv("WF_ATTN_WIN") != nullptr;
  if (use_win && !f16 && hd == 16 && attn_win_lds(N, hd, split) <= 80 * 1024) {
    const size_t lds = attn_win_lds(N, hd, split);
    auto k = split ? attn_win_kernel<16, PREC_SPLIT> : attn_win_kernel<16, PREC_BF16>;
    set_max_lds(reinterpret_cast<const void*>(k), (int)lds);
    hipLaunchKernelGGL(k, grid, dim3(256), lds, s, qkv, bias, out, lse, N, heads, sl2);
    return check_launch("attention core (window-resident)");
  }
#define WF_ATTN_CASE(HDV)                                                                  \
  case HDV: {                                                                              \
    auto k = split ? attn_core_kernel<HDV, (HDV >= 192 ? 32 : 64), PREC_SPLIT>             \
                   : (f16 ? attn_core_kernel<HDV, 64, PREC_FP16>                           \
                          : attn_core_kernel<HDV, 64, PREC_BF16>);                         \
    hipLaunchKernelGGL(k, grid, dim3(256), 0, s, qkv, bias, out, lse, N, heads, sl2);      \
    break;                                                                                 \
  }
  switch (hd) {
    WF_ATTN_CASE(16)
    WF_ATTN_CASE(32)
    WF_ATTN_CASE(48)
    WF_ATTN_CASE(64)
    WF_ATTN_CASE(96)
    WF_ATTN_CASE(128)
    WF_ATTN_CASE(192)
    WF_ATTN_CASE(384)
    default:
      return fail(WF_E_SHAPE, "attention: head_dim must be one of 16,32,48,64,96,128,192,384");
  }
#undef WF_ATTN_CASE
  return check_launch("attention core");
}

__global__ void rel_pos_bias_kernel(const float* __restrict__ table, const int64_t* __restrict__ index,
                                    float* __restrict__ bias, int64_t NN, int heads) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NN) return;
  const int64_t r = index[i];
  for (int h = 0; h < heads; ++h) bias[h * NN + i] = table[r * heads + h];
}

static int64_t act_bytes(int prec) { return store32(prec) ? 4 : 2; }

}  // namespace wf

using namespace wf;

extern "C" int wf_rel_pos_bias(const float* table, const int64_t* index, float* bias, int64_t N,
                               int64_t heads, int64_t table_rows, void* stream) {
  WF_REQUIRE(N >= 1 && heads >= 1 && table_rows >= 1, "empty bias");
  WF_REQUIRE_PTR(table);
  WF_REQUIRE_PTR(index);
  WF_REQUIRE_PTR(bias);
  const int64_t NN = N * N;
  hipLaunchKernelGGL(rel_pos_bias_kernel, dim3((unsigned)cdiv(NN, 256)), dim3(256), 0,
                     (hipStream_t)stream, table, index, bias, NN, (int)heads);
  return check_launch("wf_rel_pos_bias");
}

extern "C" int64_t wf_window_attention_workspace_bytes(int64_t B, int64_t C, int64_t D1,
                                                       int64_t H1, int64_t W1, int precision) {
  const int64_t rows = B * D1 * H1 * W1;
  const int64_t e = act_bytes(precision);
  const int64_t qkv = ((rows * 3 * C * e) + 255) & ~(int64_t)255;
  const int64_t ao = ((rows * C * e) + 255) & ~(int64_t)255;
  return qkv + ao;
}

static int window_attention_impl(const float* x, const float* ln_w, const float* ln_b,
                                 float ln_eps, const uint16_t* wqkv_bf16x2, const float* bqkv,
                                 const float* bias, int table_ws,
                                 const uint16_t* wproj_bf16x2, const float* bproj, float* out,
                                 void* workspace, float* lse, int64_t B, int64_t C, int64_t D1,
                                 int64_t H1, int64_t W1, int64_t ws, int64_t heads, float scale,
                                 int precision, void* stream) {
  WF_REQUIRE(B >= 1 && C >= 8 && C % 8 == 0, "C must be a positive multiple of 8");
  WF_REQUIRE(ws >= 1 && D1 % ws == 0 && H1 % ws == 0 && W1 % ws == 0,
             "the raster must tile into ws^3 windows (window_partition, wave_helper.py:459)");
  WF_REQUIRE(heads >= 1 && C % heads == 0, "dim must be divisible by num_heads");
  WF_REQUIRE(valid_prec(precision), "unknown precision");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(wqkv_bf16x2);
  WF_REQUIRE_PTR(bias);
  WF_REQUIRE_PTR(wproj_bf16x2);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE_PTR(workspace);
  if (ln_w) WF_REQUIRE_PTR(ln_b);
  const int64_t N = ws * ws * ws;
  const int64_t rows = B * D1 * H1 * W1;
  const int64_t Bw = rows / N;
  const int64_t e = act_bytes(precision);
  hipStream_t s = (hipStream_t)stream;
  void* qkv = workspace;
  void* ao = reinterpret_cast<char*>(workspace) + (((rows * 3 * C * e) + 255) & ~(int64_t)255);
  const int obf = !store32(precision);
  // 1. qkv = Linear(window_partition(norm1?(x)))
  GemmArgs g{};
  g.prec = precision;
  g.a_src = x;
  g.a_bf16 = 0;
  g.a_C = (int)C;
  g.a_nseg = 1;
  g.a_map = MAP_WINDOW;
  g.mB = (int)B;
  g.mD = (int)D1;
  g.mH = (int)H1;
  g.mW = (int)W1;
  g.mws = (int)ws;
  g.a_ln = ln_w ? LN_COMPUTE : LN_NONE;
  g.a_ln_w = ln_w;
  g.a_ln_b = ln_b;
  g.a_eps = ln_eps;
  g.w = wqkv_bf16x2;
  g.M = rows;
  g.N = (int)(3 * C);
  g.K = (int)C;
  g.epi = EPI_STORE;
  g.bias = bqkv;
  g.out = qkv;
  g.out_bf16 = obf;
  g.ldo = 3 * C;
  int rc = launch_gemm(g, s, "wf_window_attention_fwd(qkv)");
  if (rc) return rc;
  // 2. softmax(q k^T * scale + bias) v
  rc = launch_attn_core(qkv, bias, ao, lse, Bw, (int)N, (int)heads, (int)(C / heads), scale,
                        precision, s, table_ws);
  if (rc) return rc;
  // 3. proj; window-major rows == the reshaped raster (Q1)
  GemmArgs p{};
  p.prec = precision;
  p.a_src = ao;
  p.a_bf16 = obf;
  p.a_C = (int)C;
  p.a_nseg = 1;
  p.a_map = MAP_IDENTITY;
  p.a_ln = LN_NONE;
  p.w = wproj_bf16x2;
  p.M = rows;
  p.N = (int)C;
  p.K = (int)C;
  p.epi = EPI_STORE;
  p.bias = bproj;
  p.out = out;
  p.out_bf16 = 0;
  p.ldo = C;
  return launch_gemm(p, s, "wf_window_attention_fwd(proj)");
}

extern "C" int wf_window_attention_fwd_train(const float* x, const float* ln_w,
                                             const float* ln_b, float ln_eps,
                                             const uint16_t* wqkv_bf16x2, const float* bqkv,
                                             const float* bias, const uint16_t* wproj_bf16x2,
                                             const float* bproj, float* out, void* workspace,
                                             float* lse, int64_t B, int64_t C, int64_t D1,
                                             int64_t H1, int64_t W1, int64_t ws, int64_t heads,
                                             float scale, int precision, void* stream) {
  return window_attention_impl(x, ln_w, ln_b, ln_eps, wqkv_bf16x2, bqkv, bias, 0, wproj_bf16x2,
                               bproj, out, workspace, lse, B, C, D1, H1, W1, ws, heads, scale,
                               precision, stream);
}

extern "C" int wf_window_attention_fwd_table(const float* x, const float* ln_w,
                                             const float* ln_b, float ln_eps,
                                             const uint16_t* wqkv_bf16x2, const float* bqkv,
                                             const float* table, const uint16_t* wproj_bf16x2,
                                             const float* bproj, float* out, void* workspace,
                                             int64_t B, int64_t C, int64_t D1, int64_t H1,
                                             int64_t W1, int64_t ws, int64_t heads, float scale,
                                             int precision, void* stream) {
  WF_REQUIRE(ws == 8 && C == 16 * heads,
             "table-bias attention is implemented for window 8 and head_dim 16");
  return window_attention_impl(x, ln_w, ln_b, ln_eps, wqkv_bf16x2, bqkv, table, (int)ws,
                               wproj_bf16x2, bproj, out, workspace, nullptr, B, C, D1, H1, W1,
                               ws, heads, scale, precision, stream);
}

extern "C" int wf_window_attention_fwd(const float* x, const float* ln_w, const float* ln_b,
                                       float ln_eps, const uint16_t* wqkv_bf16x2,
                                       const float* bqkv, const float* bias,
                                       const uint16_t* wproj_bf16x2, const float* bproj,
                                       float* out, void* workspace, int64_t B, int64_t C,
                                       int64_t D1, int64_t H1, int64_t W1, int64_t ws,
                                       int64_t heads, float scale, int precision, void* stream) {
  return wf_window_attention_fwd_train(x, ln_w, ln_b, ln_eps, wqkv_bf16x2, bqkv, bias,
                                       wproj_bf16x2, bproj, out, workspace, nullptr, B, C, D1,
                                       H1, W1, ws, heads, scale, precision, stream);
}
