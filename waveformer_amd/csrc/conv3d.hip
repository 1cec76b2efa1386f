// conv3d.hip -- 3x3x3, stride 1, padding 1 convolution (the decoder's MONAI Convolution
// layers: UnetResBlock / UnetBasicBlock conv1 + conv2, UnetrIDWTBlock.conv_lf_block, monai
// dynunet_block.py:98-111 via network_backbone.py:380-407) as an implicit GEMM on the bf16
// MFMA pipes, channel-last (NDHWC) activations, fp32 in / fp32 out.
//
//   out[p, co] = bias[co] + sum_{tap, ci} W[co, ci, tap] * x[p + off(tap), ci]
//
// GEMM view: rows = output positions, columns = Cout, K = 27 * Cin ordered per 8-channel
// chunk as (tap, ci) -- 27 * 8 = 216 values, padded with zero weights to 7 K-steps of 32.
// A workgroup owns one output z-plane tile of 4 rows (y) x 16*NT columns (x) and 16*CO_T
// output channels; wave w computes row y0 + w: NT position tiles x CO_T channel tiles.
//   * per 8-channel chunk the 3 x (4+2) x (16NT+2) halo of input positions is read ONCE
//     (coalesced 64-B channel runs), split into bf16 hi / lo and parked in LDS as
//     [position][8 ch] planes; each of the 27 taps then reads its B fragments (8 channels of
//     one position, one ds_read_b128 per plane) at a shifted position -- the 27x reuse of
//     every input value is served from LDS, not L2;
//   * the weights are pre-packed fragment-major, [chunk*7 + step][hi, lo][Cout/16][64 lanes][8]
//     bf16, and staged into LDS with the activations, so the K loop is LDS reads + MFMAs only;
//   * the NEXT chunk's activations and weights are loaded into registers right after the
//     current chunk is committed to LDS, so their HBM / L2 latency hides behind 7 K-steps of
//     MFMAs (one register set, written after the barrier: the T14 staging pipeline);
//   * "transposed" product as in gemm_rows: the weight fragment is MFMA operand A (rows =
//     output channels), the activation fragment operand B (columns = positions), so each lane
//     ends with 4 consecutive output channels of one position -> one f32x4 store.
// Precision as everywhere (include/waveformer_hip.h): SPLIT = hi*hi + lo*hi + hi*lo (fp32-
// faithful), else plain bf16 operands; accumulation fp32.
// Roofline: MFMA (2 * 27 * Cin * Cout flops per position; 432 flop/B at Cin 96, Cout 48).
#include <algorithm>

#include "kernels.hpp"

namespace wf {

#ifndef WF_C3W_WDMA  // 0: conv3d_k3w stages weights through registers (round-5 form; A/B only)
#define WF_C3W_WDMA 1
#endif
#ifndef WF_CONV_DBG  // 1: timing-experiment build (Conv3Args::dbg phase skips; never the shipped library)
#define WF_CONV_DBG 0
#endif

constexpr int kConvCC = 8;                           // input channels per LDS chunk
constexpr int kConvKS = (27 * kConvCC + 31) / 32;    // K-steps of 32 per chunk (7)

struct Conv3Args {
  const float* x;     // (B, D, H, W) positions, ldx floats apart; channels [0, Cin)
  const uint16_t* w;  // [nch * kConvKS][2 (hi, lo)][Cout / 16][64 lanes][8] bf16
  const float* bias;  // (Cout) or nullptr
  float* out;         // (B, D, H, W) positions, ldo floats apart; channels [0, Cout)
  int64_t ldx, ldo;
  int B, D, H, W, Cin, Cout, nch;
  int tiles_x, tiles_y;
  int64_t nblocks;
  int64_t nblocks_pos;  // B*D*H*W: positions per split-K partial
  int ksplit;         // > 1: blockIdx.z takes chunks [z*nch/ksplit, (z+1)*nch/ksplit) and the
                      // epilogue writes its partial to part[z] (small grids only); a second
                      // pass sums the partials in z order (deterministic, no atomics)
  float* part;        // (ksplit, B*D*H*W, Cout) split-K partials (ksplit > 1)
  double* stats;      // (B, Cout, 2) fp64 {sum, sum of squares} accumulator or nullptr: the
                      // InstanceNorm statistics of the output, fused into the epilogue
  int zfirst;         // tile order: z fastest (1) or x fastest (0)
  const uint16_t* xh; // XH kernels: the input as fp16 (the operands WF_PREC_FP16 stages; same
                      // positions / ldx as x)
  int dbg;            // WF_CONV_DBG builds: 1 no activation loads, 2 no activation LDS stores,
                      // 4 no weight loads, 8 no weight LDS stores, 16 no MFMA K loop
};

// RW output rows per wave (wave w: rows w, w + 4, ...): RW = 2 halves the weight-fragment LDS
// reads per MFMA and the halo staging per output (non-split modes; the split's registers
// do not allow it)
// XH: the input is already fp16 in HBM (written by the producing norm_act with the same
// round-to-nearest-even conversion this kernel's fp16 staging applies, so the operands are
// bitwise those of the fp32 input): half the staging bytes, no convert
template <int CO_T, int NT, int P, bool PIPE = false, int RW = 1, bool XH = false>
__global__ __launch_bounds__(256, 2) void conv3d_k3_kernel(Conv3Args a) {
  constexpr bool SPLIT = P == PREC_SPLIT;  // P: Prec (operand kind)
  static_assert(!XH || P == PREC_FP16, "fp16 input only with fp16 operands");
  constexpr int TX = 16 * NT, TY = 4 * RW, HX = TX + 2, HY = TY + 2;
  constexpr int NPOS = 3 * HY * HX;
  constexpr int PS = kConvCC;                       // bf16 per position per plane
  constexpr int NPL = SPLIT ? 2 : 1;                 // operand planes staged (lo only for SPLIT)
  constexpr int NFRAG = kConvKS * NPL * CO_T;        // weight fragments (1 KB each) per chunk
  constexpr int NW = (NFRAG * 64 + 255) / 256;       // 16-B weight pieces per thread
  constexpr int QN = kConvCC / 4, PSTEP = 256 / QN;  // float4 per position, positions per pass
  constexpr int NJ = (NPOS * QN + 255) / 256;        // input float4 per thread
  // LDS: activations [hi | lo][NPOS][PS] bf16, then the chunk's weight fragments
  // [step][plane][m][lane][8] bf16 in MFMA operand order (a wave reads 1 KB contiguous)
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* s_hi = lds;
  uint16_t* s_lo = lds + NPOS * PS;                  // SPLIT only
  uint16_t* s_w = lds + NPL * NPOS * PS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g4 = lane >> 4;

  // XCD-contiguous tile order: hardware deals consecutive workgroups round-robin over the 8
  // XCDs; give each XCD a contiguous run of tiles so z / y neighbours share its L2
  int64_t t = blockIdx.x;
  if ((a.nblocks & 7) == 0) t = (t & 7) * (a.nblocks >> 3) + (t >> 3);
  int tx, ty, z, b;
  if (a.zfirst) {
    // z fastest: the workgroups an XCD runs together are consecutive z planes of one (y, x)
    // column, so each input plane's halo is read by its three z neighbours out of that XCD's
    // L2 instead of from HBM three times (large planes: 128^2 x 96 channels = 6 MB > 4 MB L2)
    z = (int)(t % a.D);
    t /= a.D;
    tx = (int)(t % a.tiles_x);
    t /= a.tiles_x;
    ty = (int)(t % a.tiles_y);
    b = (int)(t / a.tiles_y);
  } else {
    tx = (int)(t % a.tiles_x);
    t /= a.tiles_x;
    ty = (int)(t % a.tiles_y);
    t /= a.tiles_y;
    z = (int)(t % a.D);
    b = (int)(t / a.D);
  }
  const int x0 = tx * TX, y0 = ty * TY;
  const int co0 = blockIdx.y * (16 * CO_T);

  f32x4 acc[RW][CO_T][NT];
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int m = 0; m < CO_T; ++m)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[r][m][n] = f32x4{0, 0, 0, 0};

  const bf16x8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};
  const int ch_begin = (int)(((int64_t)blockIdx.z * a.nch) / a.ksplit);
  const int ch_end = (int)(((int64_t)(blockIdx.z + 1) * a.nch) / a.ksplit);

  // ---- per-lane constants, computed once (the K loop below is LDS reads and MFMAs only)
  // B fragment of K-step s: k = 32 s + 8 g4 -> tap k / CC, channels k % CC .. +7 of the halo
  // position (tap's z, wid + tap's y, l15 + tap's x); padded taps (>= 27) carry zero
  // weights, so any finite B is fine -- they read tap 26
  uint32_t boff[kConvKS];
#pragma unroll
  for (int s = 0; s < kConvKS; ++s) {
    const int k = 32 * s + 8 * g4;
    const int tap = min(k / kConvCC, 26);
    const int tz = tap / 9, tyy = (tap / 3) % 3, txx = tap % 3;
    boff[s] = (uint32_t)((((tz * HY + wid + tyy) * HX + txx + l15) * PS + k % kConvCC) * 2);
  }
  // input items j: halo position p0 + PSTEP j, channels 4 q .. +3 of the chunk; source
  // offsets relative to the chunk's channel base, clamped in range (masked to zero)
  const int q = tid % QN, p0 = tid / QN;
  uint32_t goff[NJ];
  uint32_t gmask = 0;
  {
    const int64_t plane = (int64_t)a.H * a.W;
    const int64_t sample = (int64_t)b * a.D * plane;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int pos = min(p0 + PSTEP * j, NPOS - 1);
      const int hx = pos % HX, r = pos / HX;
      const int hy = r % HY, hz = r / HY;
      const int gz = z + hz - 1, gy = y0 + hy - 1, gx = x0 + hx - 1;
      const bool ok = p0 + PSTEP * j < NPOS && gz >= 0 && gz < a.D && gy >= 0 && gy < a.H &&
                      gx >= 0 && gx < a.W;
      const int cz = min(max(gz, 0), a.D - 1), cy = min(max(gy, 0), a.H - 1),
                cx = min(max(gx, 0), a.W - 1);
      goff[j] = (uint32_t)((sample + cz * plane + (int64_t)cy * a.W + cx) * a.ldx);
      gmask |= ok ? (1u << j) : 0u;
    }
  }
  // weight pieces i = tid + 256 w: fragment f = i / 64 = (step, plane, m), lane i % 64; the
  // packed global layout is fragment-major too: [step][plane][Cout/16][64][8]
  const int64_t cblk = a.Cout / 16;

  f32x4 sa[XH ? 1 : NJ];
  bf16x4 sah[XH ? NJ : 1];
  bf16x8 sw[NW];
  auto fetch = [&](int ch) {
    // channels past Cin (the last chunk when Cin % 8 != 0) read channel 0 instead: the
    // address stays inside the tensor, commit() zeroes the value
    const int c = ch * kConvCC + 4 * q;
#if WF_CONV_DBG
    if (a.dbg & 1) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (XH) sah[j] = bf16x4{(short)ch, 0, 0, 0};
        else sa[j] = f32x4{(float)ch, 0.f, 0.f, 0.f};
      }
    } else
#endif
    if constexpr (XH) {
      const uint16_t* xs = a.xh + (c < a.Cin ? c : 0);
#pragma unroll
      for (int j = 0; j < NJ; ++j) sah[j] = *reinterpret_cast<const bf16x4*>(xs + goff[j]);
    } else {
      const float* xs = a.x + (c < a.Cin ? c : 0);
#pragma unroll
      for (int j = 0; j < NJ; ++j) sa[j] = *reinterpret_cast<const f32x4*>(xs + goff[j]);
    }
#if WF_CONV_DBG
    if (a.dbg & 4) {
#pragma unroll
      for (int w = 0; w < NW; ++w) sw[w] = bf16x8{(short)ch, 0, 0, 0, 0, 0, 0, 0};
      return;
    }
#endif
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int i = min(tid + 256 * w, NFRAG * 64 - 1);
      const int f = i >> 6, ln = i & 63;
      const int m = f % CO_T, sp = f / CO_T;  // sp = step * NPL + plane
      const int st = sp / NPL, pl = sp - st * NPL;
      const int64_t frag = ((int64_t)(ch * kConvKS + st) * 2 + pl) * cblk + co0 / 16 + m;
      sw[w] = *reinterpret_cast<const bf16x8*>(a.w + (frag * 64 + ln) * 8);
    }
  };
  auto commit = [&](int ch) {
    const bool cok = ch * kConvCC + 4 * q < a.Cin;
#if WF_CONV_DBG
    const bool skip_a = a.dbg & 2, skip_w = a.dbg & 8;
#else
    constexpr bool skip_a = false, skip_w = false;
#endif
#pragma unroll
    for (int j = 0; j < NJ && !skip_a; ++j) {
      const int pos = p0 + PSTEP * j;
      if (j == NJ - 1 && pos >= NPOS) break;
      if constexpr (XH) {
        bf16x4 h = sah[j];
        if (!cok || !((gmask >> j) & 1u)) h = bf16x4{0, 0, 0, 0};
        *reinterpret_cast<bf16x4*>(s_hi + pos * PS + 4 * q) = h;
        continue;
      }
      f32x4 v = sa[XH ? 0 : j];
      if (!cok || !((gmask >> j) & 1u)) v = f32x4{0, 0, 0, 0};
      bf16x4 h, l;
      split4<P>(v, h, l);
      *reinterpret_cast<bf16x4*>(s_hi + pos * PS + 4 * q) = h;
      if (SPLIT) *reinterpret_cast<bf16x4*>(s_lo + pos * PS + 4 * q) = l;
    }
#pragma unroll
    for (int w = 0; w < NW && !skip_w; ++w) {
      const int i = tid + 256 * w;
      if (w == NW - 1 && i >= NFRAG * 64) break;
      *reinterpret_cast<bf16x8*>(s_w + i * 8) = sw[w];
    }
  };
  const char* lb = reinterpret_cast<const char*>(lds);
  const char* lw = reinterpret_cast<const char*>(s_w) + lane * 16;

  fetch(ch_begin);
  for (int ch = ch_begin; ch < ch_end; ++ch) {
    __syncthreads();  // every wave is done with the previous chunk's LDS
    commit(ch);
    __syncthreads();
    // the next chunk's global reads fly during this chunk's MFMAs: no vmcnt wait below
    if (ch + 1 < ch_end) fetch(ch + 1);
#if WF_CONV_DBG
    if (a.dbg & 16) {
      // keep the staged values live (so the loads / stores are not removed) without MFMAs
      acc[0][0][0].x += (float)lb[tid & 63] + (float)lw[0];
      continue;
    }
#endif
#pragma unroll
    for (int s = 0; s < kConvKS; ++s) {
      bf16x8 wh[CO_T], wl[CO_T];
#pragma unroll
      for (int m = 0; m < CO_T; ++m) {
        wh[m] = *reinterpret_cast<const bf16x8*>(lw + ((s * NPL + 0) * CO_T + m) * 1024);
        wl[m] = SPLIT ? *reinterpret_cast<const bf16x8*>(lw + ((s * NPL + NPL - 1) * CO_T + m) * 1024)
                      : zero8;
      }
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        bf16x8 bh[NT], bl[NT];
        const uint32_t ro = (uint32_t)(4 * r * HX * PS * 2);  // row w + 4 r of the halo
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          bh[n] = *reinterpret_cast<const bf16x8*>(lb + boff[s] + ro + 16 * n * PS * 2);
          bl[n] = SPLIT ? *reinterpret_cast<const bf16x8*>(lb + boff[s] + ro + 16 * n * PS * 2 +
                                                             NPOS * PS * 2)
                        : zero8;
        }
#pragma unroll
        for (int n = 0; n < NT; ++n) {
#pragma unroll
          for (int m = 0; m < CO_T; ++m) {
            if (SPLIT) {
              acc[r][m][n] = mma32<P>(wh[m], bl[n], acc[r][m][n]);
              acc[r][m][n] = mma32<P>(wl[m], bh[n], acc[r][m][n]);
            }
            acc[r][m][n] = mma32<P>(wh[m], bh[n], acc[r][m][n]);
          }
        }
      }
      // keep the next step's fragment reads from being hoisted over these MFMAs (VGPRs: the
      // next chunk's prefetch registers are live across the whole loop); without the split's
      // lo operands there is room to read one step ahead (WF_CONV_PIPE A/B)
      if (SPLIT || !PIPE) __builtin_amdgcn_sched_barrier(0);
    }
  }

  // ---- InstanceNorm statistics of this tile's outputs (ksplit == 1 only): per channel, the
  // lane's NT positions, then the 16 lanes of its row (DPP), then the 4 waves (LDS), then one
  // fp64 atomic per (channel, moment) per workgroup
  if (a.stats && a.ksplit == 1) {
    f32x4 ps[CO_T], pq[CO_T];
#pragma unroll
    for (int m = 0; m < CO_T; ++m) {
      ps[m] = f32x4{0, 0, 0, 0};
      pq[m] = f32x4{0, 0, 0, 0};
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const bool rowok = y0 + wid + 4 * r < a.H;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const bool ok = rowok && x0 + 16 * n + l15 < a.W;
          f32x4 v = acc[r][m][n];
          if (a.bias) v += *reinterpret_cast<const f32x4*>(a.bias + co0 + 16 * m + 4 * g4);
          if (ok) {
            ps[m] += v;
            pq[m] += v * v;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ps[m][i] = group_sum<16>(ps[m][i]);
        pq[m][i] = group_sum<16>(pq[m][i]);
      }
    }
    __syncthreads();  // every wave is done reading the chunk tiles: reuse the LDS
    float* red = reinterpret_cast<float*>(lds);  // [4 waves][CO_T * 16][2]
    if (l15 == 0) {
#pragma unroll
      for (int m = 0; m < CO_T; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 16 * m + 4 * g4 + i;
          red[(wid * CO_T * 16 + c) * 2 + 0] = ps[m][i];
          red[(wid * CO_T * 16 + c) * 2 + 1] = pq[m][i];
        }
    }
    __syncthreads();
    for (int i = tid; i < CO_T * 16 * 2; i += 256) {
      const int c = i >> 1, mom = i & 1;
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) t += red[(w * CO_T * 16 + c) * 2 + mom];
      atomicAdd(a.stats + ((int64_t)b * a.Cout + co0 + c) * 2 + mom, (double)t);
    }
  }

  // ---- epilogue: acc[r][m][n][i] = out[(z, y0 + wid + 4 r, x0 + 16 n + l15)]
  //                                      [co0 + 16 m + 4 g4 + i]
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int gy = y0 + wid + 4 * r;
    if (gy >= a.H) break;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int gx = x0 + 16 * n + l15;
      if (gx >= a.W) continue;
      float* o = a.out + (((int64_t)(b * a.D + z) * a.H + gy) * a.W + gx) * a.ldo;
#pragma unroll
      for (int m = 0; m < CO_T; ++m) {
        const int co = co0 + 16 * m + 4 * g4;
        f32x4 v = acc[r][m][n];
        if (a.bias && blockIdx.z == 0) v += *reinterpret_cast<const f32x4*>(a.bias + co);
        if (a.ksplit > 1) {
          const int64_t p = ((int64_t)(b * a.D + z) * a.H + gy) * a.W + gx;
          *reinterpret_cast<f32x4*>(a.part + ((int64_t)blockIdx.z * a.nblocks_pos + p) * a.Cout +
                                    co) = v;
        } else {
          *reinterpret_cast<f32x4*>(o + co) = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Wide-chunk variant (non-split operands, W > 32, Cout % 48 == 0; round 5).  Phase removal in
// the WF_CONV_DBG build (profiles/r5_conv_phase_skip.txt) put 39 % of the 96 -> 48 fp16 launch
// on the activation LOADS alone: an 8-channel chunk reads 32 B of every halo position, one
// quarter of a 128-B line, and the next chunk's quarter comes back through L2 again -- the
// kernel is bound by L2 -> CU line traffic, not by MFMA or LDS.  Here a workgroup of 8 waves
// owns an 8-row x 64-column tile (wave w = row w) and stages 16 channels per step (64 B of
// every fp32 position, 32 B fp16), as two 8-channel K sub-chunks of 7 steps each behind one
// barrier pair:
//   * half the line traffic per staged byte, 3.9 instead of 4.6 halo positions per output,
//     and each weight chunk in LDS serves 512 outputs instead of 256;
//   * activations [position][16 ch] (32 B) with 16 B of padding after every 8 positions, so a
//     ds_read_b128 over 16 consecutive positions touches 16 distinct 4-bank groups;
//   * one workgroup per CU, 2 waves per SIMD as before;
//   * (round 6) the weights by LDS-DMA into two step buffers (151 KB of LDS in all): step
//     st + 1's fragments land under step st's MFMAs with no register round trip or LDS store
//     of their own; 2839-2898 vs 2929-3018 us at bf16x3 96 -> 48 128^3, 3492-3508 vs
//     3639-3678 us in the config-4 step (profiles/r6/r6ak_conv_wdma_*.txt).
// The arithmetic per output is the 8-channel kernel's (same K order, same operands): outputs
// are bitwise those of conv3d_k3_kernel (tests/test_gpu_decoder.py).
//
// PREC_SPLIT (bf16 hi + lo operands): the same 16-channel (64-B) loads, but a position's 32 B
// of LDS hold the hi and lo halves of ONE 8-channel chunk, so a load feeds two steps: lanes
// q = 0, 1 commit the first chunk, q = 2, 3 the second, and the next load is issued after the
// second commit.  The weight step is one chunk's 7 K-steps x {hi, lo} fragments.
template <int P, bool XH>
__global__ __launch_bounds__(512, 1) void conv3d_k3w_kernel(Conv3Args a) {
  constexpr bool SPLIT = P == PREC_SPLIT;
  static_assert(!XH || P == PREC_FP16, "fp16 input only with fp16 operands");
  constexpr int CO_T = 3, NT = 4, NWV = 8;
  constexpr int TX = 16 * NT, TY = NWV, HX = TX + 2, HY = TY + 2;
  constexpr int NPOS = 3 * HY * HX;                  // 1980 halo positions
  constexpr int CW = 2 * kConvCC;                    // 16 channels staged per step
  constexpr int PB = CW * 2;                         // 32 B per position
  constexpr int NFRAG = 2 * kConvKS * CO_T;          // 42 weight fragments per step
  constexpr int NW = WF_C3W_WDMA ? 1 : (NFRAG * 64 + 511) / 512;  // 16-B weight pieces per thread
  constexpr int NFW = (NFRAG + 7) / 8;               // WDMA: 1-KB fragments per wave
  constexpr int QN = XH ? CW / 8 : CW / 4;           // lanes per position (16 B each)
  constexpr int PSTEP = 512 / QN;
  constexpr int NJ = (NPOS * QN + 511) / 512;
  constexpr int ACT_B = NPOS * PB + (NPOS / 8 + 1) * 16;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  char* s_act = reinterpret_cast<char*>(lds);
  uint16_t* s_w = reinterpret_cast<uint16_t*>(s_act + ACT_B);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g4 = lane >> 4;
  auto paddr = [](int p) { return p * PB + (p >> 3) * 16; };  // byte offset of position p

  int64_t t = blockIdx.x;
  if ((a.nblocks & 7) == 0) t = (t & 7) * (a.nblocks >> 3) + (t >> 3);
  int tx, ty, z, b;
  if (a.zfirst) {
    z = (int)(t % a.D);
    t /= a.D;
    tx = (int)(t % a.tiles_x);
    t /= a.tiles_x;
    ty = (int)(t % a.tiles_y);
    b = (int)(t / a.tiles_y);
  } else {
    tx = (int)(t % a.tiles_x);
    t /= a.tiles_x;
    ty = (int)(t % a.tiles_y);
    t /= a.tiles_y;
    z = (int)(t % a.D);
    b = (int)(t / a.D);
  }
  const int x0 = tx * TX, y0 = ty * TY;
  const int co0 = blockIdx.y * (16 * CO_T);

  f32x4 acc[CO_T][NT];
#pragma unroll
  for (int m = 0; m < CO_T; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0, 0, 0, 0};

  // B fragment of K-step s (sub-chunk 0): tap (32 s + 8 g4) / 8 at halo position (tap's z,
  // wid + tap's y, l15 + tap's x) + 16 n; sub-chunk 1 reads the 16 B after it
  // (16 positions later = 2 padded groups later: paddr(p + 16 n) = paddr(p) + 544 n)
  uint32_t boff[kConvKS];
#pragma unroll
  for (int s = 0; s < kConvKS; ++s) {
    const int tap = min((32 * s + 8 * g4) / kConvCC, 26);
    const int tz = tap / 9, tyy = (tap / 3) % 3, txx = tap % 3;
    boff[s] = (uint32_t)paddr((tz * HY + wid + tyy) * HX + txx + l15);
  }
  const int q = tid % QN, p0 = tid / QN;
  uint32_t goff[NJ];
  uint32_t gmask = 0;
  {
    const int64_t plane = (int64_t)a.H * a.W;
    const int64_t sample = (int64_t)b * a.D * plane;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int pos = min(p0 + PSTEP * j, NPOS - 1);
      const int hx = pos % HX, r = pos / HX;
      const int hy = r % HY, hz = r / HY;
      const int gz = z + hz - 1, gy = y0 + hy - 1, gx = x0 + hx - 1;
      const bool ok = p0 + PSTEP * j < NPOS && gz >= 0 && gz < a.D && gy >= 0 && gy < a.H &&
                      gx >= 0 && gx < a.W;
      const int cz = min(max(gz, 0), a.D - 1), cy = min(max(gy, 0), a.H - 1),
                cx = min(max(gx, 0), a.W - 1);
      goff[j] = (uint32_t)((sample + cz * plane + (int64_t)cy * a.W + cx) * a.ldx);
      gmask |= ok ? (1u << j) : 0u;
    }
  }
  const int64_t cblk = a.Cout / 16;
  // steps: 16 channels each (the last may hold one 8-channel chunk); SPLIT: one chunk each
  const int nst = SPLIT ? a.nch : (a.nch + 1) / 2;

  f32x4 sa[XH ? 1 : NJ];
  bf16x8 sah[XH ? NJ : 1];
  bf16x8 sw[NW];
  // activations of step st (SPLIT: of steps st, st + 1, st even)
  auto fetch_act = [&](int st) {
    // channels past Cin read channel 0 (in range); commit() zeroes them
    const int c = (SPLIT ? st / 2 : st) * CW + (XH ? 8 : 4) * q;
#if WF_CONV_DBG
    if (a.dbg & 1) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (XH) sah[j] = bf16x8{(short)st, 0, 0, 0, 0, 0, 0, 0};
        else sa[j] = f32x4{(float)st, 0.f, 0.f, 0.f};
      }
      return;
    }
#endif
    if constexpr (XH) {
      const uint16_t* xs = a.xh + (c < a.Cin ? c : 0);
#pragma unroll
      for (int j = 0; j < NJ; ++j) sah[j] = *reinterpret_cast<const bf16x8*>(xs + goff[j]);
    } else {
      const float* xs = a.x + (c < a.Cin ? c : 0);
#pragma unroll
      for (int j = 0; j < NJ; ++j) sa[j] = *reinterpret_cast<const f32x4*>(xs + goff[j]);
    }
  };
  // weight fragments of step st: f = (sub * 7 + step) * CO_T + m for chunks 2 st, 2 st + 1 (a
  // missing second chunk, odd nch, reads the first one's: never used); SPLIT: f = (step * 2 +
  // plane) * CO_T + m of chunk st, the packed order
#if WF_C3W_WDMA
  // weights by LDS-DMA (buffer_load_dwordx4 ... lds, no VGPR destination) into the buffer of
  // step st's parity: wave w copies fragments w, w + 8, ... (1 KB each, lane-linear in both
  // the packed global layout and the LDS image); the buffer was last read by step st - 1's
  // K loop, which every wave left before the barrier that precedes this fetch
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.w), 0, (int)((int64_t)a.nch * kConvKS * 2 * cblk * 1024),
      0x00020000);
  auto fetch_w = [&](int st) {
    uint16_t* dst = s_w + (st & 1) * (NFRAG * 512);
#pragma unroll
    for (int i = 0; i < NFW; ++i) {
      const int f = wid + 8 * i;
      if (NFRAG % 8 != 0 && f >= NFRAG) break;
      const int m = f % CO_T, ss = f / CO_T;
      int64_t frag;
      if constexpr (SPLIT) {
        frag = ((int64_t)st * kConvKS * 2 + ss) * cblk + co0 / 16 + m;
      } else {
        const int sub = ss / kConvKS, step = ss - sub * kConvKS;
        const int ch = min(2 * st + sub, a.nch - 1);
        frag = ((int64_t)(ch * kConvKS + step) * 2) * cblk + co0 / 16 + m;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wrs, (__attribute__((address_space(3))) void*)(dst + f * 512), 16,
          (uint32_t)((frag * 64 + lane) * 16), 0, 0, 0);
    }
  };
#else
  auto fetch_w = [&](int st) {
#if WF_CONV_DBG
    if (a.dbg & 4) {
#pragma unroll
      for (int w = 0; w < NW; ++w) sw[w] = bf16x8{(short)st, 0, 0, 0, 0, 0, 0, 0};
      return;
    }
#endif
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int i = min(tid + 512 * w, NFRAG * 64 - 1);
      const int f = i >> 6, ln = i & 63;
      const int m = f % CO_T, ss = f / CO_T;
      int64_t frag;
      if constexpr (SPLIT) {
        frag = ((int64_t)st * kConvKS * 2 + ss) * cblk + co0 / 16 + m;
      } else {
        const int sub = ss / kConvKS, step = ss - sub * kConvKS;
        const int ch = min(2 * st + sub, a.nch - 1);
        frag = ((int64_t)(ch * kConvKS + step) * 2) * cblk + co0 / 16 + m;
      }
      sw[w] = *reinterpret_cast<const bf16x8*>(a.w + (frag * 64 + ln) * 8);
    }
  };
#endif
  auto fetch = [&](int st) {
    // WDMA: the weights first, so the wait for the activations (issued after) covers them
    if (WF_C3W_WDMA) fetch_w(st);
    if (!SPLIT || (st & 1) == 0) fetch_act(st);
    if (!WF_C3W_WDMA) fetch_w(st);
  };
  auto commit = [&](int st) {
    const int c = (SPLIT ? st / 2 : st) * CW + (XH ? 8 : 4) * q;
    const bool cok = c < a.Cin;
    // SPLIT: this step's chunk is held by lanes q >> 1 == st & 1 (uniform per 2 lanes)
    const bool mine = !SPLIT || (q >> 1) == (st & 1);
#if WF_CONV_DBG
    const bool skip_a = a.dbg & 2, skip_w = a.dbg & 8;
#else
    constexpr bool skip_a = false, skip_w = false;
#endif
#pragma unroll
    for (int j = 0; j < NJ && !skip_a; ++j) {
      const int pos = p0 + PSTEP * j;
      if (j == NJ - 1 && pos >= NPOS) break;
      const bool ok = cok && ((gmask >> j) & 1u);
      if constexpr (SPLIT) {
        if (mine) {
          const f32x4 v = ok ? sa[j] : f32x4{0, 0, 0, 0};
          bf16x4 h, l;
          split4<P>(v, h, l);
          *reinterpret_cast<bf16x4*>(s_act + paddr(pos) + 8 * (q & 1)) = h;
          *reinterpret_cast<bf16x4*>(s_act + paddr(pos) + 16 + 8 * (q & 1)) = l;
        }
      } else if constexpr (XH) {
        const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
        *reinterpret_cast<bf16x8*>(s_act + paddr(pos) + 16 * q) = ok ? sah[j] : z8;
      } else {
        const f32x4 v = ok ? sa[j] : f32x4{0, 0, 0, 0};
        bf16x4 h;
#pragma unroll
        for (int e = 0; e < 4; ++e) h[e] = (short)op_cvt<P>(v[e]);
        *reinterpret_cast<bf16x4*>(s_act + paddr(pos) + 8 * q) = h;
      }
    }
#if WF_C3W_WDMA
    (void)skip_w;
    // this wave's weight DMA has landed (the barrier after commit makes every wave's visible)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
#pragma unroll
    for (int w = 0; w < NW && !skip_w; ++w) {
      const int i = tid + 512 * w;
      if (w == NW - 1 && i >= NFRAG * 64) break;
      *reinterpret_cast<bf16x8*>(s_w + i * 8) = sw[w];
    }
#endif
  };
  const char* lw0 = reinterpret_cast<const char*>(s_w) + lane * 16;

  fetch(0);
  for (int st = 0; st < nst; ++st) {
    __syncthreads();  // every wave is done with the previous step's LDS
    commit(st);
    __syncthreads();
    if (st + 1 < nst) fetch(st + 1);
    const char* lw = lw0 + (WF_C3W_WDMA ? (st & 1) * NFRAG * 1024 : 0);
#if WF_CONV_DBG
    if (a.dbg & 16) {
      acc[0][0].x += (float)s_act[tid & 63] + (float)lw[0];
      continue;
    }
#endif
    if constexpr (SPLIT) {
#pragma unroll
      for (int s = 0; s < kConvKS; ++s) {
        bf16x8 wh[CO_T], wl[CO_T];
#pragma unroll
        for (int m = 0; m < CO_T; ++m) {
          wh[m] = *reinterpret_cast<const bf16x8*>(lw + ((s * 2 + 0) * CO_T + m) * 1024);
          wl[m] = *reinterpret_cast<const bf16x8*>(lw + ((s * 2 + 1) * CO_T + m) * 1024);
        }
        bf16x8 bh[NT], bl[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          bh[n] = *reinterpret_cast<const bf16x8*>(s_act + boff[s] + 544 * n);
          bl[n] = *reinterpret_cast<const bf16x8*>(s_act + boff[s] + 544 * n + 16);
        }
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int m = 0; m < CO_T; ++m) {
            acc[m][n] = mma32<P>(wh[m], bl[n], acc[m][n]);
            acc[m][n] = mma32<P>(wl[m], bh[n], acc[m][n]);
            acc[m][n] = mma32<P>(wh[m], bh[n], acc[m][n]);
          }
        __builtin_amdgcn_sched_barrier(0);
      }
      continue;
    }
    const int nsub = 2 * st + 1 < a.nch ? 2 : 1;
    for (int sub = 0; sub < nsub; ++sub) {
#pragma unroll
      for (int s = 0; s < kConvKS; ++s) {
        bf16x8 wh[CO_T];
#pragma unroll
        for (int m = 0; m < CO_T; ++m)
          wh[m] = *reinterpret_cast<const bf16x8*>(lw + ((sub * kConvKS + s) * CO_T + m) * 1024);
        bf16x8 bh[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n)
          bh[n] = *reinterpret_cast<const bf16x8*>(s_act + boff[s] + 544 * n + 16 * sub);
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int m = 0; m < CO_T; ++m) acc[m][n] = mma32<P>(wh[m], bh[n], acc[m][n]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }

  // InstanceNorm statistics (as conv3d_k3_kernel, over 8 waves)
  if (a.stats) {
    f32x4 ps[CO_T], pq[CO_T];
    const bool rowok = y0 + wid < a.H;
#pragma unroll
    for (int m = 0; m < CO_T; ++m) {
      ps[m] = f32x4{0, 0, 0, 0};
      pq[m] = f32x4{0, 0, 0, 0};
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const bool ok = rowok && x0 + 16 * n + l15 < a.W;
        f32x4 v = acc[m][n];
        if (a.bias) v += *reinterpret_cast<const f32x4*>(a.bias + co0 + 16 * m + 4 * g4);
        if (ok) {
          ps[m] += v;
          pq[m] += v * v;
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ps[m][i] = group_sum<16>(ps[m][i]);
        pq[m][i] = group_sum<16>(pq[m][i]);
      }
    }
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);  // [8 waves][CO_T * 16][2]
    if (l15 == 0) {
#pragma unroll
      for (int m = 0; m < CO_T; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 16 * m + 4 * g4 + i;
          red[(wid * CO_T * 16 + c) * 2 + 0] = ps[m][i];
          red[(wid * CO_T * 16 + c) * 2 + 1] = pq[m][i];
        }
    }
    __syncthreads();
    for (int i = tid; i < CO_T * 16 * 2; i += 512) {
      const int c = i >> 1, mom = i & 1;
      float tt = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) tt += red[(w * CO_T * 16 + c) * 2 + mom];
      atomicAdd(a.stats + ((int64_t)b * a.Cout + co0 + c) * 2 + mom, (double)tt);
    }
  }

  const int gy = y0 + wid;
  if (gy >= a.H) return;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int gx = x0 + 16 * n + l15;
    if (gx >= a.W) continue;
    float* o = a.out + (((int64_t)(b * a.D + z) * a.H + gy) * a.W + gx) * a.ldo;
#pragma unroll
    for (int m = 0; m < CO_T; ++m) {
      const int co = co0 + 16 * m + 4 * g4;
      f32x4 v = acc[m][n];
      if (a.bias) v += *reinterpret_cast<const f32x4*>(a.bias + co);
      *reinterpret_cast<f32x4*>(o + co) = v;
    }
  }
}

static size_t conv3w_lds() {
  constexpr int NPOS = 3 * 10 * 66;
  // activations + the weight fragments of one step (WDMA: of two, double-buffered)
  return (size_t)NPOS * 32 + (NPOS / 8 + 1) * 16 +
         (size_t)(WF_C3W_WDMA ? 2 : 1) * 2 * kConvKS * 3 * 1024;
}

// out[p][c] = sum_z part[z][p][c], z ascending (the split-K partials, bias in part[0])
__global__ void splitk_sum_kernel(const float* __restrict__ part, float* __restrict__ out,
                                  int64_t ldo, int C, int64_t P, int ksplit) {
  const int C4 = C >> 2;
  const int64_t total = P * C4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / C4;
    const int c = 4 * (int)(i - p * C4);
    f32x4 v = *reinterpret_cast<const f32x4*>(part + p * C + c);
    for (int z = 1; z < ksplit; ++z)
      v += *reinterpret_cast<const f32x4*>(part + ((int64_t)z * P + p) * C + c);
    *reinterpret_cast<f32x4*>(out + p * ldo + c) = v;
  }
}

// the split-K factor launch_conv3 picks for a grid of wgs workgroups (0 workspace: no split)
inline int conv3_ksplit(int64_t wgs, int nch) {
  return (wgs < 512 && nch > 1) ? (int)std::min<int64_t>(nch, cdiv(1024, wgs)) : 1;
}

// the wide-chunk kernel (conv3d_k3w_kernel): fp16 / bf16 operands, Cout % 48 == 0, W > 32, no
// split-K; WF_CONV_WIDE=0 keeps the 8-channel kernels
static bool conv3w_ok(const Conv3Args& a, int prec, int64_t wgs) {
  static const bool on = !getenv("WF_CONV_WIDE") || getenv("WF_CONV_WIDE")[0] != '0';
  // Cin > 88 for fp16 / bf16: at 48 input channels (3 steps per tile) the exposed per-tile
  // prologue of the one workgroup per CU costs more than the wider loads save
  // (profiles/r5_conv_wide_ab.txt); the split's longer K loop (three MFMAs per product) hides
  // it at 128^3: 48 -> 48 1607-1616 vs 1627-1655 us at B = 2 (profiles/r6/r6p_conv_wide48_ab.txt),
  // 3523 vs 3590 at B = 4; at 64^3 (2048 workgroups, eight per CU in turn) it measured 5 %
  // slower (profiles/r6/r6q.txt), so only planes wider than 64
  static const int env_min = getenv("WF_CONV_WIDE_MINCIN") ? atoi(getenv("WF_CONV_WIDE_MINCIN")) : 0;
  const int min_cin = env_min ? env_min : (prec == PREC_SPLIT && !a.xh && a.W > 64 ? 48 : 89);
  // fp16 input: 16-B loads of 8 channels (16-B aligned rows and channel offsets)
  return on && a.Cout % 48 == 0 && a.W > 32 && wgs >= 512 && a.Cin >= min_cin &&
         (!a.xh || (a.Cin % 8 == 0 && a.ldx % 8 == 0 && ((uintptr_t)a.xh & 15) == 0));
}

static int launch_conv3w(const Conv3Args& a0, int prec, hipStream_t stream) {
  Conv3Args a = a0;
  a.tiles_x = (int)cdiv(a.W, 64);
  a.tiles_y = (int)cdiv(a.H, 8);
  a.nblocks = (int64_t)a.B * a.D * a.tiles_y * a.tiles_x;
  if (a.nblocks >= ((int64_t)1 << 31)) return fail(WF_E_SHAPE, "wf_conv3d_k3_fwd: too many tiles");
  a.ksplit = 1;
  static const int zf = getenv("WF_CONV_ZFIRST") ? atoi(getenv("WF_CONV_ZFIRST")) : 1;
  a.zfirst = zf;
  a.dbg = WF_CONV_DBG && getenv("WF_CONV_DBG") ? atoi(getenv("WF_CONV_DBG")) : 0;
  auto kern = a.xh ? conv3d_k3w_kernel<PREC_FP16, true>
              : prec == PREC_SPLIT ? conv3d_k3w_kernel<PREC_SPLIT, false>
              : prec == PREC_FP16 ? conv3d_k3w_kernel<PREC_FP16, false>
                                  : conv3d_k3w_kernel<PREC_BF16, false>;
  const size_t lds = conv3w_lds();
  set_max_lds(reinterpret_cast<const void*>(kern), (int)lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)a.nblocks, (unsigned)(a.Cout / 48), 1), dim3(512), lds,
                     stream, a);
  return check_launch("wf_conv3d_k3_fwd (wide chunks)");
}

template <int CO_T, int NT, int RW = 1>
static int launch_conv3(const Conv3Args& a0, int prec, hipStream_t stream) {
  Conv3Args a = a0;
  constexpr int TX = 16 * NT;
  a.tiles_x = (int)cdiv(a.W, TX);
  a.tiles_y = (int)cdiv(a.H, 4 * RW);
  a.nblocks = (int64_t)a.B * a.D * a.tiles_y * a.tiles_x;
  if (a.nblocks >= ((int64_t)1 << 31)) return fail(WF_E_SHAPE, "wf_conv3d_k3_fwd: too many tiles");
  // operand planes staged: hi + lo for the split, hi only otherwise (half the LDS: twice the
  // workgroups per CU for bf16 / fp16)
  const size_t npl = prec == PREC_SPLIT ? 2 : 1;
  const size_t lds = (npl * 3 * (4 * RW + 2) * (TX + 2) * kConvCC +
                      (size_t)kConvKS * npl * CO_T * 512) * sizeof(uint16_t);
  // small grids (the 8^3 / 16^3 decoder convs): split the Cin chunks over blockIdx.z so the
  // launch covers the 256 CUs; the partials go to the caller's workspace and are summed in a
  // fixed order by splitk_sum (bitwise repeatable; no split without a workspace)
  const int64_t wgs = a.nblocks * (a.Cout / (16 * CO_T));
  a.nblocks_pos = (int64_t)a.B * a.D * a.H * a.W;
  a.ksplit = a.part ? conv3_ksplit(wgs, a.nch) : 1;
  if (a.ksplit == 1 && conv3w_ok(a, prec, wgs)) return launch_conv3w(a0, prec, stream);
  dim3 grid((unsigned)a.nblocks, (unsigned)(a.Cout / (16 * CO_T)), (unsigned)a.ksplit);
  const bool post_stats = a.stats && a.ksplit > 1;  // partial outputs: a separate pass below
  static const int zf = getenv("WF_CONV_ZFIRST") ? atoi(getenv("WF_CONV_ZFIRST")) : 1;
  a.zfirst = zf;
  a.dbg = WF_CONV_DBG && getenv("WF_CONV_DBG") ? atoi(getenv("WF_CONV_DBG")) : 0;
  // WF_CONV_PIPE=1 (A/B): non-split kernels without the per-K-step scheduling fence, so the
  // next step's fragment reads can be issued under the current step's MFMAs
  static const bool pipe = getenv("WF_CONV_PIPE") && getenv("WF_CONV_PIPE")[0] == '1';
  {
    auto kern = a.xh                ? (pipe ? conv3d_k3_kernel<CO_T, NT, PREC_FP16, true, RW, true>
                                            : conv3d_k3_kernel<CO_T, NT, PREC_FP16, false, RW, true>)
                : prec == PREC_SPLIT  ? conv3d_k3_kernel<CO_T, NT, PREC_SPLIT, false, 1>
                : prec == PREC_FP16 ? (pipe ? conv3d_k3_kernel<CO_T, NT, PREC_FP16, true, RW>
                                            : conv3d_k3_kernel<CO_T, NT, PREC_FP16, false, RW>)
                                    : (pipe ? conv3d_k3_kernel<CO_T, NT, PREC_BF16, true, RW>
                                            : conv3d_k3_kernel<CO_T, NT, PREC_BF16, false, RW>);
    set_max_lds(reinterpret_cast<const void*>(kern), (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, stream, a);
  }
  int rc = check_launch("wf_conv3d_k3_fwd");
  if (rc) return rc;
  if (a.ksplit > 1) {
    const int64_t total = a.nblocks_pos * (a.Cout / 4);
    hipLaunchKernelGGL(splitk_sum_kernel,
                       dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 8192)), dim3(256), 0,
                       stream, a.part, a.out, a.ldo, a.Cout, a.nblocks_pos, a.ksplit);
    rc = check_launch("wf_conv3d_k3_fwd (split-K sum)");
    if (rc) return rc;
  }
  if (!post_stats) return 0;
  return launch_instnorm_partial(a.out, a.ldo, a.B, a.Cout, (int64_t)a.D * a.H * a.W, a.stats,
                                 stream);
}

}  // namespace wf

using namespace wf;

extern "C" int64_t wf_conv3d_k3_packed_elems(int64_t Cin, int64_t Cout) {
  return 2 * cdiv(Cin, kConvCC) * kConvKS * Cout * 32;
}

namespace wf {
// packed[(gs * 2 + plane) * (Cout / 16) + co / 16][lane][e], lane = co % 16 + 16 (j / 8),
// e = j % 8 for K index kk = 32 ss + j of K-step gs = ch * KS + ss: tap kk / CC, input channel
// CC ch + kk % CC -- each 16 x 32 MFMA A fragment is 1 KB contiguous, in lane order
__global__ void conv3d_k3_pack_kernel(const float* __restrict__ w, uint16_t* __restrict__ packed,
                                      int Cin, int Cout, int64_t total, int f16) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int e = (int)(i & 7), ln = (int)((i >> 3) & 63);
  int64_t r = i >> 9;
  const int cb = (int)(r % (Cout / 16));
  r /= (Cout / 16);
  const int plane = (int)(r & 1);
  const int gs = (int)(r >> 1);
  const int co = cb * 16 + (ln & 15);
  const int j = 8 * (ln >> 4) + e;
  const int ch = gs / kConvKS, ss = gs - ch * kConvKS;
  const int kk = 32 * ss + j;
  const int tap = kk / kConvCC, ci = ch * kConvCC + kk % kConvCC;
  const float v = (tap < 27 && ci < Cin) ? w[((int64_t)co * Cin + ci) * 27 + tap] : 0.f;
  if (f16) {  // WF_PREC_FP16: plane 0 = fp16(w), plane 1 unused
    packed[i] = plane ? (uint16_t)0 : f2h(v);
    return;
  }
  const uint16_t h = f2bf(v);
  packed[i] = plane ? f2bf(v - bf2f(h)) : h;
}
}  // namespace wf

static int conv_pack(const float* w, uint16_t* packed, int64_t Cin, int64_t Cout, int f16,
                     void* stream) {
  WF_REQUIRE(Cin >= 1 && Cout >= 16 && Cout % 16 == 0, "Cout must be a multiple of 16");
  WF_REQUIRE_PTR(w);
  WF_REQUIRE_PTR(packed);
  const int64_t total = wf_conv3d_k3_packed_elems(Cin, Cout);
  hipLaunchKernelGGL(conv3d_k3_pack_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, w, packed, (int)Cin, (int)Cout, total, f16);
  return check_launch("wf_conv3d_k3_pack");
}

extern "C" int wf_conv3d_k3_pack(const float* w, uint16_t* packed, int64_t Cin, int64_t Cout,
                                 void* stream) {
  return conv_pack(w, packed, Cin, Cout, 0, stream);
}

extern "C" int wf_conv3d_k3_pack_f16(const float* w, uint16_t* packed, int64_t Cin, int64_t Cout,
                                     void* stream) {
  return conv_pack(w, packed, Cin, Cout, 1, stream);
}

namespace {
// the tile shape conv3_fwd dispatches to: CO_T output-channel tiles, NT x tiles, RW rows
struct Conv3Plan {
  int co_t, nt, rw;
};
Conv3Plan conv3_plan(int64_t Cout, int64_t W, int precision, bool xh) {
  const bool co3 = Cout % 48 == 0;
  // two output rows per wave (8-row tiles: halo 10/8 rows instead of 6/4), non-split modes,
  // W > 32.  Default for fp16 input only: with fp32 input the larger halo's prefetch registers
  // spill (96->48 at 128^3 fp16: 1.82 vs 1.73 ms); the fp16-input variant fits (240 VGPRs) and
  // runs 48->48 at 192^3 in 2.42 vs 2.52 ms (profiles/r3_conv/rw2_xh_ab_192.txt).
  // WF_CONV_RW=1 / 2 forces one or the other
  static const int rw = getenv("WF_CONV_RW") ? atoi(getenv("WF_CONV_RW")) : 0;
  if (W > 32 && precision != PREC_SPLIT && co3 && (rw == 2 || (rw == 0 && xh))) return {3, 4, 2};
  const int nt = W > 32 ? 4 : (W > 16 ? 2 : 1);
  return {co3 ? 3 : 1, nt, 1};
}
}  // namespace

extern "C" int64_t wf_conv3d_k3_workspace_bytes(int64_t B, int64_t Cin, int64_t Cout, int64_t D,
                                                int64_t H, int64_t W, int precision,
                                                int fp16_input) {
  if (B < 1 || D < 1 || H < 1 || W < 1 || Cin < 4 || Cout < 16 || Cout % 16) return -1;
  const Conv3Plan pl = conv3_plan(Cout, W, fp16_input ? PREC_FP16 : precision, fp16_input != 0);
  const int64_t nblocks = B * D * cdiv(H, 4 * pl.rw) * cdiv(W, 16 * pl.nt);
  const int ks = conv3_ksplit(nblocks * (Cout / (16 * pl.co_t)), (int)cdiv(Cin, kConvCC));
  return ks > 1 ? (int64_t)ks * B * D * H * W * Cout * 4 : 0;
}

static int conv3_fwd(const float* x, const uint16_t* xh, int64_t ldx, const uint16_t* w_packed,
                     const float* bias, float* out, int64_t ldo, double* stats_acc, void* work,
                     int64_t B, int64_t Cin, int64_t Cout, int64_t D, int64_t H, int64_t W,
                     int precision, void* stream) {
  WF_REQUIRE(B >= 1 && D >= 1 && H >= 1 && W >= 1, "empty tensor");
  WF_REQUIRE(Cin >= 4 && Cin % 4 == 0 && ldx >= Cin && ldx % 4 == 0,
             "Cin must be a positive multiple of 4 with ldx >= Cin, ldx % 4 == 0");
  WF_REQUIRE(Cout >= 16 && Cout % 16 == 0 && ldo >= Cout && ldo % 4 == 0,
             "Cout must be a positive multiple of 16 with ldo >= Cout, ldo % 4 == 0");
  WF_REQUIRE(B * D * H * W < ((int64_t)1 << 31) && B * D * H * W * ldx < ((int64_t)1 << 32),
             "input too large (32-bit element offsets)");
  WF_REQUIRE(valid_prec(precision), "unknown precision");
  WF_REQUIRE(x || xh, "x is NULL");
  WF_REQUIRE_PTR(w_packed);
  WF_REQUIRE_PTR(out);
  Conv3Args a{};
  a.x = x;
  a.xh = xh;
  a.w = w_packed;
  a.bias = bias;
  a.out = out;
  a.ldx = ldx;
  a.ldo = ldo;
  a.B = (int)B; a.D = (int)D; a.H = (int)H; a.W = (int)W;
  a.Cin = (int)Cin;
  a.Cout = (int)Cout;
  a.nch = (int)cdiv(Cin, kConvCC);
  a.stats = stats_acc;
  a.part = static_cast<float*>(work);
  hipStream_t s = (hipStream_t)stream;
  const Conv3Plan pl = conv3_plan(Cout, W, precision, xh != nullptr);
  if (pl.rw == 2) return launch_conv3<3, 4, 2>(a, precision, s);
  if (pl.nt == 4) return pl.co_t == 3 ? launch_conv3<3, 4>(a, precision, s) : launch_conv3<1, 4>(a, precision, s);
  if (pl.nt == 2) return pl.co_t == 3 ? launch_conv3<3, 2>(a, precision, s) : launch_conv3<1, 2>(a, precision, s);
  return pl.co_t == 3 ? launch_conv3<3, 1>(a, precision, s) : launch_conv3<1, 1>(a, precision, s);
}

extern "C" int wf_conv3d_k3_fwd(const float* x, int64_t ldx, const uint16_t* w_packed,
                                const float* bias, float* out, int64_t ldo, double* stats_acc,
                                void* workspace, int64_t B, int64_t Cin, int64_t Cout, int64_t D,
                                int64_t H, int64_t W, int precision, void* stream) {
  WF_REQUIRE_PTR(x);
  return conv3_fwd(x, nullptr, ldx, w_packed, bias, out, ldo, stats_acc, workspace, B, Cin, Cout,
                   D, H, W, precision, stream);
}

extern "C" int wf_conv3d_k3_fwd_xh(const uint16_t* x, int64_t ldx, const uint16_t* w_packed_f16,
                                   const float* bias, float* out, int64_t ldo, double* stats_acc,
                                   void* workspace, int64_t B, int64_t Cin, int64_t Cout,
                                   int64_t D, int64_t H, int64_t W, void* stream) {
  WF_REQUIRE_PTR(x);
  WF_REQUIRE(((uintptr_t)x & 7) == 0, "x must be 8-byte aligned");
  return conv3_fwd(nullptr, x, ldx, w_packed_f16, bias, out, ldo, stats_acc, workspace, B, Cin,
                   Cout, D, H, W, PREC_FP16, stream);
}
