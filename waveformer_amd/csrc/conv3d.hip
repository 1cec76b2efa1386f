// conv3d.hip -- 3x3x3, stride 1, padding 1 convolution (the decoder's MONAI Convolution
// layers: UnetResBlock / UnetBasicBlock conv1 + conv2, UnetrIDWTBlock.conv_lf_block, monai
// dynunet_block.py:98-111 via network_backbone.py:380-407) as an implicit GEMM on the bf16
// MFMA pipes, channel-last (NDHWC) activations, fp32 in / fp32 out.
//
//   out[p, co] = bias[co] + sum_{tap, ci} W[co, ci, tap] * x[p + off(tap), ci]
//
// GEMM view: rows = output positions, columns = Cout, K = 27 * Cin ordered per 16-channel
// chunk as (tap, ci) -- 27 * 16 = 432 values, padded with zero weights to 14 K-steps of 32.
// A workgroup owns one output z-plane tile of 4 rows (y) x 16*NT columns (x) and 16*CO_T
// output channels; wave w computes row y0 + w: NT position tiles x CO_T channel tiles.
//   * per 16-channel chunk the 3 x (4+2) x (16NT+2) halo of input positions is read ONCE
//     (coalesced 64-B channel runs), split into bf16 hi / lo and parked in LDS as
//     [position][16 ch] planes; each of the 27 taps then reads its B fragments (8 channels of
//     one position, one ds_read_b128 per plane) at a shifted position -- the 27x reuse of
//     every input value is served from LDS, not L2;
//   * the weights are pre-packed [2][chunk*14 + step][Cout][32] bf16 (hi plane, lo plane) so
//     a lane's A fragment (8 consecutive K of one output channel) is one 16-B load; the next
//     K-step's fragments are prefetched into registers while the current step's MFMAs run;
//   * "transposed" product as in gemm_rows: the weight fragment is MFMA operand A (rows =
//     output channels), the activation fragment operand B (columns = positions), so each lane
//     ends with 4 consecutive output channels of one position -> one f32x4 store.
// Precision as everywhere (include/waveformer_hip.h): SPLIT = hi*hi + lo*hi + hi*lo (fp32-
// faithful), else plain bf16 operands; accumulation fp32.
// Roofline: MFMA (2 * 27 * Cin * Cout flops per position; 432 flop/B at Cin 96, Cout 48).
#include <algorithm>

#include "kernels.hpp"

namespace wf {

constexpr int kConvCC = 16;                          // input channels per LDS chunk
constexpr int kConvKS = (27 * kConvCC + 31) / 32;    // 14 K-steps of 32 per chunk

struct Conv3Args {
  const float* x;     // (B, D, H, W) positions, ldx floats apart; channels [0, Cin)
  const uint16_t* w;  // [2][nch * kConvKS][Cout][32] bf16 (hi plane, then lo plane)
  const float* bias;  // (Cout) or nullptr
  float* out;         // (B, D, H, W) positions, ldo floats apart; channels [0, Cout)
  int64_t ldx, ldo, wplane;
  int B, D, H, W, Cin, Cout, nch;
  int tiles_x, tiles_y;
  int64_t nblocks;
  int ksplit;         // > 1: blockIdx.z takes chunks [z*nch/ksplit, (z+1)*nch/ksplit) and the
                      // epilogue atomically adds into a zeroed output (small grids only)
};

template <int CO_T, int NT, bool SPLIT>
__global__ __launch_bounds__(256, 2) void conv3d_k3_kernel(Conv3Args a) {
  constexpr int TX = 16 * NT, TY = 4, HX = TX + 2, HY = TY + 2;
  constexpr int NPOS = 3 * HY * HX;
  constexpr int PS = kConvCC;  // bf16 per position per plane
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];  // [2][NPOS][PS]
  uint16_t* s_hi = lds;
  uint16_t* s_lo = lds + NPOS * PS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g4 = lane >> 4;

  // XCD-contiguous tile order: hardware deals consecutive workgroups round-robin over the 8
  // XCDs; give each XCD a contiguous run of tiles so z / y neighbours share its L2
  int64_t t = blockIdx.x;
  if ((a.nblocks & 7) == 0) t = (t & 7) * (a.nblocks >> 3) + (t >> 3);
  const int tx = (int)(t % a.tiles_x);
  t /= a.tiles_x;
  const int ty = (int)(t % a.tiles_y);
  t /= a.tiles_y;
  const int z = (int)(t % a.D);
  const int b = (int)(t / a.D);
  const int x0 = tx * TX, y0 = ty * TY;
  const int co0 = blockIdx.y * (16 * CO_T);

  f32x4 acc[CO_T][NT];
#pragma unroll
  for (int m = 0; m < CO_T; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0, 0, 0, 0};

  const bf16x8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};
  const int ch_begin = (int)(((int64_t)blockIdx.z * a.nch) / a.ksplit);
  const int ch_end = (int)(((int64_t)(blockIdx.z + 1) * a.nch) / a.ksplit);
  const int nsteps = ch_end * kConvKS;
  // A fragment of step s for channel tile m: W[s][co0 + 16m + l15][8 g4 .. 8 g4 + 7]
  auto wptr = [&](int s, int m) {
    return a.w + ((int64_t)s * a.Cout + co0 + 16 * m + l15) * 32 + 8 * g4;
  };
  bf16x8 wh[CO_T], wl[CO_T];
#pragma unroll
  for (int m = 0; m < CO_T; ++m) {
    wh[m] = *reinterpret_cast<const bf16x8*>(wptr(ch_begin * kConvKS, m));
    wl[m] = SPLIT ? *reinterpret_cast<const bf16x8*>(wptr(ch_begin * kConvKS, m) + a.wplane)
                  : zero8;
  }

  for (int ch = ch_begin; ch < ch_end; ++ch) {
    __syncthreads();  // the previous chunk's fragment reads are done
    // ---- stage the halo tile of channels [16 ch, 16 ch + 16): NPOS x 4 float4
    for (int i = tid; i < NPOS * 4; i += 256) {
      const int q = i & 3, pos = i >> 2;
      const int hx = pos % HX, r = pos / HX;
      const int hy = r % HY, hz = r / HY;
      const int gz = z + hz - 1, gy = y0 + hy - 1, gx = x0 + hx - 1;
      const int c = ch * kConvCC + 4 * q;
      f32x4 v = {0, 0, 0, 0};
      if (gz >= 0 && gz < a.D && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W && c < a.Cin)
        v = *reinterpret_cast<const f32x4*>(
            a.x + (((int64_t)(b * a.D + gz) * a.H + gy) * a.W + gx) * a.ldx + c);
      bf16x4 h, l;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint16_t hb = f2bf(v[j]);
        h[j] = (short)hb;
        l[j] = SPLIT ? (short)f2bf(v[j] - bf2f(hb)) : (short)0;
      }
      *reinterpret_cast<bf16x4*>(s_hi + pos * PS + 4 * q) = h;
      if (SPLIT) *reinterpret_cast<bf16x4*>(s_lo + pos * PS + 4 * q) = l;
    }
    __syncthreads();

#pragma unroll 1
    for (int s = 0; s < kConvKS; ++s) {
      const int gs = ch * kConvKS + s;
      // prefetch the next step's weight fragments
      bf16x8 nh[CO_T], nl[CO_T];
      const int ns = min(gs + 1, nsteps - 1);
#pragma unroll
      for (int m = 0; m < CO_T; ++m) {
        nh[m] = *reinterpret_cast<const bf16x8*>(wptr(ns, m));
        nl[m] = SPLIT ? *reinterpret_cast<const bf16x8*>(wptr(ns, m) + a.wplane) : zero8;
      }
      // this lane's K slice: k = 32 s + 8 g4 -> tap k / 16, channels (k % 16) .. +7; the
      // padded taps 27.. carry zero weights, their B fragment just has to be finite
      const int k = 32 * s + 8 * g4;
      const int tap = min(k >> 4, 26), ci0 = k & 15;
      const int tz = tap / 9, tyy = (tap / 3) % 3, txx = tap % 3;
      const int base = ((tz * HY + wid + tyy) * HX + txx + l15) * PS + ci0;
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int off = base + 16 * n * PS;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(s_hi + off);
        if (SPLIT) {
          const bf16x8 bl = *reinterpret_cast<const bf16x8*>(s_lo + off);
#pragma unroll
          for (int m = 0; m < CO_T; ++m) {
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[m], bl, acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[m], bh, acc[m][n], 0, 0, 0);
          }
        }
#pragma unroll
        for (int m = 0; m < CO_T; ++m)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[m], bh, acc[m][n], 0, 0, 0);
      }
#pragma unroll
      for (int m = 0; m < CO_T; ++m) {
        wh[m] = nh[m];
        wl[m] = nl[m];
      }
    }
  }

  // ---- epilogue: acc[m][n][i] = out[(z, y0 + wid, x0 + 16 n + l15)][co0 + 16 m + 4 g4 + i]
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
      if (a.bias && blockIdx.z == 0) v += *reinterpret_cast<const f32x4*>(a.bias + co);
      if (a.ksplit > 1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) atomicAdd(o + co + j, v[j]);
      } else {
        *reinterpret_cast<f32x4*>(o + co) = v;
      }
    }
  }
}

// zero channels [0, C) of P channel-last positions (the split-K output)
__global__ void zero_cl_kernel(float* __restrict__ out, int64_t ldo, int C, int64_t total) {
  const int C4 = C >> 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / C4;
    *reinterpret_cast<f32x4*>(out + p * ldo + 4 * (i - p * C4)) = f32x4{0, 0, 0, 0};
  }
}

template <int CO_T, int NT>
static int launch_conv3(const Conv3Args& a0, int prec, hipStream_t stream) {
  Conv3Args a = a0;
  constexpr int TX = 16 * NT;
  a.tiles_x = (int)cdiv(a.W, TX);
  a.tiles_y = (int)cdiv(a.H, 4);
  a.nblocks = (int64_t)a.B * a.D * a.tiles_y * a.tiles_x;
  if (a.nblocks >= ((int64_t)1 << 31)) return fail(WF_E_SHAPE, "wf_conv3d_k3_fwd: too many tiles");
  const size_t lds = (size_t)2 * 3 * 6 * (TX + 2) * kConvCC * sizeof(uint16_t);
  // small grids (the 8^3 / 16^3 decoder convs): split the Cin chunks over blockIdx.z so the
  // launch covers the 256 CUs; partial sums meet in the zeroed output through fp32 atomics
  const int64_t wgs = a.nblocks * (a.Cout / (16 * CO_T));
  a.ksplit = 1;
  if (wgs < 512 && a.nch > 1) {
    a.ksplit = (int)std::min<int64_t>(a.nch, cdiv(1024, wgs));
    const int64_t total = (int64_t)a.B * a.D * a.H * a.W * (a.Cout / 4);
    hipLaunchKernelGGL(zero_cl_kernel, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 4096)),
                       dim3(256), 0, stream, a.out, a.ldo, a.Cout, total);
  }
  dim3 grid((unsigned)a.nblocks, (unsigned)(a.Cout / (16 * CO_T)), (unsigned)a.ksplit);
  if (prec == PREC_SPLIT) {
    auto kern = conv3d_k3_kernel<CO_T, NT, true>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, stream, a);
  } else {
    auto kern = conv3d_k3_kernel<CO_T, NT, false>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, stream, a);
  }
  return check_launch("wf_conv3d_k3_fwd");
}

}  // namespace wf

using namespace wf;

extern "C" int64_t wf_conv3d_k3_packed_elems(int64_t Cin, int64_t Cout) {
  return 2 * cdiv(Cin, kConvCC) * kConvKS * Cout * 32;
}

namespace wf {
// packed[plane][ch * 14 + ss][co][j]: K index kk = 32 ss + j -> tap kk / 16, ci 16 ch + kk % 16
__global__ void conv3d_k3_pack_kernel(const float* __restrict__ w, uint16_t* __restrict__ packed,
                                      int Cin, int Cout, int64_t plane) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= plane) return;
  const int j = (int)(i & 31);
  int64_t r = i >> 5;
  const int co = (int)(r % Cout);
  const int s = (int)(r / Cout);
  const int ch = s / kConvKS, ss = s - ch * kConvKS;
  const int kk = 32 * ss + j;
  const int tap = kk >> 4, ci = ch * kConvCC + (kk & 15);
  const float v = (tap < 27 && ci < Cin) ? w[((int64_t)co * Cin + ci) * 27 + tap] : 0.f;
  const uint16_t h = f2bf(v);
  packed[i] = h;
  packed[plane + i] = f2bf(v - bf2f(h));
}
}  // namespace wf

extern "C" int wf_conv3d_k3_pack(const float* w, uint16_t* packed, int64_t Cin, int64_t Cout,
                                 void* stream) {
  WF_REQUIRE(Cin >= 1 && Cout >= 1, "empty weight");
  WF_REQUIRE_PTR(w);
  WF_REQUIRE_PTR(packed);
  const int64_t plane = wf_conv3d_k3_packed_elems(Cin, Cout) / 2;
  hipLaunchKernelGGL(conv3d_k3_pack_kernel, dim3((unsigned)cdiv(plane, 256)), dim3(256), 0,
                     (hipStream_t)stream, w, packed, (int)Cin, (int)Cout, plane);
  return check_launch("wf_conv3d_k3_pack");
}

extern "C" int wf_conv3d_k3_fwd(const float* x, int64_t ldx, const uint16_t* w_packed,
                                const float* bias, float* out, int64_t ldo, int64_t B,
                                int64_t Cin, int64_t Cout, int64_t D, int64_t H, int64_t W,
                                int precision, void* stream) {
  WF_REQUIRE(B >= 1 && D >= 1 && H >= 1 && W >= 1, "empty tensor");
  WF_REQUIRE(Cin >= 4 && Cin % 4 == 0 && ldx >= Cin && ldx % 4 == 0,
             "Cin must be a positive multiple of 4 with ldx >= Cin, ldx % 4 == 0");
  WF_REQUIRE(Cout >= 16 && Cout % 16 == 0 && ldo >= Cout && ldo % 4 == 0,
             "Cout must be a positive multiple of 16 with ldo >= Cout, ldo % 4 == 0");
  WF_REQUIRE(B * D * H * W < ((int64_t)1 << 31), "too many positions");
  WF_REQUIRE(precision == PREC_BF16 || precision == PREC_SPLIT, "unknown precision");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(w_packed);
  WF_REQUIRE_PTR(out);
  Conv3Args a{};
  a.x = x;
  a.w = w_packed;
  a.bias = bias;
  a.out = out;
  a.ldx = ldx;
  a.ldo = ldo;
  a.B = (int)B; a.D = (int)D; a.H = (int)H; a.W = (int)W;
  a.Cin = (int)Cin;
  a.Cout = (int)Cout;
  a.nch = (int)cdiv(Cin, kConvCC);
  a.wplane = (int64_t)a.nch * kConvKS * Cout * 32;
  hipStream_t s = (hipStream_t)stream;
  const bool co3 = Cout % 48 == 0;
  if (W > 32) return co3 ? launch_conv3<3, 4>(a, precision, s) : launch_conv3<1, 4>(a, precision, s);
  if (W > 16) return co3 ? launch_conv3<3, 2>(a, precision, s) : launch_conv3<1, 2>(a, precision, s);
  return co3 ? launch_conv3<3, 1>(a, precision, s) : launch_conv3<1, 1>(a, precision, s);
}
