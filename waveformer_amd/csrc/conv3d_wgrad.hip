// conv3d_wgrad.hip -- weight gradient of the 3x3x3 / stride 1 / padding 1 convolution
// (conv3d.hip's forward; the decoder's MONAI Convolution layers in training, config 4:
// monai/networks/blocks/dynunet_block.py:98-111 under 3_train.py's loss.backward()):
//
//   dW[co, ci, tap] = sum_p  g[p, co] * x[p + off(tap), ci]          (zero outside the volume)
//
// an implicit GEMM with the K dimension = output positions (millions), M = Cout, N = Cin per
// tap, on the bf16 MFMA pipes in the fp32-faithful split (hi*hi + hi*lo + lo*hi) -- MIOpen's
// fp32 backward-weights needs a find pass per shape (minutes on a fresh box at B = 4), this
// kernel needs none.
//
// A workgroup owns (48 or 16 output channels) x (16 input channels) x all 27 taps and walks a
// contiguous range of position tiles (one z-plane x 4 rows x 32 columns = 128 positions = 4
// K-steps of 32).  Per tile it stages, split into bf16 hi / lo:
//   * g transposed to [co][position]       -> MFMA operand A (lane: 8 consecutive x of one co;
//     rows padded and swizzled against bank conflicts, see gsw)
//   * the x halo (3 z x 6 y x 34 x) as [ci][z][y][x] -> operand B (8 consecutive x of one ci,
//     at the tap's shifted row; the x shift of 1 or 2 elements is undone in registers: one
//     16-B read + one 4-B read and a funnel shift (v_alignbit) instead of 8 scalar reads).
// Wave w accumulates taps w, w + 4, ... (7 or 6 taps x 3 channel tiles = 84 fp32 VGPRs); the
// next tile's global loads are issued before the current tile's MFMAs.  Each workgroup writes
// its partial dW once (no atomics); a second kernel sums the partials in a fixed order, so the
// result is deterministic.
#include <algorithm>

#include "kernels.hpp"

namespace wf {


constexpr int WG_TX = 32, WG_TY = 4, WG_HX = 34, WG_XR = 40, WG_HY = 6;
constexpr int WG_NPOS = WG_TX * WG_TY;           // 128 positions per tile
constexpr int WG_CI = 16;                        // input channels per workgroup
constexpr int WG_XPOS = 3 * WG_HY * WG_HX;       // 612 halo positions
constexpr int WG_XROWS = 3 * WG_HY;              // 18 halo rows
constexpr int WG_GP = WG_NPOS + 8;               // g tile row pitch in bf16: 272 B (see gsw)
// g tile rows are 272 B apart (16-B chunk offset r mod 16) and chunk 4 s + g4 of row r sits at
// 4 s + (g4 ^ gsw(r)): the A reads of the 16 rows l15 at chunk 4 s + g4 then meet 16 distinct
// 4-bank groups in each of gfx950's ds_read_b128 lane groups ({0-3, 12-15 | g4 0; 20-27 |
// g4 1} and the like: r + (g4 ^ gsw(r)) covers 0..15 once per group), with the K-step s
// still an immediate offset.  256-B rows put 8 lanes of a group on the same banks (SQ: 5.8
// conflict cycles per LDS instruction, profiles/r6/r6q.txt); an XOR of the whole chunk index
// by the row removed them but cost the immediate offsets, spilled and measured 8 % slower
// (profiles/r6/r6r.txt)
__device__ __forceinline__ int gsw(int r) { return ((r + 4) >> 3) & 1; }

struct WgArgs {
  const float* x;   // (B, D, H, W) positions, ldx floats apart, channels [0, Cin)
  const float* g;   // (B, D, H, W) positions, ldg floats apart, channels [0, Cout)
  float* part;      // (nsplit, Cout, Cin * 27) partial sums
  int64_t ldx, ldg;
  int B, D, H, W, Cin, Cout;
  int tiles_x, tiles_y;
  int64_t ntiles;
  int nsplit;
};

template <int CO_T>
__global__ __launch_bounds__(256, 2) void conv3d_wgrad_kernel(WgArgs a) {
  constexpr int NCO = 16 * CO_T;
  constexpr int GQ = NCO / 4;                          // f32x4 per position (g)
  constexpr int GITEMS = (WG_NPOS / 2) * GQ;           // position pairs x channel quads
  constexpr int NG = (GITEMS + 255) / 256;
  constexpr int XITEMS = (WG_XPOS / 2) * (WG_CI / 4);  // halo position pairs x channel quads
  constexpr int NX = (XITEMS + 255) / 256;
  // LDS (bf16 words): g [2 planes][NCO][NPOS], x [2 planes][CI][18 rows][XR]
  __shared__ __attribute__((aligned(16))) uint16_t gs[2 * NCO * WG_GP];
  __shared__ __attribute__((aligned(16))) uint16_t xs[2 * WG_CI * WG_XROWS * WG_XR];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g4 = lane >> 4;
  const int co0 = blockIdx.x * NCO;
  const int ci0 = blockIdx.y * WG_CI;
  const int split = blockIdx.z;
  const int64_t t_begin = (a.ntiles * split) / a.nsplit;
  const int64_t t_end = (a.ntiles * (split + 1)) / a.nsplit;

  f32x4 acc[7][CO_T];
#pragma unroll
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int m = 0; m < CO_T; ++m) acc[i][m] = f32x4{0, 0, 0, 0};

  f32x4 rg[NG][2], rx[NX][2];
  auto fetch = [&](int64_t t) {
    const int tx = (int)(t % a.tiles_x);
    int64_t r = t / a.tiles_x;
    const int ty = (int)(r % a.tiles_y);
    r /= a.tiles_y;
    const int z = (int)(r % a.D);
    const int b = (int)(r / a.D);
    const int x0 = tx * WG_TX, y0 = ty * WG_TY;
    const int64_t sample = (int64_t)b * a.D;
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int i = min(tid + 256 * j, GITEMS - 1);
      const int q = i / (WG_NPOS / 2), pp = i - q * (WG_NPOS / 2);
      const int row = pp / (WG_TX / 2), xx = 2 * (pp - row * (WG_TX / 2));
      const int gy = y0 + row;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int gx = x0 + xx + e;
        f32x4 v = {0, 0, 0, 0};
        if (gy < a.H && gx < a.W)
          v = *reinterpret_cast<const f32x4*>(
              a.g + (((sample + z) * a.H + gy) * a.W + gx) * a.ldg + co0 + 4 * q);
        rg[j][e] = v;
      }
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = min(tid + 256 * j, XITEMS - 1);
      const int q = i / (WG_XPOS / 2), pp = i - q * (WG_XPOS / 2);
      const int hrow = pp / (WG_HX / 2), hx = 2 * (pp - hrow * (WG_HX / 2));
      const int hz = hrow / WG_HY, hy = hrow - hz * WG_HY;
      const int gz = z + hz - 1, gy = y0 + hy - 1;
      const int c = ci0 + 4 * q;
      const bool rowok = gz >= 0 && gz < a.D && gy >= 0 && gy < a.H && c < a.Cin;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int gx = x0 + hx + e - 1;
        f32x4 v = {0, 0, 0, 0};
        if (rowok && gx >= 0 && gx < a.W)
          v = *reinterpret_cast<const f32x4*>(
              a.x + (((sample + gz) * a.H + gy) * a.W + gx) * a.ldx + c);
        rx[j][e] = v;
      }
    }
  };
  // split a pair of positions' 4 channels into (hi, lo) bf16 dwords: word e holds channel e
  // of position 0 (low half) and of position 1 (high half)
  // (the residual x - hi on v_dot2c_f32_bf16: split_pair, kernels.hpp -- the same bits)
  auto pack = [](const f32x4& p0, const f32x4& p1, uint32_t (&hi)[4], uint32_t (&lo)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) split_pair<PREC_SPLIT>(p0[e], p1[e], hi[e], lo[e]);
  };
  auto commit = [&]() {
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int i = tid + 256 * j;
      if (j == NG - 1 && i >= GITEMS) break;
      const int q = i / (WG_NPOS / 2), pp = i - q * (WG_NPOS / 2);
      uint32_t hi[4], lo[4];
      pack(rg[j][0], rg[j][1], hi, lo);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 4 * q + e, c = pp >> 2;  // 16-B chunk c = 4 s + g4 of the row
        uint32_t* d = reinterpret_cast<uint32_t*>(gs + row * WG_GP) +
                      4 * ((c & ~3) | ((c & 3) ^ gsw(row))) + (pp & 3);
        d[0] = hi[e];
        d[NCO * WG_GP / 2] = lo[e];
      }
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = tid + 256 * j;
      if (j == NX - 1 && i >= XITEMS) break;
      const int q = i / (WG_XPOS / 2), pp = i - q * (WG_XPOS / 2);
      const int hrow = pp / (WG_HX / 2), hx2 = pp - hrow * (WG_HX / 2);
      uint32_t hi[4], lo[4];
      pack(rx[j][0], rx[j][1], hi, lo);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uint32_t* d = reinterpret_cast<uint32_t*>(
                          xs + ((4 * q + e) * WG_XROWS + hrow) * WG_XR) + hx2;
        d[0] = hi[e];
        d[WG_CI * WG_XROWS * WG_XR / 2] = lo[e];
      }
    }
  };

  if (t_begin < t_end) fetch(t_begin);
  for (int64_t t = t_begin; t < t_end; ++t) {
    __syncthreads();  // the previous tile's LDS reads are done
    commit();
    __syncthreads();
    if (t + 1 < t_end) fetch(t + 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {  // K-step s = tile row s, lanes g4: x = 8 g4 .. + 7
      bf16x8 ah[CO_T], al[CO_T];
#pragma unroll
      for (int m = 0; m < CO_T; ++m) {
        const uint16_t* p = gs + (16 * m + l15) * WG_GP + 8 * (4 * s + (g4 ^ gsw(l15)));
        ah[m] = *reinterpret_cast<const bf16x8*>(p);
        al[m] = *reinterpret_cast<const bf16x8*>(p + NCO * WG_GP);
      }
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const int tap = wid + 4 * i;
        if (tap >= 27) break;
        const int kz = tap / 9, ky = (tap / 3) % 3, kx = tap % 3;
        const uint16_t* rowp = xs + (l15 * WG_XROWS + kz * WG_HY + s + ky) * WG_XR + 8 * g4;
        bf16x8 bh, bl;
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
          const uint16_t* p = rowp + pl * (WG_CI * WG_XROWS * WG_XR);
          const uint32_t* pd = reinterpret_cast<const uint32_t*>(p);
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 d = *reinterpret_cast<const u32x4*>(pd);
          u32x4 r = d;
          if (kx != 0) {
            const uint32_t d4 = pd[4];
            if (kx == 1) {
              r = u32x4{__builtin_amdgcn_alignbit(d[1], d[0], 16),
                        __builtin_amdgcn_alignbit(d[2], d[1], 16),
                        __builtin_amdgcn_alignbit(d[3], d[2], 16),
                        __builtin_amdgcn_alignbit(d4, d[3], 16)};
            } else {
              r = u32x4{d[1], d[2], d[3], d4};
            }
          }
          if (pl == 0) bh = __builtin_bit_cast(bf16x8, r);
          else bl = __builtin_bit_cast(bf16x8, r);
        }
#pragma unroll
        for (int m = 0; m < CO_T; ++m) {
          acc[i][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[m], bl, acc[i][m], 0, 0, 0);
          acc[i][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[m], bh, acc[i][m], 0, 0, 0);
          acc[i][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[m], bh, acc[i][m], 0, 0, 0);
        }
      }
    }
  }
  // acc[i][m][e] = dW[co0 + 16 m + 4 g4 + e][ci0 + l15][tap wid + 4 i]
  const int ci = ci0 + l15;
  if (ci >= a.Cin) return;
  const int64_t K27 = (int64_t)a.Cin * 27;
  float* pb = a.part + (int64_t)split * a.Cout * K27;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int tap = wid + 4 * i;
    if (tap >= 27) break;
#pragma unroll
    for (int m = 0; m < CO_T; ++m)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        pb[(int64_t)(co0 + 16 * m + 4 * g4 + e) * K27 + (int64_t)ci * 27 + tap] = acc[i][m][e];
  }
}

__global__ void wgrad_reduce_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                    int64_t n, int nsplit, int accumulate) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < nsplit; ++k) s += part[(int64_t)k * n + i];
    dw[i] = accumulate ? dw[i] + s : s;
  }
}

int64_t wgrad_tiles(int64_t B, int64_t D, int64_t H, int64_t W) {
  return B * D * cdiv(H, WG_TY) * cdiv(W, WG_TX);
}

int wgrad_nsplit(int64_t ntiles, int64_t Cin, int64_t Cout) {
  const int64_t wgs = cdiv(Cin, WG_CI) * (Cout % 48 == 0 ? Cout / 48 : Cout / 16);
  // ~2048 workgroups (8 per CU), at least 8 tiles each
  int64_t ns = std::max<int64_t>(1, cdiv(2048, wgs));
  ns = std::min<int64_t>(ns, std::max<int64_t>(1, ntiles / 8));
  return (int)ns;
}

}  // namespace wf

using namespace wf;

extern "C" int64_t wf_conv3d_k3_wgrad_workspace_bytes(int64_t B, int64_t Cin, int64_t Cout,
                                                      int64_t D, int64_t H, int64_t W) {
  const int ns = wgrad_nsplit(wgrad_tiles(B, D, H, W), Cin, Cout);
  return (int64_t)ns * Cout * Cin * 27 * (int64_t)sizeof(float);
}

extern "C" int wf_conv3d_k3_wgrad(const float* x, int64_t ldx, const float* dy, int64_t ldg,
                                  float* dw, int accumulate, void* workspace, int64_t B,
                                  int64_t Cin, int64_t Cout, int64_t D, int64_t H, int64_t W,
                                  void* stream) {
  WF_REQUIRE(B >= 1 && D >= 1 && H >= 1 && W >= 1, "empty tensor");
  WF_REQUIRE(Cin >= 4 && Cin % 4 == 0 && ldx >= Cin && ldx % 4 == 0,
             "Cin must be a positive multiple of 4 with ldx >= Cin, ldx % 4 == 0");
  WF_REQUIRE(Cout >= 16 && Cout % 16 == 0 && ldg >= Cout && ldg % 4 == 0,
             "Cout must be a positive multiple of 16 with ldg >= Cout, ldg % 4 == 0");
  WF_REQUIRE(B * D * H * W < ((int64_t)1 << 31), "input too large");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(dy);
  WF_REQUIRE_PTR(dw);
  WF_REQUIRE_PTR(workspace);
  WgArgs a{};
  a.x = x;
  a.g = dy;
  a.part = reinterpret_cast<float*>(workspace);
  a.ldx = ldx;
  a.ldg = ldg;
  a.B = (int)B; a.D = (int)D; a.H = (int)H; a.W = (int)W;
  a.Cin = (int)Cin;
  a.Cout = (int)Cout;
  a.tiles_x = (int)cdiv(W, WG_TX);
  a.tiles_y = (int)cdiv(H, WG_TY);
  a.ntiles = wgrad_tiles(B, D, H, W);
  a.nsplit = wgrad_nsplit(a.ntiles, Cin, Cout);
  hipStream_t s = (hipStream_t)stream;
  const bool co3 = Cout % 48 == 0;
  const dim3 grid((unsigned)(co3 ? Cout / 48 : Cout / 16), (unsigned)cdiv(Cin, WG_CI),
                  (unsigned)a.nsplit);
  if (co3) hipLaunchKernelGGL(conv3d_wgrad_kernel<3>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(conv3d_wgrad_kernel<1>, grid, dim3(256), 0, s, a);
  int rc = check_launch("wf_conv3d_k3_wgrad");
  if (rc) return rc;
  const int64_t n = Cout * Cin * 27;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 4096)),
                     dim3(256), 0, s, a.part, dw, n, a.nsplit, accumulate);
  return check_launch("wf_conv3d_k3_wgrad (reduce)");
}
