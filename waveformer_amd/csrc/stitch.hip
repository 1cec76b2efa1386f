// stitch.hip -- sliding-window inference: importance map and the gather-form stitch.
//
// Replaces the accumulation half of MONAI's sliding_window_inference as WaveFormer's
// prediction path calls it (SlidingWindowInferer(roi 128^3, sw_batch 2, overlap 0.5,
// 'gaussian'), 4_predict.py:199-205):
//   * compute_importance_map (monai/data/utils.py:1088-1138): separable gaussian
//     exp(x^2 / (-2 sigma^2)) per axis, multiplied out, clamped below at max(min, 1e-3);
//   * the per-window `out[slice] += pred * w` / `count[slice] += w` loop and the final
//     `out /= count` (monai/inferers/utils.py:216-299).
// The scatter of the reference becomes a gather: one thread per output voxel walks the windows
// that cover it in ascending window order, so the fp32 sums are formed in exactly the
// reference's order (product and sum rounded separately, no FMA) with no atomics and one
// write per output element.  The patches may come from an RCCL all-gather of round-robin
// shards (see wf_sliding_window_stitch in include/waveformer_hip.h for the row mapping).
#include <algorithm>

#include "wf_common.hpp"

namespace wf {

constexpr int SW_MAX_WIN = 64;  // windows per axis

struct StitchArgs {
  const float* patches;  // (rows, C, rd, rh, rw)
  const float* map;      // (rd, rh, rw)
  float* out;            // (B, C, D, H, W)
  int B, C, D, H, W;
  int rd, rh, rw;
  int n[3];              // windows per axis (z, y, x)
  int world, sb;         // row mapping of the gathered shards
  int rank;              // PARTIAL: this rank's windows only (g % world == rank), local rows
  int buf;               // the patch rows fit a buffer resource (< 2^31 bytes): batched loads
  uint32_t pbytes;       // their size in bytes
  int starts[3][SW_MAX_WIN];
};

__device__ __forceinline__ void cover(const int* st, int n, int r, int p, int& lo, int& hi) {
  lo = n;
  hi = -1;
  for (int i = 0; i < n; ++i) {
    const int s = st[i];
    if (s <= p && p < s + r) {
      lo = min(lo, i);
      hi = i;
    }
  }
}
// the same, also returning the starts of the first three covering windows (the loop index is
// uniform, so the starts are scalar loads; indexing the kernel-argument table with a per-lane
// window index instead would be a dependent memory load per window)
__device__ __forceinline__ void cover3(const int* st, int n, int r, int p, int& lo, int& hi,
                                       int (&s3)[3]) {
  lo = n;
  hi = -1;
  s3[0] = s3[1] = s3[2] = 0;
  for (int i = 0; i < n; ++i) {
    const int s = st[i];
    if (s <= p && p < s + r) {
      if (hi < 0) lo = i;
      const int k = i - lo;  // covering windows are consecutive (ascending starts)
      if (k == 0) s3[0] = s;
      else if (k == 1) s3[1] = s;
      else if (k == 2) s3[2] = s;
      hi = i;
    }
  }
}

// PARTIAL (the all-reduce exchange, ABI 14): only the windows this rank predicted (g % world
// == rank, local patch row g / world), summed in window order; out is (B, C + 1, D, H, W):
// channels [0, C) the weighted sums, channel C the summed weights -- no division (the ranks'
// partials are all-reduced first, then wf_sliding_window_normalize divides)
// Index arithmetic in 32 bits (the host checks every count fits): the round-5 kernel decoded
// the voxel and mapped each window to its patch row with 64-bit divisions (a software routine
// each), which set its time at 23 % of HBM.  World 1 (one rank) needs no row mapping at all.
// one voxel's covering windows: first / last index and the first three starts per axis
struct StitchPos {
  int z, y, x, z0, y0, x0, z1, y1, x1, gb, R3;
  int sz[3], sy[3], sx[3];
};

// windows (z0 + dz0 + [0, MZ)) x (y0 + [0, MY)) x (x0 + [0, MX)) of one voxel, channels
// [c0, c0 + 4): every load of the batch issued before the first use, then the products added in
// window order (z, y, x) -- product and sum rounded separately, as the reference does.  Absent
// windows / channels load 0 (offset past the buffer resource).
template <int MZ, int MY, int MX>
__device__ __forceinline__ void stitch_batch(const StitchArgs& a, const StitchPos& q, int dz0,
                                             int c0, int nc, bool count, float (&acc)[4],
                                             float& cnt, int mz = 3, int my = 3, int mx = 3) {
#pragma clang fp contract(off)
  constexpr int MB = MZ * MY * MX;
  constexpr uint32_t NONE = 0x80000000u;
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.patches), 0, (int)a.pbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.map), 0, q.R3 * 4, 0x00020000);
  const uint32_t world = (uint32_t)a.world, sb = (uint32_t)a.sb;
  const uint32_t cstride = (uint32_t)q.R3 * 4u;
  uint32_t mo[MB], po[MB];
#pragma unroll
  for (int u = 0; u < MB; ++u) {
    const int dz = dz0 + u / (MY * MX), dy = (u / MX) % MY, dx = u % MX;
    const int iz = q.z0 + dz, iy = q.y0 + dy, ix = q.x0 + dx;
    const int zs = dz == 0 ? q.sz[0] : dz == 1 ? q.sz[1] : q.sz[2];
    const bool ok = iz <= q.z1 && iy <= q.y1 && ix <= q.x1;
    const uint32_t g = (uint32_t)(q.gb + (iz * a.n[1] + iy) * a.n[2] + ix);
    uint32_t row = g;
    if (world != 1) {  // patch row of window g in the gathered shards (see row_of)
      const uint32_t r = g % world, j = g / world;
      row = ((j / sb) * world + r) * sb + (j % sb);
    }
    const uint32_t loc =
        (uint32_t)(((q.z - zs) * a.rh + (q.y - q.sy[dy])) * a.rw + (q.x - q.sx[dx]));
    mo[u] = ok ? loc * 4u : NONE;
    po[u] = ok ? ((row * (uint32_t)a.C + (uint32_t)c0) * (uint32_t)q.R3 + loc) * 4u : NONE;
  }
  float wv[MB], pv[MB][4];
  asm volatile("" ::: "memory");  // one batch in flight at a time (registers: occupancy)
#pragma unroll
  for (int u = 0; u < MB; ++u) {
    // mz / my / mx (wave-uniform): the widest cover of the wave per axis -- slots beyond it
    // are absent for every lane, and their loads are skipped by a scalar branch
    if (u / (MY * MX) >= mz || (u / MX) % MY >= my || u % MX >= mx) {
      wv[u] = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) pv[u][c] = 0.f;
      continue;
    }
    wv[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rm, mo[u], 0, 0));
#pragma unroll
    for (int c = 0; c < 4; ++c)
      pv[u][c] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rp, c < nc ? po[u] + c * cstride : NONE, 0, 0));
  }
#pragma unroll
  for (int u = 0; u < MB; ++u) {
    if (count) cnt = cnt + wv[u];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float prod = pv[u][c] * wv[u];  // rounded on its own (no FMA)
      acc[c] = acc[c] + prod;
    }
  }
}

template <bool PARTIAL>
__global__ __launch_bounds__(256) void stitch_kernel(StitchArgs a) {
  // hipcc contracts a*b+c into an FMA by default (also across the inlined __fmul_rn /
  // __fadd_rn intrinsics); the reference rounds the product and the sum separately, so the
  // arithmetic below uses plain operators under contract(off)
#pragma clang fp contract(off)
  const uint32_t total = (uint32_t)a.B * a.D * a.H * a.W;
  const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
  if (idx >= total) return;
  uint32_t t = idx;
  const int x = (int)(t % (uint32_t)a.W);
  t /= (uint32_t)a.W;
  const int y = (int)(t % (uint32_t)a.H);
  t /= (uint32_t)a.H;
  const int z = (int)(t % (uint32_t)a.D);
  const int b = (int)(t / (uint32_t)a.D);
  int z0, z1, y0, y1, x0, x1, sz[3], sy[3], sx[3];
  cover3(a.starts[0], a.n[0], a.rd, z, z0, z1, sz);
  cover3(a.starts[1], a.n[1], a.rh, y, y0, y1, sy);
  cover3(a.starts[2], a.n[2], a.rw, x, x0, x1, sx);
  const int R3 = a.rd * a.rh * a.rw;
  const int nwin = a.n[0] * a.n[1] * a.n[2];
  const int64_t S = (int64_t)a.D * a.H * a.W;
  const int CO = PARTIAL ? a.C + 1 : a.C;
  float* dst = a.out + (int64_t)b * CO * S + ((int64_t)z * a.H + y) * a.W + x;
  const uint32_t world = (uint32_t)a.world;
  const int gb = b * nwin;
  auto mine = [&](int g) { return !PARTIAL || world == 1 || (uint32_t)g % world == (uint32_t)a.rank; };
  // patch row of global window g (batch-major, then the 'ij' meshgrid order of
  // dense_patch_slices): the gathered shards' order, or the local slot of a partial stitch
  auto row_of = [&](int g) -> int {
    if (world == 1) return g;
    const uint32_t r = (uint32_t)g % world, j = (uint32_t)g / world;
    if (PARTIAL) return (int)j;
    const uint32_t sb = (uint32_t)a.sb;
    return (int)(((j / sb) * world + r) * sb + (j % sb));
  };

  // <= 3 covering windows per axis (overlap <= 0.5, the inferer's default, gives 2, and 3
  // where the last window is shifted back to fit: [112, 128) of a 240-voxel axis lies in the
  // windows at 0, 64 and 112): the covering windows' loads are issued in batches -- all 8 of a
  // 2 x 2 x 2 cover at once, one batch of <= 3 x 3 (y, x) windows per z window otherwise --
  // as buffer loads whose offsets for absent windows and channels fall outside the resource
  // (they return 0; adding the +0 products to sums that start at +0 is exact), and summed in
  // window order.  The generic loops below wait one memory round trip per window, twice.
  if (!PARTIAL && a.buf && z1 - z0 <= 2 && y1 - y0 <= 2 && x1 - x0 <= 2) {
    StitchPos q{z, y, x, z0, y0, x0, z1, y1, x1, gb, R3,
                {sz[0], sz[1], sz[2]}, {sy[0], sy[1], sy[2]}, {sx[0], sx[1], sx[2]}};
    const bool two = z1 - z0 <= 1 && y1 - y0 <= 1 && x1 - x0 <= 1;
    // wave-uniform: does any lane of this path need a second window on the axis
    const int mz = __any(two && z1 > z0) ? 2 : 1, my = __any(two && y1 > y0) ? 2 : 1,
              mx = __any(two && x1 > x0) ? 2 : 1;
    const int ny3 = __any(!two && y1 - y0 >= 2) ? 3 : __any(!two && y1 > y0) ? 2 : 1;
    const int nx3 = __any(!two && x1 - x0 >= 2) ? 3 : __any(!two && x1 > x0) ? 2 : 1;
    float cnt = 0.f;
    for (int c0 = 0; c0 < a.C; c0 += 4) {
      const int nc = min(4, a.C - c0);
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      if (two) {
        // batch shape = the wave's widest cover per axis (z and y are nearly uniform over a
        // wave, which runs along x): absent windows still cost a load instruction each
        stitch_batch<2, 2, 2>(a, q, 0, c0, nc, c0 == 0, acc, cnt, mz, my, mx);
      } else {
#pragma nounroll
        for (int dz = 0; dz <= z1 - z0; ++dz)
          stitch_batch<1, 3, 3>(a, q, dz, c0, nc, c0 == 0, acc, cnt, 1, ny3, nx3);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < nc) dst[(int64_t)(c0 + c) * S] = __fdiv_rn(acc[c], cnt);
    }
    return;
  }

  // count map: sum of the window weights in window order (monai/inferers/utils.py:262-269)
  float cnt = 0.f;
  for (int iz = z0; iz <= z1; ++iz)
    for (int iy = y0; iy <= y1; ++iy)
      for (int ix = x0; ix <= x1; ++ix) {
        if (!mine(gb + (iz * a.n[1] + iy) * a.n[2] + ix)) continue;
        const int loc = ((z - a.starts[0][iz]) * a.rh + (y - a.starts[1][iy])) * a.rw +
                        (x - a.starts[2][ix]);
        cnt = cnt + a.map[loc];
      }
  if (PARTIAL) dst[(int64_t)a.C * S] = cnt;

  for (int c0 = 0; c0 < a.C; c0 += 4) {
    const int nc = min(4, a.C - c0);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int iz = z0; iz <= z1; ++iz)
      for (int iy = y0; iy <= y1; ++iy)
        for (int ix = x0; ix <= x1; ++ix) {
          const int g = gb + (iz * a.n[1] + iy) * a.n[2] + ix;
          if (!mine(g)) continue;
          const int loc = ((z - a.starts[0][iz]) * a.rh + (y - a.starts[1][iy])) * a.rw +
                          (x - a.starts[2][ix]);
          const float w = a.map[loc];
          const float* p = a.patches + ((int64_t)row_of(g) * a.C + c0) * R3 + loc;
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (c < nc) {
              const float prod = p[(int64_t)c * R3] * w;  // rounded on its own (no FMA)
              acc[c] = acc[c] + prod;
            }
        }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < nc) dst[(int64_t)(c0 + c) * S] = PARTIAL ? acc[c] : __fdiv_rn(acc[c], cnt);
  }
}

// out[b][c] = num[b][c] / num[b][C] (the all-reduced partial stitch)
__global__ __launch_bounds__(256) void stitch_normalize_kernel(const float* __restrict__ num,
                                                               float* __restrict__ out, int B,
                                                               int C, int64_t S) {
  const int64_t total = (int64_t)B * C * S;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    const int64_t s = i % S, bc = i / S;
    const int b = (int)(bc / C);
    out[i] = __fdiv_rn(num[((int64_t)b * (C + 1) + (bc - (int64_t)b * C)) * S + s],
                       num[((int64_t)b * (C + 1) + C) * S + s]);
  }
}

__global__ __launch_bounds__(256) void importance_map_kernel(float* out, int rd, int rh, int rw,
                                                             int mode, float sz, float sy,
                                                             float sx) {
  const int64_t total = (int64_t)rd * rh * rw;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  if (mode == 0) {
    out[idx] = 1.f;
    return;
  }
  const int x = (int)(idx % rw), y = (int)((idx / rw) % rh), z = (int)(idx / ((int64_t)rw * rh));
  // x_i = -(n-1)/2 + i; g = exp(x^2 / (-2 sigma^2)) (monai/data/utils.py:1121-1128)
  auto g = [](int i, int n, float s) {
    const float v = -(float)(n - 1) / 2.0f + (float)i;
    return expf(__fdiv_rn(__fmul_rn(v, v), -2.0f * __fmul_rn(s, s)));
  };
  const float m = __fmul_rn(__fmul_rn(g(z, rd, sz), g(y, rh, sy)), g(x, rw, sx));
  // the minimum of the map is the product of the three end-point values (all factors are
  // positive and fp multiplication is monotone); clamp below at max(min, 1e-3) (:1134-1136)
  const float mn = fmaxf(__fmul_rn(__fmul_rn(g(0, rd, sz), g(0, rh, sy)), g(0, rw, sx)), 1e-3f);
  out[idx] = fmaxf(m, mn);
}

// Flip-TTA merge (light_training/prediction.py:123-155): pass p of `pred` was computed on the
// image flipped along the axes of flips[p] (bit 0 = D, 1 = H, 2 = W); it is read back through
// the mirrored index instead of materialising torch.flip copies, summed in pass order and
// divided by the pass count.
constexpr int TTA_MAX_PASSES = 8;
struct TtaArgs {
  const float* pred;  // (P, C, D, H, W)
  float* out;         // (C, D, H, W)
  int P, C, D, H, W;
  int flips[TTA_MAX_PASSES];
};

__global__ __launch_bounds__(256) void tta_merge_kernel(TtaArgs a) {
  const int64_t S = (int64_t)a.D * a.H * a.W;
  const int64_t total = (int64_t)a.C * S;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int x = (int)(idx % a.W);
  const int y = (int)((idx / a.W) % a.H);
  const int z = (int)((idx / ((int64_t)a.W * a.H)) % a.D);
  const int64_t c = idx / S;
  float acc = 0.f;
  for (int p = 0; p < a.P; ++p) {
    const int f = a.flips[p];
    const int zz = (f & 1) ? a.D - 1 - z : z;
    const int yy = (f & 2) ? a.H - 1 - y : y;
    const int xx = (f & 4) ? a.W - 1 - x : x;
    const float v = a.pred[((int64_t)p * a.C + c) * S + ((int64_t)zz * a.H + yy) * a.W + xx];
    acc = p == 0 ? v : __fadd_rn(acc, v);
  }
  a.out[idx] = __fdiv_rn(acc, (float)a.P);
}

}  // namespace wf

using namespace wf;

extern "C" int wf_tta_merge(const float* pred, const int* flips, int npass, float* out,
                            int64_t C, int64_t D, int64_t H, int64_t W, void* stream) {
  WF_REQUIRE_PTR(pred);
  WF_REQUIRE_PTR(flips);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE(npass >= 1 && npass <= TTA_MAX_PASSES, "1..8 passes");
  WF_REQUIRE(C >= 1 && D >= 1 && H >= 1 && W >= 1, "empty volume");
  TtaArgs a{};
  a.pred = pred;
  a.out = out;
  a.P = npass;
  a.C = (int)C;
  a.D = (int)D;
  a.H = (int)H;
  a.W = (int)W;
  for (int p = 0; p < npass; ++p) {
    WF_REQUIRE(flips[p] >= 0 && flips[p] <= 7, "flip mask must be in [0, 7]");
    a.flips[p] = flips[p];
  }
  const int64_t total = C * D * H * W;
  hipLaunchKernelGGL(tta_merge_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, a);
  return check_launch("tta_merge");
}

extern "C" int wf_importance_map(int mode, const float* sigma_scale, float* out, int64_t rd,
                                 int64_t rh, int64_t rw, void* stream) {
  WF_REQUIRE(mode == 0 || mode == 1, "mode must be 0 (constant) or 1 (gaussian)");
  WF_REQUIRE(rd >= 1 && rh >= 1 && rw >= 1, "empty window");
  WF_REQUIRE_PTR(out);
  if (mode == 1) WF_REQUIRE_PTR(sigma_scale);
  const float sz = mode ? sigma_scale[0] * (float)rd : 0.f;
  const float sy = mode ? sigma_scale[1] * (float)rh : 0.f;
  const float sx = mode ? sigma_scale[2] * (float)rw : 0.f;
  if (mode) WF_REQUIRE(sz > 0.f && sy > 0.f && sx > 0.f, "sigma_scale must be positive");
  const int64_t total = rd * rh * rw;
  hipLaunchKernelGGL(importance_map_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, out, (int)rd, (int)rh, (int)rw, mode, sz, sy, sx);
  return check_launch("importance_map");
}

static int stitch_launch(const float* patches, int64_t world, int64_t slots_per_round,
                         int64_t rank, bool partial, const float* importance_map,
                         const int64_t* starts, const int64_t* nwin, float* out, int64_t B,
                         int64_t C, int64_t D, int64_t H, int64_t W, int64_t rd, int64_t rh,
                         int64_t rw, void* stream) {
  WF_REQUIRE_PTR(patches);
  WF_REQUIRE_PTR(importance_map);
  WF_REQUIRE_PTR(starts);
  WF_REQUIRE_PTR(nwin);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE(B >= 1 && C >= 1 && D >= 1 && H >= 1 && W >= 1, "empty output");
  WF_REQUIRE(world >= 1 && slots_per_round >= 1, "world and slots_per_round must be >= 1");
  WF_REQUIRE(rd <= D && rh <= H && rw <= W, "window larger than the (padded) image");
  StitchArgs a{};
  a.patches = patches;
  a.map = importance_map;
  a.out = out;
  a.B = (int)B;
  a.C = (int)C;
  a.D = (int)D;
  a.H = (int)H;
  a.W = (int)W;
  a.rd = (int)rd;
  a.rh = (int)rh;
  a.rw = (int)rw;
  a.world = (int)world;
  a.sb = (int)slots_per_round;
  WF_REQUIRE(rank >= 0 && rank < world, "rank out of range");
  a.rank = (int)rank;
  const int64_t size[3] = {D, H, W}, roi[3] = {rd, rh, rw};
  int64_t off = 0;
  for (int ax = 0; ax < 3; ++ax) {
    WF_REQUIRE(nwin[ax] >= 1 && nwin[ax] <= SW_MAX_WIN, "1..64 windows per axis");
    a.n[ax] = (int)nwin[ax];
    int64_t prev = -1;
    for (int64_t i = 0; i < nwin[ax]; ++i) {
      const int64_t s = starts[off + i];
      WF_REQUIRE(s >= 0 && s + roi[ax] <= size[ax], "window start out of range");
      WF_REQUIRE(s > prev, "window starts must be strictly ascending");
      a.starts[ax][i] = (int)s;
      prev = s;
    }
    // every voxel must be covered (dense_patch_slices guarantees it; a gap would divide by 0)
    WF_REQUIRE(a.starts[ax][0] == 0 && prev + roi[ax] == size[ax], "windows do not span the axis");
    for (int64_t i = 1; i < nwin[ax]; ++i)
      WF_REQUIRE(a.starts[ax][i] <= a.starts[ax][i - 1] + roi[ax], "gap between windows");
    off += nwin[ax];
  }
  const int64_t total = B * D * H * W;
  // the kernel's 32-bit index arithmetic
  WF_REQUIRE(total < ((int64_t)1 << 31) && rd * rh * rw < ((int64_t)1 << 31) &&
                 B * nwin[0] * nwin[1] * nwin[2] < ((int64_t)1 << 31),
             "sliding-window stitch: more than 2^31 voxels or windows");
  {  // the batched loads' 32-bit byte offsets: every patch row the kernel can address
    const int64_t R3 = rd * rh * rw, ng = B * nwin[0] * nwin[1] * nwin[2];
    int64_t rows = 0;
    for (int64_t g = 0; g < ng; ++g) {
      const int64_t r = g % world, j = g / world;
      const int64_t row = world == 1 ? g : ((j / slots_per_round) * world + r) * slots_per_round +
                                               j % slots_per_round;
      rows = std::max(rows, row + 1);
    }
    const int64_t bytes = rows * C * R3 * 4;
    a.buf = !partial && bytes < ((int64_t)1 << 31) && R3 * 16 < ((int64_t)1 << 31);
    a.pbytes = a.buf ? (uint32_t)bytes : 0u;
  }
  if (partial)
    hipLaunchKernelGGL(stitch_kernel<true>, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                       (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(stitch_kernel<false>, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                       (hipStream_t)stream, a);
  return check_launch("sliding_window_stitch");
}

extern "C" int wf_sliding_window_stitch(const float* patches, int64_t world,
                                        int64_t slots_per_round, const float* importance_map,
                                        const int64_t* starts, const int64_t* nwin, float* out,
                                        int64_t B, int64_t C, int64_t D, int64_t H, int64_t W,
                                        int64_t rd, int64_t rh, int64_t rw, void* stream) {
  return stitch_launch(patches, world, slots_per_round, 0, false, importance_map, starts, nwin,
                       out, B, C, D, H, W, rd, rh, rw, stream);
}

extern "C" int wf_sliding_window_stitch_partial(const float* patches, int64_t world,
                                                int64_t rank, const float* importance_map,
                                                const int64_t* starts, const int64_t* nwin,
                                                float* out, int64_t B, int64_t C, int64_t D,
                                                int64_t H, int64_t W, int64_t rd, int64_t rh,
                                                int64_t rw, void* stream) {
  return stitch_launch(patches, world, 1, rank, true, importance_map, starts, nwin, out, B, C, D,
                       H, W, rd, rh, rw, stream);
}

extern "C" int wf_sliding_window_normalize(const float* num, float* out, int64_t B, int64_t C,
                                           int64_t D, int64_t H, int64_t W, void* stream) {
  WF_REQUIRE_PTR(num);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE(B >= 1 && C >= 1 && D >= 1 && H >= 1 && W >= 1, "empty output");
  const int64_t S = D * H * W;
  const int64_t total = B * C * S;
  hipLaunchKernelGGL(stitch_normalize_kernel,
                     dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 65536)), dim3(256), 0,
                     (hipStream_t)stream, num, out, (int)B, (int)C, S);
  return check_launch("sliding_window_normalize");
}
