// upsample.hip -- channel-last trilinear resampling for the decoder's ProjectionUpsample
// (network_models/wave_helper.py:33-81: nn.Upsample(scale_factor=stride, mode='trilinear',
// align_corners=True) in front of its depthwise conv and of its 1x1 residual conv).
//
// Index arithmetic is PyTorch's upsample_trilinear3d (area_pixel_compute_scale /
// area_pixel_compute_source_index, fp32): align_corners=True: src = dst * (in-1)/(out-1);
// False: src = max((dst + 0.5) * in/out - 0.5, 0).  i0 = (int)src, i1 = i0 + (i0 < in-1),
// l1 = src - i0, l0 = 1 - l1, combined in PyTorch's order t0 * (h0 * (w0 a + w1 b) + h1 * (..))
// + t1 * (..).  One thread per (output position, 4 channels): the 8 source rows are L2-resident
// (the source is 8-64x smaller than the output), the output is written once (HBM roofline).
#include <algorithm>

#include "wf_common.hpp"

namespace wf {

struct Src1 {
  int i0, i1;
  float l0, l1;
};

// src_index with the axis' scale precomputed (scale = src_scale(in, out, ac), the same fp32
// division): the fused up-sample + conv forms thousands of indices per plane
__device__ __forceinline__ Src1 src_index_s(int dst, int in, float scale, bool ac) {
  Src1 s;
  const float r = ac ? scale * (float)dst : fmaxf(scale * ((float)dst + 0.5f) - 0.5f, 0.f);
  s.i0 = (int)r;
  s.i1 = s.i0 + (s.i0 < in - 1 ? 1 : 0);
  s.l1 = r - (float)s.i0;
  s.l0 = 1.f - s.l1;
  return s;
}

__device__ __forceinline__ Src1 src_index(int dst, int in, int out, bool ac) {
  Src1 s;
  float r;
  if (ac) {
    const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
    r = scale * (float)dst;
  } else {
    const float scale = (float)in / (float)out;
    r = fmaxf(scale * ((float)dst + 0.5f) - 0.5f, 0.f);
  }
  s.i0 = (int)r;
  s.i1 = s.i0 + (s.i0 < in - 1 ? 1 : 0);
  s.l1 = r - (float)s.i0;
  s.l0 = 1.f - s.l1;
  return s;
}

// l0 a + l1 b with the contraction spelled out (one multiply, one FMA): the fused
// up-sample + depthwise conv forms the same values as upsample_cl_lds_kernel bit for bit only if
// both kernels round the blends the same way, whatever the compiler would contract
__device__ __forceinline__ f32x4 blend(float l0, f32x4 a, float l1, f32x4 b) {
  return __builtin_elementwise_fma(f32x4{l1, l1, l1, l1}, b, l0 * a);
}

// one workgroup per output row (b, z, y): the z / y source rows and weights once per
// workgroup, lanes over (x, 4 channels) with one 32-bit division; ADD: out += the resampled
// value (ProjectionUpsample's `y + Up(res)`, wave_helper.py:81, without a separate add pass)
template <bool ADD>
__global__ __launch_bounds__(256) void upsample_cl_kernel(const float* __restrict__ in,
                                                          float* __restrict__ out, int C, int d,
                                                          int h, int w, int D, int H, int W,
                                                          int ac) {
  const int C4 = C >> 2;
  // XCD-contiguous row order (workgroups are dealt round-robin over the 8 XCDs): the
  // neighbouring output rows that read the same source rows run on one XCD and meet in its L2
  const int nb = gridDim.x, xcd = blockIdx.x & 7, q8 = nb >> 3, r8 = nb & 7;
  const int row = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) +
                  (blockIdx.x >> 3);  // (b * D + z) * H + y
  const int y = row % H, bz = row / H;
  const int z = bz % D, b = bz / D;
  const Src1 sz = src_index(z, d, D, ac), sy = src_index(y, h, H, ac);
  const float* base = in + (int64_t)b * ((int64_t)d * h * w * C);
  const float* r00 = base + ((int64_t)sz.i0 * h + sy.i0) * w * C;
  const float* r01 = base + ((int64_t)sz.i0 * h + sy.i1) * w * C;
  const float* r10 = base + ((int64_t)sz.i1 * h + sy.i0) * w * C;
  const float* r11 = base + ((int64_t)sz.i1 * h + sy.i1) * w * C;
  float* orow = out + (int64_t)row * W * C;
  const int n = W * C4;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int x = i / C4;
    const int c = 4 * (i - x * C4);
    const Src1 sx = src_index(x, w, W, ac);
    const int o0 = sx.i0 * C + c, o1 = sx.i1 * C + c;
    auto at = [&](const float* r, int o) { return *reinterpret_cast<const f32x4*>(r + o); };
    const f32x4 v0 = sy.l0 * (sx.l0 * at(r00, o0) + sx.l1 * at(r00, o1)) +
                     sy.l1 * (sx.l0 * at(r01, o0) + sx.l1 * at(r01, o1));
    const f32x4 v1 = sy.l0 * (sx.l0 * at(r10, o0) + sx.l1 * at(r10, o1)) +
                     sy.l1 * (sx.l0 * at(r11, o0) + sx.l1 * at(r11, o1));
    f32x4 v = sz.l0 * v0 + sz.l1 * v1;
    f32x4* op = reinterpret_cast<f32x4*>(orow + (int64_t)x * C + c);
    if (ADD) v = *op + v;
    *op = v;
  }
}

// Predictor.predict_raw_probability (light_training/prediction.py:35-63): every class channel
// of one case's (C, d, h, w) probability volume resampled to the pre-resample shape with
// F.interpolate(mode='trilinear', align_corners=False), stored fp16 (the reference's
// torch.half buffer) or fp32.  Channel-first, one thread per 4 consecutive x outputs: the 8
// source rows of a thread are shared by its x neighbours (L1 / L2), the fp16 output is
// written once, 8 B per thread, coalesced along x.
template <bool F16>
__global__ __launch_bounds__(256) void resample_cf_kernel(const float* __restrict__ in,
                                                          int64_t ldc, void* __restrict__ out,
                                                          int d, int h, int w, int D, int H,
                                                          int W, int64_t total, int ac) {
  const int W4 = (W + 3) >> 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t t = i / W4;
    const int x0 = 4 * (int)(i - t * W4);
    const int y = (int)(t % H);
    t /= H;
    const int z = (int)(t % D);
    const int64_t c = t / D;
    const Src1 sz = src_index(z, d, D, ac), sy = src_index(y, h, H, ac);
    const float* base = in + c * ldc;
    const float* r00 = base + ((int64_t)sz.i0 * h + sy.i0) * w;
    const float* r01 = base + ((int64_t)sz.i0 * h + sy.i1) * w;
    const float* r10 = base + ((int64_t)sz.i1 * h + sy.i0) * w;
    const float* r11 = base + ((int64_t)sz.i1 * h + sy.i1) * w;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int x = min(x0 + e, W - 1);
      const Src1 sx = src_index(x, w, W, ac);
      const float a0 = sy.l0 * (sx.l0 * r00[sx.i0] + sx.l1 * r00[sx.i1]) +
                       sy.l1 * (sx.l0 * r01[sx.i0] + sx.l1 * r01[sx.i1]);
      const float a1 = sy.l0 * (sx.l0 * r10[sx.i0] + sx.l1 * r10[sx.i1]) +
                       sy.l1 * (sx.l0 * r11[sx.i0] + sx.l1 * r11[sx.i1]);
      v[e] = sz.l0 * a0 + sz.l1 * a1;
    }
    const int64_t o = ((c * D + z) * H + y) * (int64_t)W + x0;
    if (F16) {
      _Float16* oh = reinterpret_cast<_Float16*>(out) + o;
      if (x0 + 4 <= W && (o & 3) == 0) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<h4*>(oh) = h4{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2],
                                        (_Float16)v[3]};
      } else {
        for (int e = 0; e < 4 && x0 + e < W; ++e) oh[e] = (_Float16)v[e];
      }
    } else {
      float* of = reinterpret_cast<float*>(out) + o;
      if (x0 + 4 <= W && (o & 3) == 0) {
        *reinterpret_cast<f32x4*>(of) = f32x4{v[0], v[1], v[2], v[3]};
      } else {
        for (int e = 0; e < 4 && x0 + e < W; ++e) of[e] = v[e];
      }
    }
  }
}


// ProjectionUpsample's conv1 (wave_helper.py:33-81, inference): nn.Upsample(trilinear) followed
// by the depthwise 3^3 conv, fused -- the up-sampled tensor (8x / 64x the source) is never
// written nor re-read.  The tiling is dwconv3d_kernel's (ffn.hip): a workgroup = 32 channels
// of one 16 x 8 (x, y) tile of a z segment, 256 threads = 16 columns x 16 channel pairs, the
// haloed 18 x 10 input plane double-buffered in LDS while the z planes stream through.  Each
// input plane is formed from the SOURCE in two LDS steps, in upsample_cl_lds_kernel's
// arithmetic order (so the values are bitwise the up-sampled tensor's): (1) the z blend of the
// tile's <= UD_SY source rows x <= UD_SX source columns (Q: 2 loads per vector, each source
// vector fetched once per plane); (2) per plane position, the y blend of Q's two rows at each
// of the two x neighbours, then the x blend.  Zero padding applies to the up-sampled volume
// (outside it the plane is 0).  Fused epilogue: per-(sample, channel) fp64 sum / sum of
// squares of the outputs (GroupNorm(C, C) statistics, as wf_dwconv3d_stats_cl).
constexpr int UD_CH = 32, UD_TX = 16, UD_TY = 8, UD_SX = 12, UD_SY = 7;

template <bool PF>
__global__ __launch_bounds__(256) void upsample_dwconv3d_kernel(
    const float* __restrict__ in, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ out, double* __restrict__ cstats, int C, int d, int h, int wd, int D,
    int H, int W, int ZS, int ac, float scz, float scy, float scx) {
  constexpr int CH = UD_CH, TX = UD_TX, TY = UD_TY, SX = UD_SX, SY = UD_SY;
  constexpr int PY = TY + 2, PX = TX + 2, NV = CH / 4;
  constexpr int NQ = (SY * SX * NV + 255) / 256;  // Q items per thread
  constexpr int VPI = 2;  // vectors per plane item (measured: 1 -> 2 -13 %, 4 no better)
  constexpr int NP = (PY * PX * NV / VPI + 255) / 256;  // plane items per thread
  __shared__ __attribute__((aligned(16))) float pl[2][PY * PX * CH];
  __shared__ __attribute__((aligned(16))) float Q[SY * SX * CH];

  const int ncc = C / CH, ntx = (W + TX - 1) / TX, nty = (H + TY - 1) / TY;
  const int nzs = (D + ZS - 1) / ZS;
  const int nb = gridDim.x;  // XCD-contiguous tile order, as dwconv3d_kernel
  const int xcd = blockIdx.x & 7, q8 = nb >> 3, r8 = nb & 7;
  int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
  const int cc = t % ncc;
  t /= ncc;
  const int xt = t % ntx;
  t /= ntx;
  const int yt = t % nty;
  t /= nty;
  const int zt = t % nzs;
  const int b = t / nzs;
  const int x0 = xt * TX, y0 = yt * TY, z0 = zt * ZS, z1 = min(z0 + ZS, D);
  const int c0 = cc * CH;
  const int tid = threadIdx.x;
  const int cp = tid % (CH / 2), xi = tid / (CH / 2);
  // the tile's first source column / row (the host checks the spans fit UD_SX / UD_SY)
  const int sxlo = src_index_s(max(x0 - 1, 0), wd, scx, ac).i0;
  const int sylo = src_index_s(max(y0 - 1, 0), h, scy, ac).i0;

  f32x2 w2[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) w2[k] = f32x2{w[(c0 + 2 * cp) * 27 + k], w[(c0 + 2 * cp + 1) * 27 + k]};
  const f32x2 bv = f32x2{bias[c0 + 2 * cp], bias[c0 + 2 * cp + 1]};

  const float* src = in + (int64_t)b * d * h * wd * C + c0;
  // step 1 loads: Q item i -> (source row sr, source column sj, vector v); the two z source
  // planes' vectors (PF: in registers during the previous plane's arithmetic)
  f32x4 ld[NQ][2];
  Src1 szp;
  auto fetch = [&](int p) {
    szp = src_index_s(min(max(p, 0), D - 1), d, scz, ac);
    int ot = tid;
    asm volatile("" : "+v"(ot));
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int i = min(j * 256 + ot, SY * SX * NV - 1);
      const int sr = i / (SX * NV), rem = i - sr * (SX * NV);
      const int sj = rem / NV, v = rem - sj * NV;
      const int ys = min(sylo + sr, h - 1), xs = min(sxlo + sj, wd - 1);
      const float* q = src + ((int64_t)ys * wd + xs) * C + 4 * v;
      ld[j][0] = *reinterpret_cast<const f32x4*>(q + (int64_t)szp.i0 * h * wd * C);
      ld[j][1] = *reinterpret_cast<const f32x4*>(q + (int64_t)szp.i1 * h * wd * C);
    }
  };
  auto commit_q = [&]() {
    int ot = tid;
    asm volatile("" : "+v"(ot));
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int i = j * 256 + ot;
      if (i < SY * SX * NV)
        *reinterpret_cast<f32x4*>(Q + (size_t)i * 4) = blend(szp.l0, ld[j][0], szp.l1, ld[j][1]);
    }
  };
  // step 2: plane position (r, x) of input plane p: y blend of Q's rows at the two x source
  // columns, then the x blend
  auto interp = [&](int buf, int p) {
    const bool pz = p >= 0 && p < D;
    int ot = tid;
    asm volatile("" : "+v"(ot));
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      // item -> (plane position, vectors v + k NV/VPI): one set of indices per VPI vectors
      const int i = j * 256 + ot;
      if (i < PY * PX * NV / VPI) {
        const int pos = i / (NV / VPI), v = i - pos * (NV / VPI);
        const int r = pos / PX, xx = x0 - 1 + pos % PX, yy = y0 - 1 + r;
        const bool ok = pz && yy >= 0 && yy < H && xx >= 0 && xx < W;
        const Src1 sx = src_index_s(min(max(xx, 0), W - 1), wd, scx, ac);
        const Src1 sy = src_index_s(min(max(yy, 0), H - 1), h, scy, ac);
        const int j0 = min(sx.i0 - sxlo, SX - 1), j1 = min(sx.i1 - sxlo, SX - 1);
        const int q0 = min(sy.i0 - sylo, SY - 1), q1 = min(sy.i1 - sylo, SY - 1);
#pragma unroll
        for (int hv = 0; hv < VPI; ++hv) {
          const int vv = v + hv * (NV / VPI);
          auto at = [&](int qr, int jc) {
            return *reinterpret_cast<const f32x4*>(Q + ((qr * SX + jc) * NV + vv) * 4);
          };
          const f32x4 a0 = blend(sy.l0, at(q0, j0), sy.l1, at(q1, j0));
          const f32x4 a1 = blend(sy.l0, at(q0, j1), sy.l1, at(q1, j1));
          const f32x4 val = blend(sx.l0, a0, sx.l1, a1);
          *reinterpret_cast<f32x4*>(pl[buf] + ((size_t)pos * NV + vv) * 4) =
              ok ? val : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  };

  f32x2 accA[TY], accB[TY], accC[TY];
#pragma unroll
  for (int o = 0; o < TY; ++o) accA[o] = accB[o] = accC[o] = f32x2{0.f, 0.f};
  const int xo = x0 + xi;
  double cs0 = 0.0, cs1 = 0.0, cq0 = 0.0, cq1 = 0.0;
  fetch(z0 - 1);
  commit_q();
  __syncthreads();
  interp(0, z0 - 1);
  __syncthreads();
  int buf = 0;
  for (int p = z0 - 1; p <= z1; ++p) {
    // PF: the next plane's source vectors in flight during this plane's arithmetic (24 more
    // registers); otherwise loaded after it
    if (PF) fetch(p + 1);
    const float* P = pl[buf] + xi * CH + 2 * cp;
#pragma unroll
    for (int r = 0; r < PY; ++r) {
      const f32x2 v0 = *reinterpret_cast<const f32x2*>(P + (r * PX + 0) * CH);
      const f32x2 v1 = *reinterpret_cast<const f32x2*>(P + (r * PX + 1) * CH);
      const f32x2 v2 = *reinterpret_cast<const f32x2*>(P + (r * PX + 2) * CH);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int o = r - ky;
        if (o < 0 || o >= TY) continue;
        const f32x2* w0 = w2 + ky * 3;
        accC[o] = w0[2] * v2 + (w0[1] * v1 + (w0[0] * v0 + accC[o]));
        accB[o] = w0[11] * v2 + (w0[10] * v1 + (w0[9] * v0 + accB[o]));
        accA[o] = w0[20] * v2 + (w0[19] * v1 + (w0[18] * v0 + accA[o]));
      }
    }
    const int zo = p - 1;
    if (zo >= z0 && xo < W) {
#pragma unroll
      for (int o = 0; o < TY; ++o) {
        const int yo = y0 + o;
        if (yo < H) {
          const f32x2 r1 = accA[o] + bv;
          const int64_t pos = (((int64_t)b * D + zo) * H + yo) * W + xo;
          *reinterpret_cast<f32x2*>(out + pos * C + c0 + 2 * cp) = r1;
          const double a0 = (double)r1.x, a1 = (double)r1.y;
          cs0 += a0;
          cs1 += a1;
          cq0 += a0 * a0;
          cq1 += a1 * a1;
        }
      }
    }
#pragma unroll
    for (int o = 0; o < TY; ++o) {
      accA[o] = accB[o];
      accB[o] = accC[o];
      accC[o] = f32x2{0.f, 0.f};
    }
    if (!PF) fetch(p + 1);
    commit_q();  // Q's last readers (interp) finished before the previous barrier
    __syncthreads();
    interp(buf ^ 1, p + 1);  // pl[buf ^ 1]'s last readers finished before the previous barrier
    __syncthreads();
    buf ^= 1;
  }
  // the 16 columns of a channel pair, then one fp64 atomic per (channel, moment)
  double* red = reinterpret_cast<double*>(&pl[0][0]);  // [TX][CH / 2][4]
  double* rr = red + (xi * (CH / 2) + cp) * 4;
  rr[0] = cs0;
  rr[1] = cs1;
  rr[2] = cq0;
  rr[3] = cq1;
  __syncthreads();
  if (tid < CH * 2) {
    const int pc = tid >> 2, mom = tid & 3;
    double s = 0.0;
#pragma unroll
    for (int xx = 0; xx < TX; ++xx) s += red[(xx * (CH / 2) + pc) * 4 + mom];
    const int c = c0 + 2 * pc + (mom & 1);
    atomicAdd(cstats + ((int64_t)b * C + c) * 2 + (mom >> 1), s);
  }
}

}  // namespace wf

using namespace wf;

extern "C" int wf_resample_trilinear_cf(const float* in, int64_t ldc, int64_t C, int64_t d,
                                        int64_t h, int64_t w, int64_t D, int64_t H, int64_t W,
                                        int align_corners, void* out, int out_f16,
                                        void* stream) {
  WF_REQUIRE(C >= 1 && d >= 1 && h >= 1 && w >= 1 && D >= 1 && H >= 1 && W >= 1,
             "empty tensor");
  WF_REQUIRE(ldc >= d * h * w, "channel stride smaller than one (d, h, w) volume");
  WF_REQUIRE(C * D * H * W < ((int64_t)1 << 40), "output too large");
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(out);
  const int64_t total = C * D * H * ((W + 3) / 4);
  int64_t blocks = cdiv(total, 256);
  if (blocks > 16384) blocks = 16384;
  auto k = out_f16 ? resample_cf_kernel<true> : resample_cf_kernel<false>;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, in, ldc, out,
                     (int)d, (int)h, (int)w, (int)D, (int)H, (int)W, total, align_corners);
  return check_launch("wf_resample_trilinear_cf");
}

// The same resampling with the z / y interpolation done once per source row: the workgroup
// (one output row) blends its 4 source rows into one (w, C) row in LDS -- each source value
// read once per workgroup instead of 8 gathered 16-B loads per output -- and each output then
// reads its two x neighbours from LDS.  Same arithmetic order as upsample_cl_kernel
// (sy.l0 * (sx...) is not reassociated: z / y first here, y outer of z as the fused
// up-sample + depthwise conv forms it), so results agree to rounding only.
template <bool ADD>
__global__ __launch_bounds__(256) void upsample_cl_lds_kernel(const float* __restrict__ in,
                                                              float* __restrict__ out, int C,
                                                              int d, int h, int w, int D, int H,
                                                              int W, int ac) {
  extern __shared__ __attribute__((aligned(16))) float rowbuf[];  // [w][C]
  const int C4 = C >> 2;
  const int nb = gridDim.x, xcd = blockIdx.x & 7, q8 = nb >> 3, r8 = nb & 7;
  const int row = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) +
                  (blockIdx.x >> 3);  // (b * D + z) * H + y
  const int y = row % H, bz = row / H;
  const int z = bz % D, b = bz / D;
  const Src1 sz = src_index(z, d, D, ac), sy = src_index(y, h, H, ac);
  const float* base = in + (int64_t)b * ((int64_t)d * h * w * C);
  const float* r00 = base + ((int64_t)sz.i0 * h + sy.i0) * w * C;
  const float* r01 = base + ((int64_t)sz.i0 * h + sy.i1) * w * C;
  const float* r10 = base + ((int64_t)sz.i1 * h + sy.i0) * w * C;
  const float* r11 = base + ((int64_t)sz.i1 * h + sy.i1) * w * C;
  const int ns = w * C4;
  for (int i = threadIdx.x; i < ns; i += blockDim.x) {
    const int o = 4 * i;  // (x' * C + c)
    auto at = [&](const float* r) { return *reinterpret_cast<const f32x4*>(r + o); };
    const f32x4 v = blend(sy.l0, blend(sz.l0, at(r00), sz.l1, at(r10)),
                          sy.l1, blend(sz.l0, at(r01), sz.l1, at(r11)));
    *reinterpret_cast<f32x4*>(rowbuf + o) = v;
  }
  __syncthreads();
  float* orow = out + (int64_t)row * W * C;
  const int n = W * C4;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int x = i / C4;
    const int c = 4 * (i - x * C4);
    const Src1 sx = src_index(x, w, W, ac);
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(rowbuf + sx.i0 * C + c);
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(rowbuf + sx.i1 * C + c);
    f32x4 v = blend(sx.l0, a0, sx.l1, a1);
    f32x4* op = reinterpret_cast<f32x4*>(orow + (int64_t)x * C + c);
    if (ADD) v = *op + v;
    *op = v;
  }
}

static int upsample_cl_launch(const float* in, float* out, int64_t B, int64_t C, int64_t d,
                              int64_t h, int64_t w, int64_t D, int64_t H, int64_t W,
                              int align_corners, bool add, void* stream, const char* who) {
  WF_REQUIRE(B >= 1 && d >= 1 && h >= 1 && w >= 1 && D >= 1 && H >= 1 && W >= 1, "empty tensor");
  WF_REQUIRE(C >= 4 && C % 4 == 0, "C must be a positive multiple of 4");
  WF_REQUIRE(B * D * H < ((int64_t)1 << 31) && W * (C / 4) < ((int64_t)1 << 31),
             "output too large");
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(out);
  const size_t lds = (size_t)w * C * sizeof(float);
  static const bool gather = getenv("WF_UPSAMPLE_GATHER") != nullptr;  // A/B: the old kernel
  if (lds <= 64 * 1024 && !gather) {
    auto k = add ? upsample_cl_lds_kernel<true> : upsample_cl_lds_kernel<false>;
    hipLaunchKernelGGL(k, dim3((unsigned)(B * D * H)), dim3(256), lds, (hipStream_t)stream, in,
                       out, (int)C, (int)d, (int)h, (int)w, (int)D, (int)H, (int)W,
                       align_corners);
    return check_launch(who);
  }
  auto k = add ? upsample_cl_kernel<true> : upsample_cl_kernel<false>;
  hipLaunchKernelGGL(k, dim3((unsigned)(B * D * H)), dim3(256), 0, (hipStream_t)stream, in, out,
                     (int)C, (int)d, (int)h, (int)w, (int)D, (int)H, (int)W, align_corners);
  return check_launch(who);
}

extern "C" int wf_upsample_trilinear_cl(const float* in, float* out, int64_t B, int64_t C,
                                        int64_t d, int64_t h, int64_t w, int64_t D, int64_t H,
                                        int64_t W, int align_corners, void* stream) {
  return upsample_cl_launch(in, out, B, C, d, h, w, D, H, W, align_corners, false, stream,
                            "wf_upsample_trilinear_cl");
}

extern "C" int wf_upsample_trilinear_add_cl(const float* in, float* out, int64_t B, int64_t C,
                                            int64_t d, int64_t h, int64_t w, int64_t D,
                                            int64_t H, int64_t W, int align_corners,
                                            void* stream) {
  return upsample_cl_launch(in, out, B, C, d, h, w, D, H, W, align_corners, true, stream,
                            "wf_upsample_trilinear_add_cl");
}

extern "C" int wf_upsample_dwconv3d_stats_cl(const float* in, const float* w, const float* bias,
                                             float* out, double* stats_acc, int64_t B, int64_t C,
                                             int64_t d, int64_t h, int64_t wd, int64_t D,
                                             int64_t H, int64_t W, int align_corners,
                                             void* stream) {
  WF_REQUIRE(B >= 1 && d >= 1 && h >= 1 && wd >= 1 && D >= 1 && H >= 1 && W >= 1, "empty tensor");
  WF_REQUIRE(C % UD_CH == 0 && C >= UD_CH, "channels must be a multiple of 32");
  WF_REQUIRE(B * D * H * W * C < ((int64_t)1 << 40), "output too large");
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(w);
  WF_REQUIRE_PTR(bias);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE_PTR(stats_acc);
  // every tile's source columns / rows (haloed, both blend neighbours) must fit the Q staging
  const bool ac = align_corners != 0;
  auto scale = [&](int64_t n_in, int64_t n_out) -> float {  // src_index's fp32 scale
    if (ac) return n_out > 1 ? (float)(n_in - 1) / (float)(n_out - 1) : 0.f;
    return (float)n_in / (float)n_out;
  };
  auto sidx =[&](int64_t dst, int64_t n_in, float sc) -> Src1 {  // src_index_s on the host
    Src1 s;
    const float r = ac ? sc * (float)dst : std::max(sc * ((float)dst + 0.5f) - 0.5f, 0.f);
    s.i0 = (int)r;
    s.i1 = s.i0 + (s.i0 < n_in - 1 ? 1 : 0);
    return s;
  };
  const float scz = scale(d, D), scy = scale(h, H), scx = scale(wd, W);
  for (int64_t x0 = 0; x0 < W; x0 += UD_TX) {
    const int lo = sidx(std::max<int64_t>(x0 - 1, 0), wd, scx).i0;
    const int hi = sidx(std::min<int64_t>(x0 + UD_TX, W - 1), wd, scx).i1;
    WF_REQUIRE(hi - lo + 1 <= UD_SX, "up-sampling factor along x below 2 (source span > 12)");
  }
  for (int64_t y0 = 0; y0 < H; y0 += UD_TY) {
    const int lo = sidx(std::max<int64_t>(y0 - 1, 0), h, scy).i0;
    const int hi = sidx(std::min<int64_t>(y0 + UD_TY, H - 1), h, scy).i1;
    WF_REQUIRE(hi - lo + 1 <= UD_SY, "up-sampling factor along y below 2 (source span > 7)");
  }
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(stats_acc, 0, (size_t)(B * C * 2) * sizeof(double), s) != hipSuccess)
    return check_launch("wf_upsample_dwconv3d_stats_cl (memset)");
  const int64_t base = B * (C / UD_CH) * cdiv(H, UD_TY) * cdiv(W, UD_TX);
  int64_t ZS = D;  // z segment as launch_dwconv3d
  while (ZS > 8 && base * cdiv(D, ZS) < 2048) ZS = (ZS + 1) / 2;
  const int64_t blocks = base * cdiv(D, ZS);
  WF_REQUIRE(blocks < ((int64_t)1 << 31), "grid too large");
  static const int pf = getenv("WF_UPDW_PF") ? atoi(getenv("WF_UPDW_PF")) : 1;  // A/B
  auto k = pf ? upsample_dwconv3d_kernel<true> : upsample_dwconv3d_kernel<false>;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), 0, s, in, w, bias, out, stats_acc,
                     (int)C, (int)d, (int)h, (int)wd, (int)D, (int)H, (int)W, (int)ZS,
                     align_corners, scz, scy, scx);
  return check_launch("wf_upsample_dwconv3d_stats_cl");
}
