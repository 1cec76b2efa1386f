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
#include "wf_common.hpp"

namespace wf {

struct Src1 {
  int i0, i1;
  float l0, l1;
};

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
// (sy.l0 * (sx...) is not reassociated: z / y first here), so results agree to rounding only.
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
    const f32x4 v = sz.l0 * (sy.l0 * at(r00) + sy.l1 * at(r01)) +
                    sz.l1 * (sy.l0 * at(r10) + sy.l1 * at(r11));
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
    f32x4 v = sx.l0 * a0 + sx.l1 * a1;
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
