// hfref.hip -- HFRefinementRes (idwt_upsample.py:12-50) over the 7 detail tensors of one
// wavelet level, the config-5 branch the decoder applies before the IDWT (:153-156):
//
//     out = x * sigmoid( conv1x1( relu( IN_affine( dwconv3^3(x) + b1 ) ) ) + b2 )
//
// in two streaming passes over channel-last (B, D, H, W, C) fp32 tensors, nothing written in
// between:
//   hf_stats_kernel  depthwise 3^3 conv (zero padding) of each detail tensor, marching down
//                    whole z columns with a 3-plane rolling accumulator (each input plane is
//                    read once per column: 9 neighbour loads, L1/L2-resident), and the
//                    InstanceNorm moments per (detail, sample, channel): fp32 per thread,
//                    fp64 per workgroup, one fp64 atomic per channel and workgroup.
//   hf_apply_kernel  recomputes the conv for a tile of NPOS (y, x) positions x 8 planes,
//                    normalises (mean / rstd from the moments, affine), ReLU -> LDS as
//                    [channel][voxel]; then the C x C 1x1 conv in fp32 FMAs (each thread: 8
//                    voxels x 4 output channels, weights streamed from L1 once per 4 input
//                    channels), bias, sigmoid, times x, one store.
// The 1x1 conv is 2 C^2 flops per voxel (<= 74 KFLOP at C = 192), small against the HBM
// time of the three tensor passes (read x twice, write out once), so it stays exact fp32 on
// the VALU: the branch is HBM-bound.  Thread mapping in both kernels: tid -> (position, 4-
// channel group), NPOS = 256 / (C / 4) positions per workgroup.
#include "kernels.hpp"

namespace wf {


constexpr int HF_ZS = 8;  // planes per apply tile

struct HfArgs {
  const float* x[7];  // detail tensors, channel-last, batch stride ldb
  int64_t ldb;
  float* out;         // (7, B, D, H, W, C)
  const float* dw_w;  // (C, 27)
  const float* dw_b;  // (C)
  const float* in_w;  // InstanceNorm affine weight / bias (C)
  const float* in_b;
  const float* pw_w;  // (C, C) [co][ci]
  const float* pw_b;  // (C)
  double* acc;        // (7, B, C, 2) {sum, sum of squares}
  int B, C, D, H, W;
  int npos, tiles_xy;
  float eps;
  int sigmoid;
};

// the 27 taps of channels [4 cg, 4 cg + 4) from a [27][C] LDS copy of the weights
__device__ __forceinline__ void load_taps(const float* wl, int C, int cg, f32x4 (&w)[27]) {
#pragma unroll
  for (int t = 0; t < 27; ++t) w[t] = *reinterpret_cast<const f32x4*>(wl + t * C + 4 * cg);
}

// stage the (C, 27) depthwise weights transposed to [27][C] in LDS
__device__ __forceinline__ void stage_taps(const float* __restrict__ w, float* wl, int C) {
  for (int i = threadIdx.x; i < 27 * C; i += blockDim.x) {
    const int c = i / 27, t = i - c * 27;
    wl[t * C + c] = w[i];
  }
}

// the 3 x 3 in-plane neighbourhood of (z, y, x), channels [4 cg, +4), zero outside
__device__ __forceinline__ void load_plane(const float* __restrict__ xb, int z, int y, int x,
                                           int cg, const HfArgs& a, f32x4 (&v)[9]) {
  const bool zin = z >= 0 && z < a.D;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int yy = y + dy - 1, xx = x + dx - 1;
      const bool in = zin && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
      f32x4 t = {0.f, 0.f, 0.f, 0.f};
      if (in)
        t = *reinterpret_cast<const f32x4*>(
            xb + (((int64_t)z * a.H + yy) * a.W + xx) * a.C + 4 * cg);
      v[dy * 3 + dx] = t;
    }
}

// acc += sum over the 9 in-plane taps of depth kz
__device__ __forceinline__ f32x4 taps9(const f32x4 (&v)[9], const f32x4 (&w)[27], int kz,
                                       f32x4 acc) {
#pragma unroll
  for (int i = 0; i < 9; ++i) acc += v[i] * w[kz * 9 + i];
  return acc;
}

__global__ __launch_bounds__(256) void hf_stats_kernel(HfArgs a) {
  __shared__ float wl[27 * 256];
  __shared__ float red[2 * 256 * 4];  // [moment][thread][4]
  const int C = a.C, C4 = C >> 2;
  const int tid = threadIdx.x;
  const int pi = tid / C4, cg = tid - pi * C4;
  const int kb = blockIdx.y;  // detail * B + b
  const int k = kb / a.B, b = kb - k * a.B;
  const int p = blockIdx.x * a.npos + pi;
  const bool act = pi < a.npos && p < a.H * a.W;
  stage_taps(a.dw_w, wl, C);
  __syncthreads();
  f32x4 s = {0.f, 0.f, 0.f, 0.f}, q = {0.f, 0.f, 0.f, 0.f};
  if (act) {
    f32x4 w[27];
    load_taps(wl, C, cg, w);
    const f32x4 bias = *reinterpret_cast<const f32x4*>(a.dw_b + 4 * cg);
    const float* xb = a.x[k] + (int64_t)b * a.ldb;
    const int y = p / a.W, x = p - y * a.W;
    // rolling accumulators: o0 -> plane z - 1, o1 -> z, o2 -> z + 1 while reading plane z
    f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = o0, o2 = o0;
    f32x4 v[9];
    for (int z = 0; z <= a.D; ++z) {
      if (z < a.D) {
        load_plane(xb, z, y, x, cg, a, v);
        o0 = taps9(v, w, 2, o0);
        o1 = taps9(v, w, 1, o1);
        o2 = taps9(v, w, 0, o2);
      }
      if (z >= 1) {  // plane z - 1 is complete
        const f32x4 yv = o0 + bias;
        s += yv;
        q += yv * yv;
      }
      o0 = o1;
      o1 = o2;
      o2 = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  *reinterpret_cast<f32x4*>(red + tid * 4) = s;
  *reinterpret_cast<f32x4*>(red + (256 + tid) * 4) = q;
  __syncthreads();
  for (int i = tid; i < 2 * C; i += blockDim.x) {
    const int c = i >> 1, mom = i & 1;
    const int g = c >> 2, j = c & 3;
    double t = 0;
    for (int r = 0; r < a.npos; ++r) t += (double)red[(mom * 256 + r * C4 + g) * 4 + j];
    atomicAdd(a.acc + ((int64_t)kb * C + c) * 2 + mom, t);
  }
}

__global__ __launch_bounds__(256) void hf_apply_kernel(HfArgs a) {
  extern __shared__ float sm[];
  const int C = a.C, C4 = C >> 2;
  const int NV = a.npos * HF_ZS;
  float* wl = sm;                    // [27][C]
  float* nsc = wl + 27 * C;          // [C] scale
  float* nsh = nsc + C;              // [C] shift
  float* zt = nsh + C;               // [C][NV] normalised, activated conv output
  const int tid = threadIdx.x;
  const int pi = tid / C4, cg = tid - pi * C4;
  const int kb = blockIdx.y;
  const int k = kb / a.B, b = kb - k * a.B;
  const int zseg = blockIdx.x / a.tiles_xy;
  const int tile = blockIdx.x - zseg * a.tiles_xy;
  const int z0 = zseg * HF_ZS;
  const int p = tile * a.npos + pi;
  const int64_t P = (int64_t)a.D * a.H * a.W;
  const bool act = pi < a.npos && p < a.H * a.W;
  stage_taps(a.dw_w, wl, C);
  for (int c = tid; c < C; c += blockDim.x) {
    const double* m = a.acc + ((int64_t)kb * C + c) * 2;
    const double mean = m[0] / (double)P;
    double var = m[1] / (double)P - mean * mean;
    if (var < 0) var = 0;
    const float rstd = (float)(1.0 / sqrt(var + (double)a.eps));
    const float sc = rstd * a.in_w[c];
    nsc[c] = sc;
    nsh[c] = a.in_b[c] - (float)mean * sc;
  }
  __syncthreads();
  const float* xb = a.x[k] + (int64_t)b * a.ldb;
  const int y = act ? p / a.W : 0, x = act ? p - y * a.W : 0;
  if (pi < a.npos) {
    // rolling accumulators as in hf_stats_kernel; each completed plane is normalised,
    // activated and written to zt at once (zero outside the volume / for idle positions)
    f32x4 w[27];
    f32x4 bias = {0.f, 0.f, 0.f, 0.f}, sc = bias, sh = bias;
    if (act) {
      load_taps(wl, C, cg, w);
      bias = *reinterpret_cast<const f32x4*>(a.dw_b + 4 * cg);
      sc = *reinterpret_cast<const f32x4*>(nsc + 4 * cg);
      sh = *reinterpret_cast<const f32x4*>(nsh + 4 * cg);
    }
    f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = o0, o2 = o0;
    f32x4 v[9];
    float* zc = zt + (int64_t)(4 * cg) * NV + pi * HF_ZS;
    for (int i = 0; i < HF_ZS + 2; ++i) {  // input plane z0 - 1 + i
      if (act) {
        load_plane(xb, z0 - 1 + i, y, x, cg, a, v);
        o0 = taps9(v, w, 2, o0);
        o1 = taps9(v, w, 1, o1);
        o2 = taps9(v, w, 0, o2);
      }
      if (i >= 2) {  // output plane j = i - 2 (z0 + j) is complete
        const int j = i - 2;
        f32x4 t = (o0 + bias) * sc + sh;
#pragma unroll
        for (int e = 0; e < 4; ++e) t[e] = fmaxf(t[e], 0.f);
        if (!act || z0 + j >= a.D) t = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) zc[e * NV + j] = t[e];
      }
      o0 = o1;
      o1 = o2;
      o2 = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __syncthreads();
  if (!act) return;
  // 1x1 conv: o[j][e] = sum_ci zt[ci][pi * 8 + j] * W[4 cg + e][ci]
  f32x4 o[HF_ZS];
#pragma unroll
  for (int j = 0; j < HF_ZS; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* wrow = a.pw_w + (int64_t)(4 * cg) * C;
  for (int c0 = 0; c0 < C; c0 += 4) {
    f32x4 wv[4];  // wv[e] = W[4 cg + e][c0 .. c0 + 4)
#pragma unroll
    for (int e = 0; e < 4; ++e) wv[e] = *reinterpret_cast<const f32x4*>(wrow + e * C + c0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float* zr = zt + (int64_t)(c0 + u) * NV + pi * HF_ZS;
      const f32x4 za = *reinterpret_cast<const f32x4*>(zr);
      const f32x4 zb = *reinterpret_cast<const f32x4*>(zr + 4);
      const f32x4 wc = {wv[0][u], wv[1][u], wv[2][u], wv[3][u]};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] += za[j] * wc;
        o[4 + j] += zb[j] * wc;
      }
    }
  }
  const f32x4 pb = *reinterpret_cast<const f32x4*>(a.pw_b + 4 * cg);
  float* ob = a.out + ((int64_t)kb * P) * C;
#pragma unroll
  for (int j = 0; j < HF_ZS; ++j) {
    const int z = z0 + j;
    if (z >= a.D) break;
    const int64_t off = (((int64_t)z * a.H + y) * a.W + x) * C + 4 * cg;
    const f32x4 xv = *reinterpret_cast<const f32x4*>(xb + off);
    f32x4 g = o[j] + pb;
    if (a.sigmoid) {
#pragma unroll
      for (int e = 0; e < 4; ++e) g[e] = 1.f / (1.f + __expf(-g[e]));
    }
    *reinterpret_cast<f32x4*>(ob + off) = xv * g;
  }
}

}  // namespace wf

using namespace wf;

extern "C" int64_t wf_hf_refine_workspace_bytes(int64_t B, int64_t C) {
  return 7 * B * C * 2 * (int64_t)sizeof(double);
}

extern "C" int wf_hf_refine_fwd(const float* const* details, int64_t ldb, const float* dw_w,
                                const float* dw_b, const float* in_w, const float* in_b,
                                float eps, const float* pw_w, const float* pw_b, int sigmoid,
                                float* out, void* workspace, int64_t B, int64_t C, int64_t D,
                                int64_t H, int64_t W, void* stream) {
  WF_REQUIRE(B >= 1 && D >= 1 && H >= 1 && W >= 1, "empty tensor");
  WF_REQUIRE(C >= 4 && C % 4 == 0 && C <= 256, "C must be a multiple of 4 in [4, 256]");
  WF_REQUIRE(ldb >= D * H * W * C, "batch stride smaller than one channel-last sample");
  WF_REQUIRE_PTR(details);
  WF_REQUIRE_PTR(dw_w);
  WF_REQUIRE_PTR(dw_b);
  WF_REQUIRE_PTR(in_w);
  WF_REQUIRE_PTR(in_b);
  WF_REQUIRE_PTR(pw_w);
  WF_REQUIRE_PTR(pw_b);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE_PTR(workspace);
  HfArgs a{};
  for (int i = 0; i < 7; ++i) {
    WF_REQUIRE_PTR(details[i]);
    a.x[i] = details[i];
  }
  a.ldb = ldb;
  a.out = out;
  a.dw_w = dw_w;
  a.dw_b = dw_b;
  a.in_w = in_w;
  a.in_b = in_b;
  a.pw_w = pw_w;
  a.pw_b = pw_b;
  a.acc = reinterpret_cast<double*>(workspace);
  a.B = (int)B;
  a.C = (int)C;
  a.D = (int)D;
  a.H = (int)H;
  a.W = (int)W;
  a.npos = 256 / (int)(C / 4);
  a.tiles_xy = (int)cdiv(H * W, a.npos);
  a.eps = eps;
  a.sigmoid = sigmoid;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(a.acc, 0, (size_t)wf_hf_refine_workspace_bytes(B, C), s) != hipSuccess)
    return check_launch("wf_hf_refine_fwd (memset)");
  hipLaunchKernelGGL(hf_stats_kernel, dim3((unsigned)a.tiles_xy, (unsigned)(7 * B)), dim3(256), 0,
                     s, a);
  int rc = check_launch("wf_hf_refine_fwd (stats)");
  if (rc) return rc;
  const int zsegs = (int)cdiv(D, HF_ZS);
  const size_t lds = (size_t)(27 * C + 2 * C + C * a.npos * HF_ZS) * sizeof(float);
  hipLaunchKernelGGL(hf_apply_kernel, dim3((unsigned)(a.tiles_xy * zsegs), (unsigned)(7 * B)),
                     dim3(256), lds, s, a);
  return check_launch("wf_hf_refine_fwd (apply)");
}
