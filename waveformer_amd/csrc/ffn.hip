// ffn.hip -- CCF_FFN with the Block's norm2 + double residual (a7, quirk Q4),
// and PatchMerging (a9, quirk Q3).
//
// CCF_FFN.forward (network_models/wave_helper.py:260-294), for input n (B,D,H,W,C):
//   h1 = GELU(LN_eps1(pwconv(n)))              pwconv = Conv3d(C, 4C, 1) (+bias)    :278-279
//   h2 = GELU(LN_eps2(dwconv(h1)))             dwconv = Conv3d(4C, 4C, 3, pad 1, groups=4C) :285-286
//   return n + fc(h2)                          fc = Linear(4C, C)                    :289-293
// and the Block adds it to attn_fused again: out = x + (n + fc(h2)), n = norm2(x)   :509
// Launches: gemm(pw, LN2 of x in the loader, LN+GELU epilogue) -> dwconv_ln_gelu ->
//           gemm(fc, residual epilogue).  h1/h2 live in the caller's workspace (bf16 for
//           PREC_BF16, fp32 for PREC_SPLIT).
#include "kernels.hpp"

namespace wf {

template <typename T>
struct Store4;
template <>
struct Store4<uint16_t> {  // bf16 storage
  typedef bf16x4 vec;
  static __device__ __forceinline__ f32x4 up(vec u) {
    return f32x4{bf2f((uint16_t)u[0]), bf2f((uint16_t)u[1]), bf2f((uint16_t)u[2]),
                 bf2f((uint16_t)u[3])};
  }
  static __device__ __forceinline__ uint16_t down(float v) { return f2bf(v); }
  static __device__ __forceinline__ vec zero() { return vec{0, 0, 0, 0}; }
};
template <>
struct Store4<float> {  // fp32 storage
  typedef f32x4 vec;
  static __device__ __forceinline__ f32x4 up(vec u) { return u; }
  static __device__ __forceinline__ float down(float v) { return v; }
  static __device__ __forceinline__ vec zero() { return vec{0, 0, 0, 0}; }
};

// Depthwise 3x3x3 conv + bias, then LayerNorm over the Hd channels of each position and
// GELU.  Workgroup = R rows (y) x TW columns (x) of one (b, z) plane, all channels; a thread
// owns 4 channels of one row and slides a 3x3x3 register window along x (9 new loads per
// output).  Outputs are staged in LDS for the per-position LayerNorm.
template <int TW, typename T>
__global__ __launch_bounds__(512) void dwconv_ln_gelu_kernel(
    const T* __restrict__ in, const float* __restrict__ w, const float* __restrict__ bias,
    const float* __restrict__ ln_w, const float* __restrict__ ln_b, float eps,
    T* __restrict__ out, int B, int Hd, int D, int H, int W, int R) {
  typedef Store4<T> S;
  typedef typename S::vec vec;
  extern __shared__ __attribute__((aligned(16))) float rb[];  // [R*TW][Hd+4]
  const int HP = Hd + 4;
  const int nchunk = Hd >> 2;
  const int ntx = (W + TW - 1) / TW, nty = (H + R - 1) / R;
  int t = blockIdx.x;
  const int xt = t % ntx;
  t /= ntx;
  const int yt = t % nty;
  t /= nty;
  const int z = t % D;
  const int b = t / D;
  const int tid = threadIdx.x;
  const int chunk = tid % nchunk, rr = tid / nchunk;
  const int y = yt * R + rr;
  const int xb = xt * TW;
  const bool act = rr < R && y < H;

  if (act) {
    f32x4 wt[27];
#pragma unroll
    for (int k = 0; k < 27; ++k) {
      wt[k].x = w[(4 * chunk + 0) * 27 + k];
      wt[k].y = w[(4 * chunk + 1) * 27 + k];
      wt[k].z = w[(4 * chunk + 2) * 27 + k];
      wt[k].w = w[(4 * chunk + 3) * 27 + k];
    }
    const f32x4 bv = reinterpret_cast<const f32x4*>(bias)[chunk];
    // The 9 (dz, dy) input rows: clamped base pointers + a validity mask.  Loads are always
    // issued (clamped in-bounds addresses) and zeroed by a select afterwards: a branch around
    // each load would make hipcc wait vmcnt(0) per load and serialise the 9-load batch.
    const T* rowp[9];
    unsigned rvalid = 0;
#pragma unroll
    for (int r9 = 0; r9 < 9; ++r9) {
      const int zz = z + r9 / 3 - 1, yy = y + r9 % 3 - 1;
      const bool ok = zz >= 0 && zz < D && yy >= 0 && yy < H;
      rvalid |= (ok ? 1u : 0u) << r9;
      const int zc = min(max(zz, 0), D - 1), yc = min(max(yy, 0), H - 1);
      rowp[r9] = in + (((int64_t)b * D + zc) * H + yc) * (int64_t)W * Hd + 4 * chunk;
    }
    auto ld = [&](int r9, int xx) -> vec {
      const int xc = min(max(xx, 0), W - 1);
      const vec v = *reinterpret_cast<const vec*>(rowp[r9] + (int64_t)xc * Hd);
      const bool ok = ((rvalid >> r9) & 1u) && xx >= 0 && xx < W;
      return ok ? v : S::zero();
    };
    vec win[9][3];
#pragma unroll
    for (int r9 = 0; r9 < 9; ++r9) {
      win[r9][0] = ld(r9, xb - 1);
      win[r9][1] = ld(r9, xb);
    }
#pragma unroll 1
    for (int xi = 0; xi < TW; ++xi) {
      const int x = xb + xi;
#pragma unroll
      for (int r9 = 0; r9 < 9; ++r9) win[r9][2] = ld(r9, x + 1);
      f32x4 acc = bv;
#pragma unroll
      for (int r9 = 0; r9 < 9; ++r9)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) acc += wt[r9 * 3 + dx] * S::up(win[r9][dx]);
      *reinterpret_cast<f32x4*>(rb + (size_t)(rr * TW + xi) * HP + 4 * chunk) = acc;
#pragma unroll
      for (int r9 = 0; r9 < 9; ++r9) {
        win[r9][0] = win[r9][1];
        win[r9][1] = win[r9][2];
      }
    }
  }
  __syncthreads();
  // LayerNorm + GELU per position: one wave per position, lanes over channels
  const int lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
  for (int p = wv; p < R * TW; p += nw) {
    const int yy = yt * R + p / TW, xx = xb + p % TW;
    if (yy >= H || xx >= W) continue;
    const float* row = rb + (size_t)p * HP;
    float s = 0.f;
    for (int e = lane; e < Hd; e += 64) s += row[e];
    const float mean = group_sum<64>(s) / (float)Hd;
    float q = 0.f;
    for (int e = lane; e < Hd; e += 64) {
      const float d = row[e] - mean;
      q += d * d;
    }
    const float rstd = rsqrtf(group_sum<64>(q) / (float)Hd + eps);
    T* dst = out + ((((int64_t)b * D + z) * H + yy) * W + xx) * Hd;
    for (int e = lane; e < Hd; e += 64)
      dst[e] = S::down(gelu_erf((row[e] - mean) * rstd * ln_w[e] + ln_b[e]));
  }
}

template <typename T>
static void launch_dw(int tw, dim3 grid, dim3 block, size_t lds, hipStream_t s, const void* in,
                      const float* w, const float* b, const float* ln_w, const float* ln_b,
                      float eps, void* out, int B, int Hd, int D, int H, int W, int R) {
  const T* i = reinterpret_cast<const T*>(in);
  T* o = reinterpret_cast<T*>(out);
  switch (tw) {
    case 2: hipLaunchKernelGGL((dwconv_ln_gelu_kernel<2, T>), grid, block, lds, s, i, w, b, ln_w, ln_b, eps, o, B, Hd, D, H, W, R); break;
    case 4: hipLaunchKernelGGL((dwconv_ln_gelu_kernel<4, T>), grid, block, lds, s, i, w, b, ln_w, ln_b, eps, o, B, Hd, D, H, W, R); break;
    case 8: hipLaunchKernelGGL((dwconv_ln_gelu_kernel<8, T>), grid, block, lds, s, i, w, b, ln_w, ln_b, eps, o, B, Hd, D, H, W, R); break;
    default: hipLaunchKernelGGL((dwconv_ln_gelu_kernel<16, T>), grid, block, lds, s, i, w, b, ln_w, ln_b, eps, o, B, Hd, D, H, W, R); break;
  }
}

int launch_dwconv_ln_gelu(const void* in, const float* w, const float* b, const float* ln_w,
                          const float* ln_b, float eps, void* out, int B, int Hd, int D, int H,
                          int W, int prec, hipStream_t s) {
  if (Hd % 4 != 0) return fail(WF_E_SHAPE, "dwconv: hidden width must be a multiple of 4");
  const int nchunk = Hd / 4;
  if (nchunk > 512) return fail(WF_E_SHAPE, "dwconv: hidden width > 2048 is not supported");
  int R = 256 / nchunk;
  if (R < 1) R = 1;
  if (R > H) R = H;
  int TW = Hd >= 1536 ? 8 : 16;
  // LDS budget: R * TW * (Hd + 4) floats <= 64 KB
  while (TW > 2 && (size_t)R * TW * (Hd + 4) * 4 > 64 * 1024) TW >>= 1;
  while (R > 1 && (size_t)R * TW * (Hd + 4) * 4 > 64 * 1024) --R;
  const int threads = (int)cdiv((int64_t)nchunk * R, 64) * 64;
  const int tw_eff = TW > W ? W : TW;
  int tw_t = 16;
  if (tw_eff <= 2) tw_t = 2;
  else if (tw_eff <= 4) tw_t = 4;
  else if (tw_eff <= 8) tw_t = 8;
  const size_t lds = (size_t)R * tw_t * (Hd + 4) * 4;
  const int64_t blocks = (int64_t)B * D * cdiv(H, R) * cdiv(W, tw_t);
  if (prec == PREC_SPLIT)
    launch_dw<float>(tw_t, dim3((unsigned)blocks), dim3(threads), lds, s, in, w, b, ln_w, ln_b,
                     eps, out, B, Hd, D, H, W, R);
  else
    launch_dw<uint16_t>(tw_t, dim3((unsigned)blocks), dim3(threads), lds, s, in, w, b, ln_w,
                        ln_b, eps, out, B, Hd, D, H, W, R);
  return check_launch("dwconv_ln_gelu");
}

}  // namespace wf

using namespace wf;

extern "C" int64_t wf_ccf_ffn_workspace_bytes(int64_t B, int64_t C, int64_t hidden, int64_t D,
                                              int64_t H, int64_t W, int precision) {
  (void)C;
  const int64_t e = precision == PREC_SPLIT ? 4 : 2;
  const int64_t one = ((B * D * H * W * hidden * e) + 255) & ~(int64_t)255;
  return 2 * one;
}

extern "C" int wf_ccf_ffn_fwd(const float* xh, const float* stats, const float* n2_w,
                              const float* n2_b, const uint16_t* pw_bf16x2, const float* pw_b,
                              const float* ln1_w, const float* ln1_b, float eps1,
                              const float* dw_w, const float* dw_b, const float* ln2_w,
                              const float* ln2_b, float eps2, const uint16_t* fc_bf16x2,
                              const float* fc_b, const float* branch_scale, float* out,
                              void* workspace, int64_t B, int64_t C, int64_t hidden, int64_t D,
                              int64_t H, int64_t W, int precision, void* stream) {
  WF_REQUIRE(B >= 1 && D >= 1 && H >= 1 && W >= 1, "empty volume");
  WF_REQUIRE(C % 8 == 0 && hidden % 8 == 0, "C and hidden must be multiples of 8");
  WF_REQUIRE(precision == PREC_BF16 || precision == PREC_SPLIT, "unknown precision");
  WF_REQUIRE_PTR(xh);
  WF_REQUIRE_PTR(pw_bf16x2);
  WF_REQUIRE_PTR(ln1_w);
  WF_REQUIRE_PTR(ln1_b);
  WF_REQUIRE_PTR(dw_w);
  WF_REQUIRE_PTR(dw_b);
  WF_REQUIRE_PTR(ln2_w);
  WF_REQUIRE_PTR(ln2_b);
  WF_REQUIRE_PTR(fc_bf16x2);
  WF_REQUIRE_PTR(out);
  WF_REQUIRE_PTR(workspace);
  if (stats) {
    WF_REQUIRE_PTR(n2_w);
    WF_REQUIRE_PTR(n2_b);
  }
  hipStream_t s = (hipStream_t)stream;
  const int64_t M = B * D * H * W;
  const int64_t e = precision == PREC_SPLIT ? 4 : 2;
  const int64_t one = ((M * hidden * e) + 255) & ~(int64_t)255;
  void* h1 = workspace;
  void* h2 = reinterpret_cast<char*>(workspace) + one;
  const int hbf = precision == PREC_BF16;

  GemmArgs g{};
  g.prec = precision;
  g.a_src = xh;
  g.a_bf16 = 0;
  g.a_C = (int)C;
  g.a_nseg = 1;
  g.a_map = MAP_IDENTITY;
  g.a_ln = stats ? LN_GIVEN : LN_NONE;
  g.a_stats = stats;
  g.a_ln_w = n2_w;
  g.a_ln_b = n2_b;
  g.w = pw_bf16x2;
  g.M = M;
  g.N = (int)hidden;
  g.K = (int)C;
  g.epi = EPI_LN_GELU;
  g.bias = pw_b;
  g.e_ln_w = ln1_w;
  g.e_ln_b = ln1_b;
  g.e_eps = eps1;
  g.out = h1;
  g.out_bf16 = hbf;
  g.ldo = hidden;
  int rc = launch_gemm(g, s, "wf_ccf_ffn_fwd(pwconv)");
  if (rc) return rc;
  rc = launch_dwconv_ln_gelu(h1, dw_w, dw_b, ln2_w, ln2_b, eps2, h2, (int)B, (int)hidden,
                             (int)D, (int)H, (int)W, precision, s);
  if (rc) return rc;
  GemmArgs f{};
  f.prec = precision;
  f.a_src = h2;
  f.a_bf16 = hbf;
  f.a_C = (int)hidden;
  f.a_nseg = 1;
  f.a_map = MAP_IDENTITY;
  f.a_ln = LN_NONE;
  f.w = fc_bf16x2;
  f.M = M;
  f.N = (int)C;
  f.K = (int)hidden;
  f.epi = EPI_RESID;
  f.bias = fc_b;
  f.r_x = xh;
  f.r_stats = stats;
  f.r_ln_w = n2_w;
  f.r_ln_b = n2_b;
  f.r_scale = branch_scale;
  f.rows_per_sample = D * H * W;
  f.out = out;
  f.out_bf16 = 0;
  f.ldo = C;
  return launch_gemm(f, s, "wf_ccf_ffn_fwd(fc)");
}

extern "C" int wf_patch_merging_fwd(const float* x, const float* ln_w, const float* ln_b,
                                    float eps, const uint16_t* red_bf16x2, int v2, float* out,
                                    int64_t B, int64_t C, int64_t D, int64_t H, int64_t W,
                                    int precision, void* stream) {
  WF_REQUIRE(B >= 1 && C % 8 == 0 && C >= 8, "C must be a positive multiple of 8");
  WF_REQUIRE(D % 2 == 0 && H % 2 == 0 && W % 2 == 0 && D >= 2 && H >= 2 && W >= 2,
             "odd sizes (the F.pad branch, wave_helper.py:180-182) are not supported");
  WF_REQUIRE(precision == PREC_BF16 || precision == PREC_SPLIT, "unknown precision");
  WF_REQUIRE_PTR(x);
  WF_REQUIRE_PTR(ln_w);
  WF_REQUIRE_PTR(ln_b);
  WF_REQUIRE_PTR(red_bf16x2);
  WF_REQUIRE_PTR(out);
  GemmArgs g{};
  g.prec = precision;
  g.a_src = x;
  g.a_bf16 = 0;
  g.a_C = (int)C;
  g.a_nseg = 8;
  g.a_map = MAP_MERGE;
  // (d,h,w) offsets of the 8 sub-lattices, one nibble each (bit2 d, bit1 h, bit0 w):
  //   PatchMerging (wave_helper.py:183-190, quirk Q3): 000,100,010,001,101,010,001,111
  //   PatchMergingV2 (itertools.product, :154-156):     000,001,010,011,100,101,110,111
  g.merge_code = v2 ? 0x76543210 : 0x71251240;
  g.mB = (int)B;
  g.mD = (int)D;
  g.mH = (int)H;
  g.mW = (int)W;
  g.a_ln = LN_COMPUTE;
  g.a_ln_w = ln_w;
  g.a_ln_b = ln_b;
  g.a_eps = eps;
  g.w = red_bf16x2;
  g.M = B * (D / 2) * (H / 2) * (W / 2);
  g.N = (int)(2 * C);
  g.K = (int)(8 * C);
  g.epi = EPI_STORE;
  g.bias = nullptr;
  g.out = out;
  g.out_bf16 = 0;
  g.ldo = 2 * C;
  return launch_gemm(g, (hipStream_t)stream, "wf_patch_merging_fwd");
}
