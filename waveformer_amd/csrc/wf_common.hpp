// wf_common.hpp -- shared device/host helpers for the gfx950 WaveFormer kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/waveformer_hip.h"

namespace wf {

// ---------------------------------------------------------------------------------------
// error reporting (thread-local message, C-ABI returns an int code)
// ---------------------------------------------------------------------------------------
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per kernel and size (not before every
// launch: re-setting it while the same kernel is in flight on another queue is avoided)
void set_max_lds(const void* fn, int bytes);

#define WF_REQUIRE(cond, msg)                                              \
  do {                                                                     \
    if (!(cond)) return ::wf::fail(WF_E_SHAPE, std::string(__func__) + ": " + (msg)); \
  } while (0)
#define WF_REQUIRE_PTR(p)                                                  \
  do {                                                                     \
    if ((p) == nullptr) return ::wf::fail(WF_E_NULLPTR, std::string(__func__) + ": " #p " is NULL"); \
  } while (0)

// ---------------------------------------------------------------------------------------
// vector types
// ---------------------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // round-to-nearest-even, NaN-preserving (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float bf2f(uint16_t u) {
  return __builtin_bit_cast(float, (uint32_t)u << 16);
}

__device__ __forceinline__ float gelu_erf(float x) {
  // nn.GELU() default (approximate='none'): 0.5 x (1 + erf(x / sqrt 2)).  erf(|u|) by
  // Abramowitz & Stegun 7.1.26, 1 - t (a1 + t (a2 + ... a5 t)) e^(-u^2), t = 1 / (1 + p |u|),
  // |error| <= 1.5e-7 -- inside fp32 GELU's own rounding (max |gelu - gelu_fp64| measured
  // 4.6e-7 over [-12, 12], torch's fp32 CPU GELU 1.2e-6).  One v_rcp, one v_exp and ~12
  // FMA-class ops instead of ocml erff's ~40: GELU is the largest VALU cost of CCF_FFN.
  const float u = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, u, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f((x * x) * -0.72134752044448170f);  // e^(-x^2/2)
  const float erfa = fmaf(-p, e, 1.0f);
  const float hx = 0.5f * x;
  return fmaf(hx, copysignf(erfa, x), hx);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
// the register pairs of an f32x4 (f32x2 arithmetic on them compiles to scalar v_*_f32 pairs:
// the build disables packed FP32)
__device__ __forceinline__ f32x2 lo2(f32x4 v) { return __builtin_shufflevector(v, v, 0, 1); }
__device__ __forceinline__ f32x2 hi2(f32x4 v) { return __builtin_shufflevector(v, v, 2, 3); }
// GELU on a pair given HALF its input, hx = x / 2:  GELU(x) = x Phi(x) = hx + |hx| erf(sqrt2 |hx|)
// (no sign restore: x erf(x / sqrt2) = |x| erf(|x| / sqrt2)).  erf by Abramowitz & Stegun 7.1.26
// as in gelu_erf, with the polynomial's coefficients negated so 1 - p e is one FMA, and the
// sqrt2 folded into its constants; the FMA-class steps are f32x2 pair ops.  A caller
// whose input comes out of an affine step (LayerNorm) folds the 1/2 into that step for free.
__device__ __forceinline__ f32x2 gelu_half2(f32x2 hx) {
  const f32x2 a = f32x2{fabsf(hx.x), fabsf(hx.y)};
  const f32x2 d = a * 0.46328425f + 1.0f;                  // 1 + p |x| / sqrt2
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = t * -1.061405429f + 1.453152027f;              // -(a1 t + ... + a5 t^5)
  p = t * p + -1.421413741f;
  p = t * p + 0.284496736f;
  p = t * p + -0.254829592f;
  p = p * t;
  const f32x2 q = (a * a) * -2.88539008177792681f;          // -(x^2 / 2) log2 e
  const f32x2 e = f32x2{__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
  return a * (p * e + 1.0f) + hx;
}
// gelu_erf on a pair
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) { return gelu_half2(x * 0.5f); }

// four / eight lanes' worth as packed pairs
__device__ __forceinline__ f32x4 gelu_half4(f32x4 h) {
  const f32x2 a = gelu_half2(f32x2{h.x, h.y});
  const f32x2 b = gelu_half2(f32x2{h.z, h.w});
  return f32x4{a.x, a.y, b.x, b.y};
}
__device__ __forceinline__ f32x4 gelu_erf4(f32x4 v) {
  const f32x2 a = gelu_erf2(f32x2{v.x, v.y});
  const f32x2 b = gelu_erf2(f32x2{v.z, v.w});
  return f32x4{a.x, a.y, b.x, b.y};
}
__device__ __forceinline__ void gelu_erf8(float* v) {
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const f32x2 r = gelu_erf2(f32x2{v[j], v[j + 1]});
    v[j] = r.x;
    v[j + 1] = r.y;
  }
}

// ---------------------------------------------------------------------------------------
// sub-wave reductions: a "row group" is G consecutive lanes (G a power of two <= 64)
// ---------------------------------------------------------------------------------------
// Butterflies on the VALU's DPP lane crossbar where the partner lies in the same 16-lane row
// (quad_perm xor 1 / xor 2, row_half_mirror, row_mirror -- each leaves every lane of the 2/4/
// 8/16-lane group holding the group total), ds_swizzle (xor 16 inside 32 lanes) and one
// ds_bpermute for the 32-lane halves: no LDS-routed shuffle below 32 lanes.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float swz_xor16(float v) {
  // ds_swizzle bit-mask mode: and 0x1F, or 0, xor 0x10 (within each 32-lane half)
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));
}
template <int G>
__device__ __forceinline__ float group_sum(float v) {
  if (G >= 2) v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  if (G >= 4) v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  if (G >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror
  if (G >= 16) v += dpp_mov<0x140>(v); // row_mirror
  if (G >= 32) v += swz_xor16(v);
  if (G >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}
template <int G>
__device__ __forceinline__ float group_max(float v) {
  if (G >= 2) v = fmaxf(v, dpp_mov<0xB1>(v));
  if (G >= 4) v = fmaxf(v, dpp_mov<0x4E>(v));
  if (G >= 8) v = fmaxf(v, dpp_mov<0x141>(v));
  if (G >= 16) v = fmaxf(v, dpp_mov<0x140>(v));
  if (G >= 32) v = fmaxf(v, swz_xor16(v));
  if (G >= 64) v = fmaxf(v, __shfl_xor(v, 32, 64));
  return v;
}

// v + v[lane ^ 16] and v + v[lane ^ 32] on the VALU lane-swap instructions (round 4): the
// same bits as v + __shfl_xor(v, 16 / 32) (the two addends of a pair are the same values in
// either order), without __shfl_xor's ds_bpermute round trip through the LDS unit on the
// reductions' dependency chains
__device__ __forceinline__ float xsum16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), true, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), true, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace wf
