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
  // nn.GELU() default (approximate='none'): 0.5 x (1 + erf(x / sqrt 2))
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}

// ---------------------------------------------------------------------------------------
// sub-wave reductions: a "row group" is G consecutive lanes (G a power of two <= 64)
// ---------------------------------------------------------------------------------------
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int G>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace wf
