// wf_api.hip -- error plumbing and small utilities of the C-ABI (include/waveformer_hip.h).
#include "wf_common.hpp"

namespace wf {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return (int)e;
  }
  return WF_OK;
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ in, uint16_t* __restrict__ out,
                                     int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = f2bf(in[i]);
}

__global__ void split_f32_bf16x2_kernel(const float* __restrict__ in, uint16_t* __restrict__ out,
                                        int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    const float v = in[i];
    const uint16_t hi = f2bf(v);
    out[i] = hi;
    out[n + i] = f2bf(v - bf2f(hi));
  }
}

}  // namespace wf

extern "C" int wf_abi_version(void) { return WF_ABI_VERSION; }

extern "C" const char* wf_last_error(void) { return wf::g_last_error.c_str(); }

extern "C" int wf_cast_f32_to_bf16(const float* in, uint16_t* out, int64_t n, void* stream) {
  WF_REQUIRE(n >= 0, "n < 0");
  if (n == 0) return WF_OK;
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(out);
  int64_t blocks = wf::cdiv(n, 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(wf::cast_f32_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, in, out, n);
  return wf::check_launch("wf_cast_f32_to_bf16");
}

extern "C" int wf_split_f32_to_bf16x2(const float* in, uint16_t* out, int64_t n, void* stream) {
  WF_REQUIRE(n >= 0, "n < 0");
  if (n == 0) return WF_OK;
  WF_REQUIRE_PTR(in);
  WF_REQUIRE_PTR(out);
  int64_t blocks = wf::cdiv(n, 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(wf::split_f32_bf16x2_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, in, out, n);
  return wf::check_launch("wf_split_f32_to_bf16x2");
}
