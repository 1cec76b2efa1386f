// Probe: what __builtin_amdgcn_fdot2_f32_bf16 computes for the split's lo part (p - hi).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/probe_dot2 tools/probe_dot2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef __bf16 bf16v2 __attribute__((ext_vector_type(2)));
__global__ void k(const float* p, float* out, int n) {
  const int i = threadIdx.x;
  const float p0 = p[2 * i], p1 = p[2 * i + 1];
  const bf16v2 h2 = bf16v2{(__bf16)p0, (__bf16)p1};
  const float r0 = __builtin_amdgcn_fdot2_f32_bf16(h2, __builtin_bit_cast(bf16v2, 0x0000BF80u), p0, false);
  const float r1 = __builtin_amdgcn_fdot2_f32_bf16(h2, __builtin_bit_cast(bf16v2, 0xBF800000u), p1, false);
  // the form kernels.hpp split_pair uses: the constants in SGPRs the compiler cannot fold
  uint32_t m0, m1;
  asm("s_mov_b32 %0, 0xbf80" : "=s"(m0));
  asm("s_mov_b32 %0, 0xbf800000" : "=s"(m1));
  const float q0 = __builtin_amdgcn_fdot2_f32_bf16(h2, __builtin_bit_cast(bf16v2, m0), p0, false);
  const float q1 = __builtin_amdgcn_fdot2_f32_bf16(h2, __builtin_bit_cast(bf16v2, m1), p1, false);
  out[4 * i] = q0;
  out[4 * i + 1] = q1;
  out[4 * n + 2 * i] = r0;  // the literal-constant form (hipcc folds (-1, 0) into an inline -1.0)
  out[4 * n + 2 * i + 1] = r1;
  out[4 * i + 2] = p0 - (float)h2.x;
  out[4 * i + 3] = p1 - (float)h2.y;
}
int main() {
  const int n = 64;
  float hp[2 * n], ho[6 * n];
  for (int i = 0; i < 2 * n; ++i) hp[i] = std::ldexp(1.0f + 0.37f * std::sin(1.3f * i), (i % 17) - 8);
  float *dp, *dout;
  hipMalloc(&dp, sizeof hp);
  hipMalloc(&dout, sizeof ho);
  hipMemcpy(dp, hp, sizeof hp, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(n), 0, 0, dp, dout, n);
  hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 2; ++j)
      if (ho[4 * i + j] != ho[4 * i + 2 + j]) {
        if (bad < 8) printf("lane %d elem %d: dot2 %.9g  ref %.9g  (p %.9g)\n", i, j, ho[4 * i + j], ho[4 * i + 2 + j], hp[2 * i + j]);
        ++bad;
      }
  int bad_lit = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 2; ++j) bad_lit += ho[4 * n + 2 * i + j] != ho[4 * i + 2 + j];
  printf("probe_dot2: SGPR-constant form %d of %d mismatches; literal form %d of %d\n", bad, 2 * n,
         bad_lit, 2 * n);
  return bad != 0;
}
