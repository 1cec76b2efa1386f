// ubench_valu.hip -- SIMD issue-rate microbenchmark (diagnostic, not part of the library).
// How many cycles does one SIMD need per wave64 VALU instruction when W waves share it?
// One workgroup per CU (the dynamic LDS request forbids a second), 4*W waves, so W waves per
// SIMD.  Each wave runs N iterations of U independent v_fma_f32 chains (or v_exp_f32, or
// ds_read_b32 + FMAs in the D-wave pattern of ffn_dwfc_sb).  Cycles come from s_memtime around
// the loop (shader clock); per SIMD: cycles / (W * instructions per wave).
//   hipcc --offload-arch=gfx950 -O3 -o gpurun_out/ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

template <int MODE, int U>
__global__ void ub_kernel(float* out, unsigned long long* cyc, int n, float s) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  float a[U];
#pragma unroll
  for (int u = 0; u < U; ++u) a[u] = s * (tid + u);
  for (int i = tid; i < 4096; i += blockDim.x) lds[i] = (float)i * 1e-3f;
  __syncthreads();
  unsigned long long t0;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  if (MODE == 0) {  // independent FMA chains
    for (int it = 0; it < n; ++it) {
#pragma unroll
      for (int u = 0; u < U; ++u) asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(a[u]) : "v"(s));
    }
  } else if (MODE == 1) {  // v_exp_f32 chains
    for (int it = 0; it < n; ++it) {
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] = __builtin_amdgcn_exp2f(a[u]);
    }
  } else if (MODE == 2) {  // D-wave pattern: 3 ds_read_b32 per 18 FMAs (6 FMA per read)
    int base = lane;
    for (int it = 0; it < n; ++it) {
      float v0 = lds[(base) & 4095], v1 = lds[(base + 64) & 4095], v2 = lds[(base + 128) & 4095];
      base += 192;
#pragma unroll
      for (int u = 0; u < U; u += 3) {
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[u]) : "v"(v0), "v"(s));
        if (u + 1 < U) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[u + 1]) : "v"(v1), "v"(s));
        if (u + 2 < U) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[u + 2]) : "v"(v2), "v"(s));
      }
    }
  } else if (MODE == 4) {  // v_fmac_f32 with three VGPR sources (acc += x * w), the scatter's form
    float w[U], x0 = s * lane;
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = s + u * 1e-3f;
    for (int it = 0; it < n; ++it) {
#pragma unroll
      for (int u = 0; u < U; ++u) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[u]) : "v"(x0), "v"(w[u]));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] += w[u];
  } else if (MODE == 3) {  // v_pk_fma_f32 on pairs (compiler packs float2 fma)
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 b[U / 2];
#pragma unroll
    for (int u = 0; u < U / 2; ++u) b[u] = f2{a[2 * u], a[2 * u + 1]};
    const f2 ss = f2{s, s}, hh = f2{0.5f, 0.5f};
    for (int it = 0; it < n; ++it) {
#pragma unroll
      for (int u = 0; u < U / 2; ++u) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(b[u]) : "v"(ss), "v"(hh));
    }
#pragma unroll
    for (int u = 0; u < U / 2; ++u) { a[2 * u] = b[u].x; a[2 * u + 1] = b[u].y; }
  }
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  float r = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) r += a[u];
  out[blockIdx.x * blockDim.x + tid] = r;
  if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + tid / 64] = t1 - t0;
}

template <int MODE, int U>
void run(const char* name, int waves_per_simd, int n, int inst_per_iter) {
  const int nb = 256, nth = 256 * waves_per_simd;
  float* out;
  unsigned long long* cyc;
  CK(hipMalloc(&out, (size_t)nb * nth * 4));
  CK(hipMalloc(&cyc, (size_t)nb * (nth / 64) * 8));
  const size_t lds = 96 * 1024;  // one workgroup per CU
  CK(hipFuncSetAttribute((const void*)ub_kernel<MODE, U>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((ub_kernel<MODE, U>), nb, nth, lds, 0, out, cyc, n, 0.999f);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL((ub_kernel<MODE, U>), nb, nth, lds, 0, out, cyc, n, 0.999f);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h((size_t)nb * (nth / 64));
  CK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
  std::sort(h.begin(), h.end());
  const double med = (double)h[h.size() / 2], mx = (double)h.back();
  const double inst_wave = (double)n * inst_per_iter;
  // per SIMD: W waves each issue inst_wave instructions within ~max wave cycles
  printf("%-10s W=%d U=%2d  wave cycles med %.0f max %.0f | cyc/instr per wave %.2f | per SIMD %.2f | %.3f ms\n",
         name, waves_per_simd, U, med, mx, med / inst_wave, med / inst_wave / waves_per_simd, ms);
  CK(hipFree(out));
  CK(hipFree(cyc));
}

int main() {
  const int n = 4096;
  for (int w = 1; w <= 4; ++w) run<0, 16>("fma", w, n, 16);
  for (int w = 1; w <= 4; ++w) run<0, 4>("fma", w, n, 4);
  for (int w = 1; w <= 4; ++w) run<3, 16>("pk_fma", w, n, 8);
  for (int w = 1; w <= 4; ++w) run<4, 16>("fmac3v", w, n, 16);
  for (int w = 1; w <= 3; ++w) run<1, 8>("exp", w, n / 4, 8);
  for (int w = 1; w <= 3; ++w) run<2, 18>("lds+fma", w, n, 18);
  return 0;
}
