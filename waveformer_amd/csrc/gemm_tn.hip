// gemm_tn.hip -- the weight-gradient GEMM of the training path (config 4, 3_train.py:96-102):
//
//   c[n][k] = sum_m a[m][n] * b[m][k]          (c = a^T b: dW = dY^T X of a Linear / 1x1 conv)
//
// with M = the positions (10^5 .. 10^6 rows), N, K = channels (16 .. 1536).  The platform BLAS
// runs these fp32 "TN" shapes on a handful of workgroups (13-49 for M = 2^20: 1.8-8 ms each,
// 19 % of the round-4 train step); here the M rows are dealt to as many workgroups as fill the
// chip, each writing its partial tile once, and a second kernel sums the partials in a fixed
// order: deterministic, no atomics.
//
// Arithmetic: the fp32-faithful bf16x3 split (kernels.hpp PREC_SPLIT) on v_mfma_f32_16x16x32_bf16
// with fp32 accumulation.  These are leaf gradients (nothing downstream consumes them), so the
// split's 2^-17 product rounding averages over the long reduction instead of being amplified.
//
// Layout of one workgroup (256 threads, 4 waves): a TN x TK = 64 x 64 tile of c over a chunk of
// M.  Per K-step of 32 rows the MFMA operands need 8 consecutive m of one column (operand A:
// lane = (n % 16, m-octet), operand B: lane = (k % 16, m-octet)), i.e. column segments of the
// row-major a / b.  Wave w gathers the m-octet w: lane j loads a[m0 + 8w + i][n0 + j] for
// i < 8 (each load: 64 lanes x 4 B of one row, coalesced), splits the 8 values into bf16 hi / lo
// and writes them as one 16-B LDS word per plane at [n][octet] -- the transpose happens in the
// registers, the LDS image is already in fragment order.  Then wave w runs the MFMAs of column
// tile n = 16 w .. 16 w + 15 against the 4 column tiles of b: 12 MFMAs per K-step.  The next
// step's loads are issued before the current step's MFMAs (two LDS buffers).
#include <algorithm>

#include "kernels.hpp"

namespace wf {

constexpr int TN_T = 64;             // tile columns of a (rows of c)
constexpr int TN_KS = 32;            // m per K-step
constexpr int TN_LD = 48;            // LDS row stride in bf16 (24 dwords: 8 mod 16)
constexpr int TN_PLANE = TN_T * TN_LD;

struct TnArgs {
  const float* a;   // (M, >= N), lda floats apart
  const float* b;   // (M, >= K), ldb floats apart
  float* part;      // (nchunk, N, K)
  int64_t lda, ldb;
  int64_t M;
  int N, K;
  int ntn, ntk;     // column tiles of a / b
  int64_t chunk;    // rows per chunk (multiple of TN_KS)
  int xcd;          // 1-D XCD-contiguous grid (see gemm_tn_kernel)
};

__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(TnArgs g) {
  // [buffer][hi, lo][64 columns][48] for a and for b
  __shared__ __attribute__((aligned(16))) uint16_t as[2 * 2 * TN_PLANE];
  __shared__ __attribute__((aligned(16))) uint16_t bs[2 * 2 * TN_PLANE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g4 = lane >> 4;
  // g.xcd (1-D grid): the ntn x ntk tiles of one m chunk read the same rows of a and b (column
  // slices of them), so they run adjacent on one XCD (XCD-contiguous runs of the linear id)
  // instead of being dealt round-robin over the XCDs' separate L2s
  int bx = blockIdx.x, by = blockIdx.y;
  if (g.xcd) {
    const int nb = gridDim.x, xcd = blockIdx.x & 7, q8 = nb >> 3, r8 = nb & 7;
    const int lb = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
    const int nt = g.ntn * g.ntk;
    bx = lb % nt;
    by = lb / nt;
  }
  const int tn = bx % g.ntn, tk = bx / g.ntn;
  const int n0 = tn * TN_T, k0 = tk * TN_T;
  const int64_t m_begin = (int64_t)by * g.chunk;
  const int64_t m_end = std::min<int64_t>(m_begin + g.chunk, g.M);
  const int nsteps = (int)((m_end - m_begin + TN_KS - 1) / TN_KS);
  // this lane's gather columns (clamped: out-of-range columns load a valid address, zeroed)
  const int na = n0 + lane, kb = k0 + lane;
  const bool va = na < g.N, vb = kb < g.K;
  const float* pa = g.a + (va ? na : 0);
  const float* pb = g.b + (vb ? kb : 0);

  float ra[8], rb[8];
  auto fetch = [&](int s) {
    const int64_t m = m_begin + (int64_t)s * TN_KS + 8 * wid;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t mm = std::min<int64_t>(m + i, g.M - 1);
      ra[i] = pa[mm * g.lda];
      rb[i] = pb[mm * g.ldb];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool mv = m + i < m_end;
      ra[i] = (mv && va) ? ra[i] : 0.f;
      rb[i] = (mv && vb) ? rb[i] : 0.f;
    }
  };
  auto commit = [&](int buf) {
    bf16x8 ah, al, bh, bl;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint16_t h = f2bf(ra[i]);
      ah[i] = (short)h;
      al[i] = (short)f2bf(ra[i] - bf2f(h));
      const uint16_t hb = f2bf(rb[i]);
      bh[i] = (short)hb;
      bl[i] = (short)f2bf(rb[i] - bf2f(hb));
    }
    uint16_t* ab = as + buf * 2 * TN_PLANE + lane * TN_LD + 8 * wid;
    uint16_t* bb = bs + buf * 2 * TN_PLANE + lane * TN_LD + 8 * wid;
    *reinterpret_cast<bf16x8*>(ab) = ah;
    *reinterpret_cast<bf16x8*>(ab + TN_PLANE) = al;
    *reinterpret_cast<bf16x8*>(bb) = bh;
    *reinterpret_cast<bf16x8*>(bb + TN_PLANE) = bl;
  };

  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nsteps > 0) {
    fetch(0);
    commit(0);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) fetch(s + 1);  // in flight across this step's MFMAs
    const uint16_t* ab = as + buf * 2 * TN_PLANE + (16 * wid + l15) * TN_LD + 8 * g4;
    const bf16x8 a_hi = *reinterpret_cast<const bf16x8*>(ab);
    const bf16x8 a_lo = *reinterpret_cast<const bf16x8*>(ab + TN_PLANE);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint16_t* bb = bs + buf * 2 * TN_PLANE + (16 * t + l15) * TN_LD + 8 * g4;
      const bf16x8 b_hi = *reinterpret_cast<const bf16x8*>(bb);
      const bf16x8 b_lo = *reinterpret_cast<const bf16x8*>(bb + TN_PLANE);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_hi, b_lo, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_lo, b_hi, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_hi, b_hi, acc[t], 0, 0, 0);
    }
    if (s + 1 < nsteps) commit(buf ^ 1);  // the other buffer: last read two steps ago
    __syncthreads();
  }
  // acc[t][i] = c[n0 + 16 wid + 4 g4 + i][k0 + 16 t + l15]  (MFMA 16x16 output layout:
  // lane holds rows 4 g4 .. 4 g4 + 3 of column l15)
  float* pc = g.part + (int64_t)by * g.N * g.K;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int k = k0 + 16 * t + l15;
    if (k >= g.K) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + 16 * wid + 4 * g4 + i;
      if (n < g.N) pc[(int64_t)n * g.K + k] = acc[t][i];
    }
  }
}

// c[n][k] (ldc apart, + c when accumulate) = sum over the chunks in index order
__global__ __launch_bounds__(256) void gemm_tn_reduce_kernel(const float* __restrict__ part,
                                                             float* __restrict__ c, int64_t ldc,
                                                             int N, int K, int nchunk,
                                                             int accumulate) {
  const int64_t n_el = (int64_t)N * K;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_el;
       i += (int64_t)gridDim.x * blockDim.x) {
    float s = part[i];
    for (int j = 1; j < nchunk; ++j) s += part[(int64_t)j * n_el + i];
    const int64_t n = i / K, k = i - n * K;
    float* dst = c + n * ldc + k;
    *dst = accumulate ? *dst + s : s;
  }
}

namespace {
// rows per chunk: enough workgroups to cover the CUs a few times, chunks of >= 8 K-steps
int64_t tn_chunk(int64_t M, int tiles) {
  const int64_t target = std::max<int64_t>(1, 1024 / tiles);
  int64_t chunk = cdiv(M, target);
  chunk = std::max<int64_t>(chunk, 8 * TN_KS);
  return cdiv(chunk, TN_KS) * TN_KS;
}
}  // namespace

}  // namespace wf

using namespace wf;

extern "C" int64_t wf_gemm_tn_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  if (M < 1 || N < 1 || K < 1) return 0;
  const int tiles = (int)(cdiv(N, TN_T) * cdiv(K, TN_T));
  return cdiv(M, tn_chunk(M, tiles)) * N * K * (int64_t)sizeof(float);
}

extern "C" int wf_gemm_tn(const float* a, int64_t lda, const float* b, int64_t ldb, float* c,
                          int64_t ldc, int accumulate, void* workspace, int64_t M, int64_t N,
                          int64_t K, void* stream) {
  WF_REQUIRE(M >= 1 && N >= 1 && K >= 1, "empty GEMM");
  WF_REQUIRE(lda >= N && ldb >= K && ldc >= K, "leading dimensions too small");
  WF_REQUIRE(N <= 65536 && K <= 65536 && M < ((int64_t)1 << 40), "shape too large");
  WF_REQUIRE_PTR(a);
  WF_REQUIRE_PTR(b);
  WF_REQUIRE_PTR(c);
  WF_REQUIRE_PTR(workspace);
  TnArgs g{};
  g.a = a;
  g.b = b;
  g.part = static_cast<float*>(workspace);
  g.lda = lda;
  g.ldb = ldb;
  g.M = M;
  g.N = (int)N;
  g.K = (int)K;
  g.ntn = (int)cdiv(N, TN_T);
  g.ntk = (int)cdiv(K, TN_T);
  g.chunk = tn_chunk(M, g.ntn * g.ntk);
  const int64_t nchunk = cdiv(M, g.chunk);
  WF_REQUIRE(nchunk <= 65535 && (int64_t)g.ntn * g.ntk < ((int64_t)1 << 31), "grid too large");
  hipStream_t s = (hipStream_t)stream;
  static const bool xcd = !getenv("WF_TN_XCD") || getenv("WF_TN_XCD")[0] != '0';
  g.xcd = xcd && g.ntn * g.ntk * nchunk < ((int64_t)1 << 31);
  if (g.xcd)
    hipLaunchKernelGGL(gemm_tn_kernel, dim3((unsigned)(g.ntn * g.ntk * nchunk)), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL(gemm_tn_kernel, dim3((unsigned)(g.ntn * g.ntk), (unsigned)nchunk),
                       dim3(256), 0, s, g);
  int rc = check_launch("wf_gemm_tn");
  if (rc) return rc;
  const int64_t n_el = N * K;
  hipLaunchKernelGGL(gemm_tn_reduce_kernel,
                     dim3((unsigned)std::min<int64_t>(cdiv(n_el, 256), 4096)), dim3(256), 0, s,
                     g.part, c, ldc, (int)N, (int)K, (int)nchunk, accumulate);
  return check_launch("wf_gemm_tn (reduce)");
}
