// kernels.hpp -- internal launchers shared by the C-ABI translation units.
#pragma once
#include "wf_common.hpp"

namespace wf {

// Arithmetic of the MFMA operands (see include/waveformer_hip.h, WF_PREC_*):
//   PREC_BF16  -- operands rounded to bf16, fp32 accumulation; intermediates stored bf16.
//   PREC_SPLIT -- "bf16x3": every fp32 operand x is carried as hi = bf16(x) plus
//                 lo = bf16(x - hi); products use hi*hi + lo*hi + hi*lo (the lo*lo term is
//                 below 2^-17 relative), i.e. fp32-faithful results on the bf16 MFMA pipes;
//                 intermediates stay fp32.
//   PREC_FP16  -- operands rounded to fp16 (10-bit mantissa), fp32 accumulation on the
//                 v_mfma_f32_*_f16 pipes; intermediates stay fp32 like PREC_SPLIT (config 5).
enum Prec { PREC_BF16 = 0, PREC_SPLIT = 1, PREC_FP16 = 2 };

// ---- MFMA operand kinds (compile-time twin of Prec): conversion and matrix instruction
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

template <int P>
__device__ __forceinline__ uint16_t op_cvt(float x) {  // the operand (hi part) of x
  if constexpr (P == PREC_FP16) return f2h(x);
  else return f2bf(x);
}
template <int P>
__device__ __forceinline__ short op_lo(float x, uint16_t hi) {  // the split's lo part, else 0
  if constexpr (P == PREC_SPLIT) return (short)f2bf(x - bf2f(hi));
  else return (short)0;
}
template <int P>
__device__ __forceinline__ f32x4 mma32(bf16x8 a, bf16x8 b, f32x4 c) {  // 16x16x32
  if constexpr (P == PREC_FP16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <int P>
__device__ __forceinline__ f32x4 mma16(bf16x4 a, bf16x4 b, f32x4 c) {  // 16x16x16
  if constexpr (P == PREC_FP16)
    return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(f16x4, a),
                                                 __builtin_bit_cast(f16x4, b), c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
// The operand words of a pair of values (first value in the low half): hi = op_cvt, lo = the
// split's lo part (PREC_SPLIT) or 0.  For PREC_SPLIT, y - hi comes from v_dot2c_f32_bf16 of the
// packed hi pair against (-1, 0) / (0, -1) accumulated onto y -- one VALU op per value instead
// of unpacking hi back to fp32 and subtracting; y - hi is exact in fp32, so the words are
// bitwise op_cvt / op_lo's.
// The two constant pairs go through SGPRs the compiler cannot see into: hipcc encodes the
// pair (-1, 0) as the inline constant -1.0, which gfx950 applies to BOTH bf16 halves
// (tools/probe_dot2.hip: p0 - hi0 - hi1 instead of p0 - hi0).
typedef __bf16 bf16v2 __attribute__((ext_vector_type(2)));
template <int P>
__device__ __forceinline__ void split_pair(float y0, float y1, uint32_t& hi, uint32_t& lo) {
  if constexpr (P == PREC_SPLIT) {
    uint32_t m0, m1;
    asm("s_mov_b32 %0, 0xbf80" : "=s"(m0));      // (-1, 0)
    asm("s_mov_b32 %0, 0xbf800000" : "=s"(m1));  // (0, -1)
    const bf16v2 h = bf16v2{(__bf16)y0, (__bf16)y1};  // v_cvt_pk_bf16_f32 (RNE, as f2bf)
    const float r0 = __builtin_amdgcn_fdot2_f32_bf16(h, __builtin_bit_cast(bf16v2, m0), y0, false);
    const float r1 = __builtin_amdgcn_fdot2_f32_bf16(h, __builtin_bit_cast(bf16v2, m1), y1, false);
    hi = __builtin_bit_cast(uint32_t, h);
    lo = __builtin_bit_cast(uint32_t, bf16v2{(__bf16)r0, (__bf16)r1});
  } else {
    hi = (uint32_t)op_cvt<P>(y0) | ((uint32_t)op_cvt<P>(y1) << 16);
    lo = 0;
  }
}
// four values: the hi / lo operand quads (op_cvt / op_lo of each, bitwise)
template <int P>
__device__ __forceinline__ void split4(f32x4 v, bf16x4& h, bf16x4& l) {
  uint32_t h0, h1, l0, l1;
  split_pair<P>(v[0], v[1], h0, l0);
  split_pair<P>(v[2], v[3], h1, l1);
  h = __builtin_bit_cast(bf16x4, u32x2{h0, h1});
  l = __builtin_bit_cast(bf16x4, u32x2{l0, l1});
}
// eight values (an MFMA K-octet): the hi / lo operand octets
template <int P>
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& h, bf16x8& l) {
  uint32_t hw[4], lw[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) split_pair<P>(x[2 * j], x[2 * j + 1], hw[j], lw[j]);
  h = __builtin_bit_cast(bf16x8, u32x4{hw[0], hw[1], hw[2], hw[3]});
  l = __builtin_bit_cast(bf16x8, u32x4{lw[0], lw[1], lw[2], lw[3]});
}
// fp32 storage of the GEMM-to-GEMM intermediates (workspaces): every mode but PREC_BF16
__host__ __device__ constexpr bool store32(int p) { return p != PREC_BF16; }
inline bool valid_prec(int p) { return p == PREC_BF16 || p == PREC_SPLIT || p == PREC_FP16; }

// ---- A-resident MFMA GEMM:  out[m, n] = epilogue( sum_k A[m, k] * Wt[n, k] ) -------------
// A rows are produced by a loader (gather + optional LayerNorm + bf16 rounding) into LDS once
// per workgroup; the weight Wt [2][N][K] (bf16 hi plane, then lo plane) streams from L2.
enum RowMap { MAP_IDENTITY = 0, MAP_WINDOW = 1, MAP_MERGE = 2 };
// LN_PARTIAL: a_stats holds a_np (mean, M2) pairs per row, each over K / a_np consecutive
// columns (written by the producing kernel); the loader combines them (Chan et al.).
enum LnMode { LN_NONE = 0, LN_GIVEN = 1, LN_COMPUTE = 2, LN_PARTIAL = 3 };
// EPI_SUBVOXEL: ConvTranspose3d(k = s = 2) -- row m = position (b, z, y, x) of a (B, d, h, w)
// raster (mB..mW), column s * (N / 8) + c stored + bias at channel c of output position
// (b, 2z + dz, 2y + dy, 2x + dx), s = dz * 4 + dy * 2 + dx, rows ldo floats apart
enum EpiMode { EPI_STORE = 0, EPI_LN_GELU = 1, EPI_RESID = 2, EPI_SUBVOXEL = 3 };

struct GemmArgs {
  int prec;              // Prec
  // ---- A loader
  const void* a_src;     // fp32 or bf16 rows
  int a_bf16;            // 1: a_src is bf16
  int a_C;               // contiguous segment (channels) per source row
  int a_nseg;            // K = a_nseg * a_C
  int a_map;             // RowMap
  int mB, mD, mH, mW, mws;  // geometry of the source raster for MAP_WINDOW / MAP_MERGE
  int merge_code;        // MAP_MERGE: 8 nibbles, sub-lattice s offset (d<<2|h<<1|w) at bits 4s
  int a_ln;              // LnMode
  const float* a_stats;  // LN_GIVEN: (M, 2) {mean, rstd};  LN_PARTIAL: (M, a_np, 2) {mean, M2}
  int a_np;
  const float* a_ln_w;
  const float* a_ln_b;
  float a_eps;
  int a_gelu;            // 1: GELU(erf) on the loaded A values (after the LayerNorm, if any)
  // ---- B
  const uint16_t* w;     // [2][N][K] bf16 (hi plane; lo plane read only for PREC_SPLIT)
  // ---- problem
  int64_t M;
  int N, K;
  // ---- epilogue
  int epi;               // EpiMode
  const float* bias;     // (N) or NULL
  void* out;             // fp32 or bf16 rows of stride ldo
  int out_bf16;
  int64_t ldo;
  const float* e_ln_w;   // EPI_LN_GELU: LN over N (gamma, beta, eps)
  const float* e_ln_b;
  float e_eps;
  const float* r_x;      // EPI_RESID: residual rows (M, N) fp32
  const float* r_stats;  //   if non-NULL also add LN(r_x; r_stats, r_ln_w, r_ln_b)
  const float* r_ln_w;
  const float* r_ln_b;
  const float* r_scale;  //   per-sample factor on the added branch (DropPath) or NULL
  int64_t rows_per_sample; // M / B for r_scale
  int dbg;               // timing experiments only (builds with WF_ROWS_DBG=1): phases skipped
  float* o_pstats;       // EPI_STORE (gemm_kc): if non-NULL, per (row, column chunk) {mean, M2}
                         //   of the stored values, (M, N / chunk, 2) -- LN statistics partials
  float* kpart;          // gemm_kc split-K scratch (caller-owned, kpart_bytes), or NULL: small
  int64_t kpart_bytes;   //   grids split the k loop over grid.z into (ksplit, M, N) fp32
                         //   partials, summed in split order by a second kernel + epilogue
  int ksplit;            // set by the launcher (kernel side), 1 = no split
};

int launch_gemm(const GemmArgs& g, hipStream_t s, const char* who);
// column tiles (of 16) per workgroup gemm_kc would use for g, 0 if it does not take the shape
int gemm_kc_pick_nt(const GemmArgs& g);
// InstanceNorm partial sums (sum, sum of squares per (b, c)) of a channel-last tensor into a
// zeroed (B, C, 2) fp64 accumulator (instnorm.hip)
int launch_instnorm_partial(const float* x, int64_t ldx, int64_t B, int64_t C, int64_t P,
                            double* acc, hipStream_t s);
// streaming variant (gemm_rows.hip); returns 1 if it took the shape, 0 to fall back
int try_launch_gemm_rows(const GemmArgs& g, hipStream_t s, bool single_chunk_only);

// ---- windowed attention core over a (B_, N, 3C) qkv buffer (bf16, or fp32 when SPLIT) ----
// table_ws != 0: `bias` is the (T, heads) relative_position_bias_table and the index is the
// reference's formula for window table_ws (8 with head_dim 16 implemented)
int launch_attn_core(const void* qkv, const float* bias, void* out, float* lse, int64_t Bw,
                     int N, int heads, int hd, float scale, int prec, hipStream_t s,
                     int table_ws = 0);

// ---- depthwise 3^3 conv + bias + LayerNorm + GELU over a channel-last volume ------------
// (bf16 storage for PREC_BF16, fp32 for PREC_SPLIT)
int launch_dwconv_ln_gelu(const void* in, const float* w, const float* b, const float* ln_w,
                          const float* ln_b, float eps, void* out, int B, int Hd, int D, int H,
                          int W, int prec, hipStream_t s);
// ---- depthwise 3^3 conv + bias only (the LayerNorm + GELU run in the next GEMM's loader);
// returns 0 on success, WF_E_SHAPE if the shape is not covered (Hd % 32 != 0)
// pstats (optional): (M, Hd / 32, 2) {mean, M2} of each 32-channel group of every output row
// cstats (optional): zeroed (B, Hd, 2) fp64 {sum, sum of squares} of the outputs per channel
int launch_dwconv3d(const void* in, const float* w, const float* b, void* out, float* pstats,
                    int B, int Hd, int D, int H, int W, int prec, hipStream_t s,
                    double* cstats = nullptr, const float* ln1_stats = nullptr,
                    const float* ln1_w = nullptr, const float* ln1_b = nullptr, int flip = 0);
// per-row {mean, rstd} from np equal-size {mean, M2} partials (Chan et al.), (M, 2)
int launch_ln_stats_finalize(const float* pstats, int np, int group, float eps, float* out,
                             int64_t M, hipStream_t s);
constexpr int DW_STAT_GROUP = 32;
// ---- CCF_FFN back half fused (ffn_dwfc.hip): dwconv + bias + LN2 + GELU + fc + bias + the
// Block's Q4 residual, for C = 48, hidden = 192 (h1 fp32 for PREC_SPLIT, bf16 for PREC_BF16)
struct DwFcArgs {
  const void* h1;        // (B, D, H, W, HID) fp32 (SPLIT) or bf16
  const float* dw_w;     // (HID, 27)
  const float* dw_b;     // (HID)
  const float* ln2_w;    // (HID)
  const float* ln2_b;
  float eps2;
  const uint16_t* fc;    // [2][C][HID] bf16 {hi, lo}
  const float* fc_b;     // (C) or NULL
  const float* x;        // (B, D, H, W, C) residual rows
  const float* stats;    // (M, 2) {mean, rstd} of x for norm2, or NULL
  const float* n2_w;
  const float* n2_b;
  const float* bscale;   // (B) or NULL
  float* out;            // (B, D, H, W, C)
  int B, D, H, W, ZS;
  // whole-FFN kernel (ffn_fused.hip) only: the front half, recomputed on chip from x
  const uint16_t* pw;    // [2][HID][C] bf16 {hi, lo}
  const float* pw_b;     // (HID) or NULL
  const float* ln1_w;    // (HID)
  const float* ln1_b;
  float eps1;
  int dbg;               // timing experiments only (WF_FFN_DBG): bit mask of phases skipped
  int ws_split;          // wave-specialised ffn_dwfc: D rows of a plane in phase 1 (1..5)
};
int launch_ffn_dwfc(const DwFcArgs& a, int prec, hipStream_t s);
// stage-1 shape, three VALU waves per SIMD and one barrier per plane (ffn_dwfc_tb.hip)
int launch_ffn_dwfc_tb(const DwFcArgs& a, int prec, hipStream_t s);
// the same on 4 x 8 tiles with two barriers per plane (ffn_dwfc_tb.hip, WF_FFN_DWFC_TB=4)
int launch_ffn_dwfc_tb4(const DwFcArgs& a, int prec, hipStream_t s);
// h1 plane staging: fp32 (SPLIT / FP16 workspaces) or bf16 (BF16) rows widened to fp32
template <typename T>
struct H1Load;
template <>
struct H1Load<float> {
  typedef f32x4 raw;
  static __device__ __forceinline__ raw load(const float* p, int64_t i) {
    return *reinterpret_cast<const f32x4*>(p + i);
  }
  static __device__ __forceinline__ f32x4 up(raw u) { return u; }
};
template <>
struct H1Load<uint16_t> {
  typedef bf16x4 raw;
  static __device__ __forceinline__ raw load(const uint16_t* p, int64_t i) {
    return *reinterpret_cast<const bf16x4*>(p + i);
  }
  static __device__ __forceinline__ f32x4 up(raw u) {
    return f32x4{bf2f((uint16_t)u[0]), bf2f((uint16_t)u[1]), bf2f((uint16_t)u[2]),
                 bf2f((uint16_t)u[3])};
  }
};

// the same for C = 96, hidden = 384 (4 x 4 tiles, one plane buffer, fc weight hi in LDS)
int launch_ffn_dwfc2(const DwFcArgs& a, int prec, hipStream_t s);
// ---- the whole CCF_FFN + norm2 + Q4 residual in one kernel for C = 48, hidden = 192: the
// haloed h1 plane is computed in LDS from the x rows (pw MFMA + LN1 + GELU), never stored
int launch_ffn_fused(const DwFcArgs& a, int prec, hipStream_t s);
// K-chunked MFMA GEMM (gemm_kc.hip) for the shapes whose weight does not fit gemm_rows' LDS
// in one column chunk; returns 1 if it took the shape
int try_launch_gemm_kc(const GemmArgs& g, hipStream_t s);
// PatchMerging 1 -> 2 (C = 48) with the whole weight resident in LDS (merge.hip); returns 1
// if it took the shape
int try_launch_merge_resident(const GemmArgs& g, hipStream_t s);
// the stage-2 CCF_FFN pwconv (K = 96, N = 384) with the whole weight resident in LDS (pw2.hip);
// returns 1 if it took the shape
int try_launch_pw2_resident(const GemmArgs& g, hipStream_t s);
// stage-2 CCF_FFN pwconv (N = 384 with the LayerNorm + GELU epilogue, gemm_lnw.hip): columns
// split over the waves; returns 1 if it took the shape
int try_launch_gemm_lnw(const GemmArgs& g, hipStream_t s);
// the stage-3/4 wide-row pwconv shapes gemm_lnw takes (LayerNorm + GELU epilogue)
bool gemm_lnw_wide_shape(const GemmArgs& g);

}  // namespace wf
