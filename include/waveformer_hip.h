/*
 * waveformer_hip.h -- C-ABI of the MI355X (gfx950) WaveFormer hot-path library
 * (libwaveformer_hip.so).
 *
 * The library is the drop-in boundary for the WaveFormer encoder/decoder hot path
 * (SURVEY.md section 8a rows a1-a11).  Every entry point:
 *   - takes device pointers, int64 sizes and a hipStream_t (passed as void*),
 *   - never allocates (scratch is caller-owned; see the *_workspace_bytes queries),
 *   - is stream-ordered and reentrant (no mutable global state except the thread-local
 *     error string),
 *   - returns 0 on success, a positive hipError_t from the launch, or a negative
 *     WF_E* library code; wf_last_error() returns the message of the last failure on
 *     the calling thread.
 *
 * Tensor layouts (all row-major / C-contiguous unless a stride argument says otherwise):
 *   "channel-last"  (B, D, H, W, C)   -- the residual stream, LL bands, attention rasters
 *   "bands"         (8, B, d, h, w, C) -- band 0 = LL ('aaa'), bands 1..7 = the ptwt detail
 *                                         keys 'aad','ada','add','daa','dad','dda','ddd'
 *                                         (key char i <-> axis (D,H,W)[i]; 'a' low, 'd' high)
 *   "NCDHW"         (B, C, D, H, W)    -- PyTorch / MONAI convolution layout
 * Activations are fp32.  MFMA operands follow `precision`:
 *   WF_PREC_BF16  (0): operands rounded to bf16, fp32 accumulation, GEMM-to-GEMM intermediates
 *                      (qkv, attention output, FFN hidden) stored as bf16;
 *   WF_PREC_BF16X3 (1): fp32-faithful -- every operand x is split into hi = bf16(x) and
 *                      lo = bf16(x - hi) and products take hi*hi + lo*hi + hi*lo on the bf16
 *                      MFMA pipes (relative error ~2^-17); intermediates stored fp32.
 *   WF_PREC_FP16  (2): operands rounded to fp16 (relative error 2^-11), fp32 accumulation on
 *                      the v_mfma_f32_*_f16 pipes; intermediates stored fp32 (config 5).
 * LayerNorm, softmax, GELU, wavelets, interpolation and residual adds are fp32 in all modes.
 * Weights passed as `*_bf16x2` are nn.Linear / 1x1x1-Conv3d weights [N][K] as two 16-bit
 * planes [2][N][K]: {hi, lo} bf16 (wf_split_f32_to_bf16x2) for WF_PREC_BF16X3 and WF_PREC_BF16
 * (which reads the hi plane only); for WF_PREC_FP16 plane 0 holds fp16(W) (wf_cast_f32_to_f16x2,
 * plane 1 unused).  Every other parameter is the fp32 module tensor as-is.
 */
#ifndef WAVEFORMER_HIP_H
#define WAVEFORMER_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WF_ABI_VERSION 18

enum { WF_PREC_BF16 = 0, WF_PREC_BF16X3 = 1, WF_PREC_FP16 = 2 };

enum {
  WF_OK = 0,
  WF_E_SHAPE = -1,    /* a size or stride is unsupported (message names it) */
  WF_E_NULLPTR = -2,  /* a required pointer is NULL */
  WF_E_LAUNCH = -3    /* kernel launch failed (message has the HIP error string) */
};

int wf_abi_version(void);
const char* wf_last_error(void);

/* ---- utilities ------------------------------------------------------------------ */

/* out[i] = bf16(in[i]) (round-to-nearest-even). Weight preparation; no reference analogue. */
int wf_cast_f32_to_bf16(const float* in, uint16_t* out, int64_t n, void* stream);

/* out[i] = hi = bf16(in[i]), out[n + i] = bf16(in[i] - hi): the [2][...] weight planes. */
int wf_split_f32_to_bf16x2(const float* in, uint16_t* out, int64_t n, void* stream);

/* wf_split_f32_to_bf16x2 of n weights in one launch (the per-forward weight arena of
 * waveformer_amd.ops.weight_scope).  table_dev (device memory, int64): [n + 1] prefix sums of
 * the element counts, then the n fp32 source pointers, then the n destination pointers
 * ([2][numel] bf16 each); total = table[n].                                                */
int wf_split_f32_to_bf16x2_multi(const int64_t* table_dev, int64_t n, int64_t total,
                                 void* stream);

/* The WF_PREC_FP16 weight planes: out[i] = fp16(in[i]), out[n + i] = 0.  _multi: as
 * wf_split_f32_to_bf16x2_multi.                                                            */
int wf_cast_f32_to_f16x2(const float* in, uint16_t* out, int64_t n, void* stream);
int wf_cast_f32_to_f16x2_multi(const int64_t* table_dev, int64_t n, int64_t total,
                               void* stream);

/* Test support, not a reference op: `blocks` workgroups that each fill `lds_bytes` of LDS
 * with a NaN pattern and exit, so the next workgroups on those CUs start on garbage LDS (a
 * kernel that reads LDS it did not write then shows it).                                  */
int wf_debug_poison_lds(int64_t blocks, int lds_bytes, void* stream);

/* ---- a10: PatchEmbed -------------------------------------------------------------- */
/* Replaces monai PatchEmbed.proj = Conv3d(Cin, Cout, k=2, s=2) as called at
 * network_models/waveformer.py:281 (monai/networks/blocks/patchembedding.py:214).
 * x: NCDHW (B, Cin, 2D, 2H, 2W); w: (Cout, Cin, 2, 2, 2) fp32; bias: (Cout);
 * out: channel-last (B, D, H, W, Cout)  (== the rearrange at waveformer.py:286).        */
int wf_patch_embed_fwd(const float* x, const float* w, const float* bias, float* out,
                       int64_t B, int64_t Cin, int64_t Cout, int64_t D, int64_t H, int64_t W,
                       void* stream);
/* PatchEmbed fused with the first Block's norm1 + Haar LL (ABI 15; inference, when that Block's
 * detail bands are dropped): out as wf_patch_embed_fwd (exactly the same values), ll =
 * LL(LayerNorm(out; ln_w, ln_b, ln_eps)) (B, D/2, H/2, W/2, Cout) as wf_dwt3d_haar_fwd_ll would
 * give it up to the LayerNorm moments' summation order.  Cin 4 or 1, Cout 48, D/H/W even,
 * W <= 64.                                                                                 */
int wf_patch_embed_ll_fwd(const float* x, const float* w, const float* bias, float* out,
                          const float* ln_w, const float* ln_b, float ln_eps, float* ll,
                          int64_t B, int64_t Cin, int64_t Cout, int64_t D, int64_t H, int64_t W,
                          void* stream);

/* ---- a1: 1-level Haar analysis ----------------------------------------------------- */
/* Replaces ptwt.wavedec3(x, 'db1', level=1, mode='zero') at network_models/wave_helper.py:350,
 * including the NDHWC<->NCDHW permutes around it (wave_helper.py:484,486).
 * x: channel-last (B, D, H, W, C), D/H/W even. If ln_w != NULL the input is first
 * LayerNorm'ed over C with (ln_w, ln_b, ln_eps) -- Block.norm1 (wave_helper.py:477) fused.
 * bands: (8, B, D/2, H/2, W/2, C); band 0 is the LL that feeds the window attention.      */
int wf_dwt3d_haar_fwd(const float* x, const float* ln_w, const float* ln_b, float ln_eps,
                      float* bands, int64_t B, int64_t C, int64_t D, int64_t H, int64_t W,
                      void* stream);
/* The LL band alone (ABI 15): ll (B, D/2, H/2, W/2, C) bitwise equal to band 0 of
 * wf_dwt3d_haar_fwd.  For a Block whose detail bands nobody reads (wave_helper.py:509 keeps
 * only the LAST block's hf of each stage, waveformer.py:288-292): the 7 detail stores are
 * dropped, 8/9 of the launch's writes.                                                     */
int wf_dwt3d_haar_fwd_ll(const float* x, const float* ln_w, const float* ln_b, float ln_eps,
                         float* ll, int64_t B, int64_t C, int64_t D, int64_t H, int64_t W,
                         void* stream);

/* ---- a11: multi-level Haar synthesis ------------------------------------------------- */
/* Replaces ptwt.waverec3((LL,) + hf, 'db1') at network_models/idwt_upsample.py:160 and the
 * torch.cat((out, skip), dim=1) after it (:163): the reconstruction is written into channels
 * [0, C) of an NCDHW output whose batch stride is out_bstride elements.
 * ll: NCDHW (B, C, d, h, w) at the coarsest level (batch stride ll_bstride).
 * det[l*7 + k], l = 0..levels-1 coarse->fine, k = detail key 0..6 ('aad'..'ddd'):
 *   element (b, c, z, y, x) of level l lives at det[l*7+k][b*det_s[4l+0] + c*det_s[4l+1]
 *   + z*det_s[4l+2] + (y*W_l + x)*det_s[4l+3]]  (W_l = w * 2^l); channel-last band views and
 *   contiguous NCDHW tensors are both expressible.  levels in [1, 4].
 * out: (B, >=C, d*2^levels, h*2^levels, w*2^levels).                                     */
int wf_idwt3d_haar(const float* ll, int64_t ll_bstride, const float* const* det,
                   const int64_t* det_s, int levels, float* out, int64_t out_bstride,
                   int64_t B, int64_t C, int64_t d, int64_t h, int64_t w, void* stream);
/* The same into a channel-last output (ABI 12): element (b, c, z, y, x) of out lives at
 * out[b*out_bstride + ((z*H + y)*W + x)*ldo + c] -- channels [0, C) of a channels_last_3d
 * buffer of ldo >= C channels, so the decoder's concat buffer (idwt_upsample.py:163) stays in
 * the channel-last layout its convolutions read; the LL element (b, c, z, y, x) is read at
 * ll[b*ll_bstride + c*ll_cstride + ((z*h + y)*w + x)*ll_pstride] (NCDHW: d*h*w, 1;
 * channel-last: 1, its position stride).                                                  */
int wf_idwt3d_haar_cl(const float* ll, int64_t ll_bstride, int64_t ll_cstride,
                      int64_t ll_pstride, const float* const* det, const int64_t* det_s,
                      int levels, float* out, int64_t out_bstride, int64_t ldo, int64_t B,
                      int64_t C, int64_t d, int64_t h, int64_t w, void* stream);

/* wf_idwt3d_haar_cl fused with the concatenation that follows it (ABI 13; idwt_upsample.py:
 * 160-163, torch.cat((out, skip), 1)): also writes the C skip channels into channels [C, 2C)
 * of the same rows, skip element (b, c, pos) at skip[b*skip_bstride + pos*skip_ld + c]
 * (channel-last; skip_ld, skip_bstride multiples of 4, 16-byte aligned; ldo >= 2C).  Whole
 * 2C-channel rows leave the kernel instead of two half-row passes.                        */
int wf_idwt3d_haar_cl_cat(const float* ll, int64_t ll_bstride, int64_t ll_cstride,
                          int64_t ll_pstride, const float* const* det, const int64_t* det_s,
                          int levels, const float* skip, int64_t skip_bstride, int64_t skip_ld,
                          float* out, int64_t out_bstride, int64_t ldo, int64_t B, int64_t C,
                          int64_t d, int64_t h, int64_t w, void* stream);

/* ---- channel-last data movement of the decoder (ABI 12) ---------------------------- */
/* dst[p*ldd + c] = src[p*lds + c] for P positions x C channels (C, lds, ldd multiples of 4,
 * 16-byte aligned): a channel slice of one channels_last_3d tensor into another -- the
 * torch.cat((out, skip), 1) of UnetrUpBlock / UnetrIDWTBlock (monai unetr_block.py:84,
 * idwt_upsample.py:163) and network_backbone.py:404's torch.cat([..., dec2], 1).   */
int wf_copy_cl(const float* src, int64_t lds, float* dst, int64_t ldd, int64_t P, int64_t C,
               void* stream);
/* ConvTranspose3d(k = s = 2) output placement (monai unetr_block.py:73-80): g holds
 * (B*d*h*w, 8*C) GEMM rows, column s*C + c with s = dz*4 + dy*2 + dx; each goes to channel c of
 * position (b, 2z+dz, 2y+dy, 2x+dx) of the channel-last dst (positions ldd floats apart), plus
 * bias[c] (bias may be NULL).                                                              */
int wf_subvoxel_scatter_cl(const float* g, const float* bias, float* dst, int64_t ldd,
                           int64_t B, int64_t C, int64_t d, int64_t h, int64_t w, void* stream);
/* ConvTranspose3d(Cin, Cout, k = 2, s = 2) of the dense channel-last x (B, d, h, w, Cin) as one
 * MFMA GEMM (positions x Cin) . (Cin x 8 Cout) whose epilogue stores each 4-channel group, +
 * bias[c], straight to its sub-voxel of the channel-last out (positions ldo floats apart): the
 * transposed conv of UnetrUpBlock (monai unetr_block.py:73-80) without the (8 Cout)-wide
 * intermediate.  w_bf16x2: [2][8 Cout][Cin] 16-bit planes of weight.permute(2, 3, 4, 1, 0)
 * (row s * Cout + c).  Cin % 8 == 0, Cout % 4 == 0, ldo % 4 == 0.                           */
int wf_convtranspose2_cl(const float* x, const uint16_t* w_bf16x2, const float* bias, float* out,
                         int64_t ldo, int64_t B, int64_t Cin, int64_t Cout, int64_t d, int64_t h,
                         int64_t w, int precision, void* stream);

/* ---- C5: general wavelets (db1..db4), NCDHW, any sizes ------------------------------- */
/* One analysis level of ptwt.wavedec3(x, wavelet, mode='zero') (wave_helper.py:350 with a
 * wavelet other than 'db1'; BASELINE config 5 "db2 3-level DWT").  dec_lo / dec_hi are HOST
 * arrays of `taps` floats (pywt Wavelet.dec_lo / dec_hi, taps in {2,4,6,8}).
 * x: P contiguous (D, H, W) planes (P = B*C of an NCDHW tensor).
 * bands: (8, P, d, h, w) with d = (D + taps - 1) / 2 (same for h, w); band k bits
 * (z, y, x) = (k>>2, k>>1 & 1, k & 1), 'a' = 0 -- band 0 is LL, bands 1..7 'aad'..'ddd'.     */
int wf_dwt3d_fwd(const float* x, float* bands, int64_t P, int64_t D, int64_t H, int64_t W,
                 const float* dec_lo, const float* dec_hi, int taps, void* stream);

/* One synthesis level of ptwt.waverec3 (idwt_upsample.py:160 with a wavelet other than
 * 'db1').  coef[8]: band k as above (coef[0] = LL, already cropped to the details' shape by
 * the caller, pywt's rule), each (B, C, n_z, n_y, n_x) with its own 5 element strides
 * coef_strides[5k .. 5k+4] = (b, c, z, y, x).  rec_lo / rec_hi: HOST arrays of `taps` floats.
 * out: element (b, c, z, y, x) at b*out_bstride + c*out_cstride + (z*Oy + y)*Ox + x with
 * O = 2n - taps + 2 per axis.                                                               */
int wf_idwt3d_level(const float* const* coef, const int64_t* coef_strides, int64_t B, int64_t C,
                    int64_t n_z, int64_t n_y, int64_t n_x, const float* rec_lo,
                    const float* rec_hi, int taps, float* out, int64_t out_bstride,
                    int64_t out_cstride, void* stream);

/* ---- decoder: 3x3x3 convolution ------------------------------------- */
/* Replaces the decoder's Conv3d(Cin, Cout, 3, stride 1, padding 1) of MONAI's Convolution /
 * get_conv_layer (monai/networks/blocks/dynunet_block.py:98-111, :270-301), as called by
 * UnetResBlock / UnetBasicBlock / UnetrIDWTBlock.conv_lf_block (network_backbone.py:380-407).
 * Activations channel-last: position p = ((b*D + z)*H + y)*W + x at x[p*ldx + c] (a
 * channels_last_3d tensor, or a channel slice of one with ldx = its channel count), out the
 * same with ldo.  Cin % 4 == 0, Cout % 16 == 0.  bias (Cout) or NULL.
 * w_packed: wf_conv3d_k3_packed_elems(Cin, Cout) bf16 made by wf_conv3d_k3_pack from the
 * fp32 (Cout, Cin, 3, 3, 3) weight ([2] hi / lo planes, K-step-major).  precision WF_PREC_*. */
int64_t wf_conv3d_k3_packed_elems(int64_t Cin, int64_t Cout);
int wf_conv3d_k3_pack(const float* w, uint16_t* packed, int64_t Cin, int64_t Cout, void* stream);
/* The same packing as fp16 (plane 0 = fp16(W), plane 1 zero) for WF_PREC_FP16.             */
int wf_conv3d_k3_pack_f16(const float* w, uint16_t* packed, int64_t Cin, int64_t Cout,
                          void* stream);
/* stats_acc: NULL, or a ZEROED (B, Cout, 2) fp64 buffer that receives each output channel's
 * sum and sum of squares per sample (InstanceNorm statistics fused into the epilogue; finish
 * with wf_instnorm_finalize).
 * workspace: wf_conv3d_k3_workspace_bytes(...) bytes (0 for most shapes; NULL allowed).  Small
 * grids (the 8^3 / 16^3 decoder convs) split the input channels over several workgroups whose
 * partial outputs land there and are summed in a fixed order (ABI 14: bitwise repeatable; was
 * fp32 atomics).  With workspace NULL such grids run unsplit.                                 */
int64_t wf_conv3d_k3_workspace_bytes(int64_t B, int64_t Cin, int64_t Cout, int64_t D, int64_t H,
                                     int64_t W, int precision, int fp16_input);
int wf_conv3d_k3_fwd(const float* x, int64_t ldx, const uint16_t* w_packed, const float* bias,
                     float* out, int64_t ldo, double* stats_acc, void* workspace, int64_t B,
                     int64_t Cin, int64_t Cout, int64_t D, int64_t H, int64_t W, int precision,
                     void* stream);
/* wf_conv3d_k3_fwd at WF_PREC_FP16 with the input already fp16 (channel-last, ldx halves per
 * position, 8-byte aligned; w packed by wf_conv3d_k3_pack_f16): the operands are those the fp32
 * path stages after rounding, so the output is bitwise the same for an input written by
 * wf_norm_act_h_cl.  Half the staging bytes, no conversion.                                 */
int wf_conv3d_k3_fwd_xh(const uint16_t* x, int64_t ldx, const uint16_t* w_packed_f16,
                        const float* bias, float* out, int64_t ldo, double* stats_acc,
                        void* workspace, int64_t B, int64_t Cin, int64_t Cout, int64_t D,
                        int64_t H, int64_t W, void* stream);

/* Weight gradient of wf_conv3d_k3_fwd (training, config 4):
 *   dw[co, ci, kz, ky, kx] (+)= sum_p dy[p, co] * x[p + (kz-1, ky-1, kx-1), ci]
 * x, dy channel-last (positions ldx / ldg floats apart), dw (Cout, Cin, 3, 3, 3) fp32
 * (accumulate = 1 adds to it).  fp32-faithful bf16x3 MFMAs, deterministic (per-workgroup
 * partials in workspace, summed in a fixed order).  Cin % 4 == 0, Cout % 16 == 0.
 * workspace: wf_conv3d_k3_wgrad_workspace_bytes(B, Cin, Cout, D, H, W) bytes.                */
int64_t wf_conv3d_k3_wgrad_workspace_bytes(int64_t B, int64_t Cin, int64_t Cout, int64_t D,
                                           int64_t H, int64_t W);
int wf_conv3d_k3_wgrad(const float* x, int64_t ldx, const float* dy, int64_t ldg, float* dw,
                       int accumulate, void* workspace, int64_t B, int64_t Cin, int64_t Cout,
                       int64_t D, int64_t H, int64_t W, void* stream);

/* InstanceNorm3d(affine=False) statistics of a channel-last tensor: P positions per sample,
 * element (b, p, c) at x[(b*P + p)*ldx + c].  stats: (B, 2, C) fp32 {mean row, rstd row},
 * rstd = 1/sqrt(biased var + eps).  workspace: wf_instnorm_workspace_bytes(B, C) bytes.
 * The norm / act / residual glue of MONAI UnetResBlock / UnetBasicBlock
 * (monai/networks/blocks/dynunet_block.py:98-111, :170-185):
 *   out = act((a - mean_a) * rstd_a + r'),  r' = (r - mean_r) * rstd_r if stats_r, r if only
 *   r, 0 if r == NULL;  act = LeakyReLU(slope) (slope 1.0 = identity).  out may alias a.  */
int64_t wf_instnorm_workspace_bytes(int64_t B, int64_t C);
int wf_instnorm_stats_cl(const float* x, int64_t ldx, int64_t B, int64_t C, int64_t P, float eps,
                         float* stats, void* workspace, void* stream);
/* (B, C, 2) {sum, sum of squares} fp64 over P positions -> (B, 2, C) {mean, rstd} fp32. */
int wf_instnorm_finalize(const double* acc, float* stats, int64_t B, int64_t C, int64_t P,
                         float eps, void* stream);
int wf_norm_act_cl(const float* a, int64_t lda, const float* stats_a, const float* r, int64_t ldr,
                   const float* stats_r, float* out, int64_t ldo, int64_t B, int64_t C, int64_t P,
                   float slope, void* stream);
/* act((a - mean_a) * rstd_a) stored fp16 (round to nearest even, channel-last, ldo halves per
 * position): UnetResBlock / UnetBasicBlock's norm1 + lrelu (dynunet_block.py:101-103) feeding an
 * fp16 conv2 (wf_conv3d_k3_fwd_xh).                                                          */
int wf_norm_act_h_cl(const float* a, int64_t lda, const float* stats_a, uint16_t* out,
                     int64_t ldo, int64_t B, int64_t C, int64_t P, float slope, void* stream);

/* The norm3'ed 1x1 residual of UnetResBlock (monai dynunet_block.py:77-80, 104-108) for few
 * input channels (K = Cin <= 7; encoder1: 4 -> 48) without materialising it: wf_moments_cl
 * writes acc (B, K + K*K) fp64 = {sum_p x_k, sum_p x_k x_l} of the channel-last x (zeroed
 * first); the host folds InstanceNorm's mean_r = W mean_x + b, var_r = W_c^T Cov_x W_c into
 * per-sample wfold (B, C, K) = rstd_r W and bfold (B, C) = (b - mean_r) rstd_r, and
 * wf_norm_act_lin_cl applies out = act((a - mean_a) rstd_a + wfold x + bfold).              */
int wf_moments_cl(const float* x, int64_t ldx, int64_t B, int64_t K, int64_t P, double* acc,
                  void* stream);
int wf_norm_act_lin_cl(const float* a, int64_t lda, const float* stats_a, const float* x,
                       int64_t ldx, int64_t K, const float* wfold, const float* bfold,
                       float* out, int64_t ldo, int64_t B, int64_t C, int64_t P, float slope,
                       void* stream);

/* HFRefinementRes (network_models/idwt_upsample.py:12-50, config 5) over the 7 detail
 * tensors of one wavelet level: out_k = x_k * sigmoid(conv1x1(relu(IN_affine(dwconv3(x_k)))))
 * (sigmoid = 0: no sigmoid, hf_refinement.use_sigmoid False).  details: host array of 7
 * device pointers, each a channel-last (B, D, H, W, C) fp32 tensor with batch stride ldb
 * (the detail bands of wf_dwt3d_haar_fwd qualify); dw_w (C, 27), dw_b (C): the depthwise
 * conv1; in_w / in_b (C): the InstanceNorm3d affine, eps its eps (biased variance per
 * (detail, sample, channel)); pw_w (C, C), pw_b (C): conv2.  out: (7, B, D, H, W, C).
 * workspace: wf_hf_refine_workspace_bytes(B, C) bytes.  fp32 arithmetic throughout.          */
int64_t wf_hf_refine_workspace_bytes(int64_t B, int64_t C);
int wf_hf_refine_fwd(const float* const* details, int64_t ldb, const float* dw_w,
                     const float* dw_b, const float* in_w, const float* in_b, float eps,
                     const float* pw_w, const float* pw_b, int sigmoid, float* out,
                     void* workspace, int64_t B, int64_t C, int64_t D, int64_t H, int64_t W,
                     void* stream);

/* Backward of y = LeakyReLU(slope)((a - mean_a) * rstd_a + r') (wf_norm_act_cl; training of
 * UnetResBlock / UnetBasicBlock): dz = dy * (y > 0 ? 1 : slope),
 *   da = rstd_a * (dz - mean_P(dz) - xhat_a * mean_P(dz * xhat_a)),
 *   dr = rstd_r * (dz - mean_P(dz) - xhat_r * mean_P(dz * xhat_r)) with stats_r (normed
 *   residual, r given), dz without (plain residual), not written when dr == NULL.
 * Channel-last operands (positions ld* floats apart), stats (B, 2, C) {mean, rstd} as
 * wf_instnorm_stats_cl returns them.  workspace: wf_norm_act_bwd_workspace_bytes(B, C).      */
int64_t wf_norm_act_bwd_workspace_bytes(int64_t B, int64_t C);
int wf_norm_act_bwd_cl(const float* dy, int64_t ldd, const float* y, int64_t ldy,
                       const float* a, int64_t lda, const float* stats_a, const float* r,
                       int64_t ldr, const float* stats_r, float* da, int64_t ldda, float* dr,
                       int64_t lddr, int64_t B, int64_t C, int64_t P, float slope,
                       void* workspace, void* stream);

/* nn.Upsample(scale_factor=s, mode='trilinear', align_corners) of a channel-last tensor
 * (B, d, h, w, C) -> (B, D, H, W, C), PyTorch's upsample_trilinear3d index arithmetic: the
 * decoder's ProjectionUpsample (network_models/wave_helper.py:33-81, align_corners=True).    */
int wf_upsample_trilinear_cl(const float* in, float* out, int64_t B, int64_t C, int64_t d,
                             int64_t h, int64_t w, int64_t D, int64_t H, int64_t W,
                             int align_corners, void* stream);
/* out += the same resampling (ProjectionUpsample's y + Up(res_conv(x)), wave_helper.py:81). */
int wf_upsample_trilinear_add_cl(const float* in, float* out, int64_t B, int64_t C, int64_t d,
                                 int64_t h, int64_t w, int64_t D, int64_t H, int64_t W,
                                 int align_corners, void* stream);
/* ProjectionUpsample.conv1 fused (wave_helper.py:33-81, inference): nn.Upsample(trilinear,
 * align_corners) x (B, d, h, wd, C) channel-last -> depthwise 3^3 conv (zero padding on the
 * up-sampled volume) -> out (B, D, H, W, C) channel-last, the up-sampled tensor never stored;
 * its values are bitwise wf_upsample_trilinear_cl's.  stats_acc (B, C, 2) fp64: the outputs'
 * per-channel sum / sum of squares (zeroed here), for wf_instnorm_finalize.  C % 32 == 0,
 * bias required, W >= 2 wd (each 16-column tile's haloed source span <= 12 columns).        */
int wf_upsample_dwconv3d_stats_cl(const float* in, const float* w, const float* bias, float* out,
                                  double* stats_acc, int64_t B, int64_t C, int64_t d, int64_t h,
                                  int64_t wd, int64_t D, int64_t H, int64_t W, int align_corners,
                                  void* stream);
/* UnetOutBlock (monai dynunet_block.py:188-210, network_backbone.py:407): 1x1x1 conv of the
 * channel-last x (B, P positions ldx floats apart, K channels) with weight (N, K) + bias (N)
 * into the NCDHW out (B, N, P).  K % 4 == 0, K <= 120, N <= 16; fp32 FMAs.                  */
int wf_conv1x1_head_cl(const float* x, int64_t ldx, const float* weight, const float* bias,
                       float* out, int64_t B, int64_t K, int64_t N, int64_t P, void* stream);
/* y (M, N) = x (M, K) . w (N, K)^T + bias for K in [1, 7] (ABI 18): the shapes the MFMA GEMM
 * (wf_linear_fwd, K % 8 == 0) does not take -- in training, UnetResBlock's 1x1 residual conv of
 * the 4-channel input (dynunet_block.py:77-80) and the input gradient of the 4-class
 * UnetOutBlock (:188-210).  Row strides ldx / ldy floats; N % 4 == 0, y 16-B aligned; exact
 * fp32 FMAs (bias first, then k in order).                                                   */
int wf_linear_smallk_fwd(const float* x, int64_t ldx, const float* w, const float* bias,
                         float* y, int64_t ldy, int64_t M, int64_t K, int64_t N, void* stream);
/* Depthwise Conv3d(C, C, 3, padding 1, groups C) + bias of a dense channel-last fp32 tensor
 * (ProjectionUpsample.conv1, wave_helper.py:43-46) with the per-(sample, channel) fp64 {sum, sum
 * of squares} of its output accumulated in the epilogue into stats_acc (B, C, 2) (zeroed here)
 * -- the GroupNorm(C, C) statistics of wave_helper.py:60 without a second pass.  C % 32 == 0. */
int wf_dwconv3d_stats_cl(const float* in, const float* w, const float* bias, float* out,
                         double* stats_acc, int64_t B, int64_t C, int64_t D, int64_t H,
                         int64_t W, void* stream);

/* Predictor.predict_raw_probability (light_training/prediction.py:35-63): channel-first
 * (C, d, h, w) fp32 (channel stride ldc) -> (C, D, H, W) per channel
 * F.interpolate(mode='trilinear', align_corners), written fp16 (out_f16 = 1, the reference's
 * torch.half buffer) or fp32.  PyTorch's upsample_trilinear3d index arithmetic.             */
int wf_resample_trilinear_cf(const float* in, int64_t ldc, int64_t C, int64_t d, int64_t h,
                             int64_t w, int64_t D, int64_t H, int64_t W, int align_corners,
                             void* out, int out_f16, void* stream);

/* out (M, N) = bias + act(x) (M, K) . W^T, act = GELU(erf) if gelu_in else identity; fp32
 * rows, W as [2][N][K] bf16 hi / lo planes (wf_split_f32_to_bf16x2).  The 1x1x1 convolutions
 * of the decoder's ProjectionUpsample (network_models/wave_helper.py:33-81), GELU fused into
 * the next GEMM's operand loader.  K % 8 == 0, N % 4 == 0.                                    */
int wf_linear_fwd(const float* x, const uint16_t* w_bf16x2, const float* bias, float* out,
                  int64_t M, int64_t K, int64_t N, int gelu_in, int precision, void* stream);

/* wf_window_attention_fwd with the bias taken from the (T, heads) relative_position_bias_table
 * directly: the index is the reference's formula (attention.py:40-56, Q2 depth stride 3ws-1)
 * computed from the token coordinates, the table column staged in LDS -- valid when the
 * module's relative_position_index buffer equals that formula (the caller checks).  ws = 8,
 * head_dim = 16.                                                                             */
int wf_window_attention_fwd_table(const float* x, const float* ln_w, const float* ln_b,
                                  float ln_eps, const uint16_t* wqkv_bf16x2, const float* bqkv,
                                  const float* table, const uint16_t* wproj_bf16x2,
                                  const float* bproj, float* out, void* workspace, int64_t B,
                                  int64_t C, int64_t D1, int64_t H1, int64_t W1, int64_t ws,
                                  int64_t heads, float scale, int precision, void* stream);

/* ---- a2: relative-position bias ------------------------------------------------------ */
/* bias[h][i][j] = table[index[i][j]][h]  (attention.py:94-97), index is the int64
 * relative_position_index buffer (N, N), table (T, heads).                                */
int wf_rel_pos_bias(const float* table, const int64_t* index, float* bias, int64_t N,
                    int64_t heads, int64_t table_rows, void* stream);

/* ---- a3/a4/a5: windowed multi-head self-attention ------------------------------------- */
/* Replaces Block.window_partition (wave_helper.py:450-461) + Attention.forward
 * (attention.py:83-104) + the window "reverse" reshape (wave_helper.py:498-499, quirk Q1).
 * x: channel-last raster (B, D1, H1, W1, C); windows of ws^3 tokens are gathered with the
 * (B, D/ws, H/ws, W/ws) window-major order of window_partition.  If ln_w != NULL the tokens
 * are LayerNorm'ed first (Block.norm1 for level-0 blocks, wave_helper.py:477).
 * out: (B*nW*N, C) fp32 in window-major order, which IS the (B, D1, H1, W1, C) raster that
 * the reference's reshape produces (Q1).  raster_rows: x is (B*D1*H1*W1, C); when
 * D1=H1=W1=ws=N^(1/3) and x is a plain (B_, N, C) token batch this is Attention.forward.
 * wqkv_bf16x2 [2](3C, C), bqkv (3C) or NULL, bias (heads, N, N) from wf_rel_pos_bias,
 * wproj_bf16x2 [2](C, C), bproj (C).  scale = qk_scale or head_dim^-0.5.
 * head_dim in {16, 32, 48, 64, 96, 128, 192, 384}.
 * workspace: wf_window_attention_workspace_bytes(...) bytes, 256-B aligned.               */
int64_t wf_window_attention_workspace_bytes(int64_t B, int64_t C, int64_t D1, int64_t H1,
                                            int64_t W1, int precision);
int wf_window_attention_fwd(const float* x, const float* ln_w, const float* ln_b, float ln_eps,
                            const uint16_t* wqkv_bf16x2, const float* bqkv,
                            const float* bias, const uint16_t* wproj_bf16x2, const float* bproj,
                            float* out, void* workspace, int64_t B, int64_t C, int64_t D1,
                            int64_t H1, int64_t W1, int64_t ws, int64_t heads, float scale,
                            int precision, void* stream);

/* ---- a6: multi-scale fuse ------------------------------------------------------------- */
/* Replaces the F.interpolate(trilinear, align_corners=False) + sum + shortcut of
 * wave_helper.py:500-508 and computes the per-position LayerNorm statistics that Block.norm2
 * (wave_helper.py:509) needs.
 * src[s]: channel-last (B, sd[s], sh[s], sw[s], C), s < nsrc <= 4; a source whose size equals
 * (D,H,W) is added as-is (level-0 path, wave_helper.py:505).  shortcut, out: (B, D, H, W, C).
 * stats: (B*D*H*W, 2) = {mean, rstd} of out rows with eps ln_eps (NULL: not computed).
 * branch_scale: NULL, or (B) per-sample factors applied to the fused attention branch --
 * the DropPath (timm, train mode) of wave_helper.py:508 as a per-sample keep/(1-p) mask.   */
int wf_msfuse_fwd(const float* const* src, const int64_t* src_dhw, int nsrc,
                  const float* shortcut, const float* branch_scale, float* out, float* stats,
                  float ln_eps, int64_t B, int64_t C, int64_t D, int64_t H, int64_t W,
                  void* stream);

/* ---- a7/a8: CCF_FFN + the Block's norm2 and double residual (quirk Q4) ---------------- */
/* Replaces attn_fused + mlp(norm2(attn_fused)) (wave_helper.py:509) with CCF_FFN.forward
 * (wave_helper.py:260-294): pwconv(1x1x1, bias) -> LN(4C, eps1) -> GELU(erf) ->
 * dwconv(3^3, groups=4C, pad 1, bias) -> LN(4C, eps1) -> GELU -> fc(Linear, bias) -> +input.
 * xh: channel-last (B, D, H, W, C).  If stats != NULL the FFN input is
 * n2 = LN(xh; stats, n2_w, n2_b) and out = xh + n2 + ffn(n2) (Block, Q4);
 * if stats == NULL the input is xh itself and out = xh + ffn(xh) (bare CCF_FFN.forward).
 * pw_bf16x2 [2](4C, C), pw_b (4C), ln1_w/b (4C), dw_w (4C, 27) fp32, dw_b (4C),
 * ln2_w/b (4C), fc_bf16x2 [2](C, 4C), fc_b (C).  branch_scale: NULL or (B) per-sample
 * DropPath factors on the FFN branch (wave_helper.py:509).
 * workspace: wf_ccf_ffn_workspace_bytes(...) bytes.                                        */
int64_t wf_ccf_ffn_workspace_bytes(int64_t B, int64_t C, int64_t hidden, int64_t D, int64_t H,
                                   int64_t W, int precision);
int wf_ccf_ffn_fwd(const float* xh, const float* stats, const float* n2_w, const float* n2_b,
                   const uint16_t* pw_bf16x2, const float* pw_b, const float* ln1_w,
                   const float* ln1_b, float eps1, const float* dw_w, const float* dw_b,
                   const float* ln2_w, const float* ln2_b, float eps2,
                   const uint16_t* fc_bf16x2, const float* fc_b, const float* branch_scale,
                   float* out, void* workspace,
                   int64_t B, int64_t C, int64_t hidden, int64_t D, int64_t H, int64_t W,
                   int precision, void* stream);
/* The same three launches one at a time (stage 1: pwconv GEMM -> workspace h1; 2: depthwise
 * conv h1 -> h2 + per-32-channel LayerNorm partials; 3: LN2 + GELU + fc GEMM + residuals ->
 * out), with the same arguments; stage 0 runs all three (== wf_ccf_ffn_fwd).  Lets a caller
 * time or interleave the stages.  stage | 16 (training) forces the staged kernels for every
 * shape, so that on return the workspace holds h1 = GELU(LN1(pwconv(n))) at offset 0 and
 * h2 = dwconv(h1) + dw_b (before LN2) at the next 256-B boundary, both fp32 (WF_PREC_BF16X3). */
int wf_ccf_ffn_stage(int stage, const float* xh, const float* stats, const float* n2_w,
                     const float* n2_b, const uint16_t* pw_bf16x2, const float* pw_b,
                     const float* ln1_w, const float* ln1_b, float eps1, const float* dw_w,
                     const float* dw_b, const float* ln2_w, const float* ln2_b, float eps2,
                     const uint16_t* fc_bf16x2, const float* fc_b, const float* branch_scale,
                     float* out, void* workspace, int64_t B, int64_t C, int64_t hidden,
                     int64_t D, int64_t H, int64_t W, int precision, void* stream);

/* ---- a9: PatchMerging (quirk Q3) ------------------------------------------------------ */
/* Replaces PatchMerging.forward (wave_helper.py:173-194): the 8-way strided gather with its
 * duplicated sub-lattices, LN(8C, eps) and Linear(8C -> 2C, no bias).  v2 != 0 selects
 * PatchMergingV2.forward's itertools.product order instead (wave_helper.py:147-167).
 * x: channel-last (B, D, H, W, C) (D, H, W even); out: channel-last (B, D/2, H/2, W/2, 2C).
 * red_bf16x2: [2](2C, 8C).                                                                 */
int wf_patch_merging_fwd(const float* x, const float* ln_w, const float* ln_b, float eps,
                         const uint16_t* red_bf16x2, int v2, float* out, int64_t B, int64_t C,
                         int64_t D, int64_t H, int64_t W, int precision, void* stream);

/* ---- a10: stage output projection (quirk Q5) ----------------------------------------- */
/* Replaces MultiscaleTransformer.proj_out (waveformer.py:182-204) together with the
 * rearrange to NCDHW before it (waveformer.py:289): non-affine LayerNorm over C with eps,
 * x channel-last (B, S, C) (S = D*H*W) -> out NCDHW (B, C, S).  normalize=0 only transposes. */
int wf_proj_out_fwd(const float* x, float* out, int normalize, float eps, int64_t B,
                    int64_t C, int64_t S, void* stream);
/* proj_out for a channel-last consumer (the full model's encoder2-4 / encoder10 UnetResBlocks,
 * network_backbone.py:387-392): the same non-affine LayerNorm, x (M, C) -> out (M, C), values
 * bitwise those wf_proj_out_fwd writes, with no NCDHW round trip.                           */
int wf_proj_out_cl_fwd(const float* x, float* out, float eps, int64_t M, int64_t C, void* stream);

/* ---- sliding-window inference (config 3) ----------------------- */
/* Replaces monai.data.utils.compute_importance_map (monai/data/utils.py:1088-1138) as called
 * by sliding_window_inference (monai/inferers/utils.py:194-207).  mode 0 = 'constant' (ones),
 * 1 = 'gaussian': exp(x^2 / (-2 sigma^2)) per axis with x = -(n-1)/2 .. (n-1)/2 and
 * sigma = sigma_scale[axis] * n, multiplied out in (z, y, x) order and clamped below at
 * max(min, 1e-3).  out: (rd, rh, rw) fp32.  sigma_scale: 3 host floats (NULL for mode 0).   */
int wf_importance_map(int mode, const float* sigma_scale, float* out, int64_t rd, int64_t rh,
                      int64_t rw, void* stream);

/* Replaces the accumulation loop of sliding_window_inference (monai/inferers/utils.py:216-299:
 * out[slice] += pred * w, count[slice] += w, out /= count) for predictor outputs of the
 * window's own spatial size.  Gather form: every output voxel sums the windows covering it
 * in ascending window order with the reference's fp32 operation order.
 * starts: host int64 array of nwin[0] + nwin[1] + nwin[2] window starts (z, then y, then x;
 *   strictly ascending per axis, spanning the axis -- dense_patch_slices,
 *   monai/data/utils.py:171-211); windows are numbered in its 'ij' meshgrid order and images
 *   batch-major: g = b * nwin_total + (iz * nwin[1] + iy) * nwin[2] + ix.
 * patches: (rows, C, rd, rh, rw) fp32.  Window g lives in row
 *   ((j / slots_per_round) * world + g % world) * slots_per_round + j % slots_per_round,
 *   j = g / world: the layout of per-round all-gathers of round-robin shards (window g on
 *   rank g % world, slot j).  world = 1 (any slots_per_round) is plain window order.
 * importance_map: (rd, rh, rw) fp32 (wf_importance_map or a caller's roi_weight_map).
 * out: (B, C, D, H, W) fp32, D/H/W the (padded) image size.                                 */
int wf_sliding_window_stitch(const float* patches, int64_t world, int64_t slots_per_round,
                             const float* importance_map, const int64_t* starts,
                             const int64_t* nwin, float* out, int64_t B, int64_t C, int64_t D,
                             int64_t H, int64_t W, int64_t rd, int64_t rh, int64_t rw,
                             void* stream);

/* The all-reduce exchange of the sharded sliding window (ABI 14): each rank sums
 * only the windows it predicted -- g % world == rank, held in its local patch rows
 * j = g / world: patches (slots, C, rd, rh, rw) -- in ascending window order, into
 * out (B, C + 1, D, H, W): channels [0, C) = sum pred * w, channel C = sum w (no division).
 * The ranks' outputs are then summed (one all-reduce of (C + 1) x D x H x W per image) and
 * wf_sliding_window_normalize divides.  world = 1 gives, after normalising, bitwise the
 * wf_sliding_window_stitch result.                                                          */
int wf_sliding_window_stitch_partial(const float* patches, int64_t world, int64_t rank,
                                     const float* importance_map, const int64_t* starts,
                                     const int64_t* nwin, float* out, int64_t B, int64_t C,
                                     int64_t D, int64_t H, int64_t W, int64_t rd, int64_t rh,
                                     int64_t rw, void* stream);
/* out (B, C, D, H, W) = num[:, :C] / num[:, C] for num (B, C + 1, D, H, W).                */
int wf_sliding_window_normalize(const float* num, float* out, int64_t B, int64_t C, int64_t D,
                                int64_t H, int64_t W, void* stream);

/* Flip test-time augmentation merge of Predictor.maybe_mirror_and_predict
 * (light_training/prediction.py:110-160): out = (sum_p flip_p(pred[p])) / npass, summed in
 * pass order.  pred: (npass, C, D, H, W) fp32, pass p computed on the input flipped along the
 * axes of flips[p] (host int mask: bit 0 = D, bit 1 = H, bit 2 = W; 0 = no flip), npass <= 8.
 * out: (C, D, H, W) fp32.                                                                    */
int wf_tta_merge(const float* pred, const int* flips, int npass, float* out, int64_t C,
                 int64_t D, int64_t H, int64_t W, void* stream);

/* ======================================================================================
 * Training (config 4: fwd + bwd DiceCE on 128^3 x 4 crops, DDP).  The reference trains with
 * PyTorch autograd through the modules of SURVEY 8a (3_train.py:99-135, trainer.py:454); these
 * entry points are the backward halves of the forward ops above, plus the few gather/reduce
 * primitives the Python autograd.Functions need.  Dense GEMM gradients are left to the
 * caller's BLAS (hipBLASLt).  All fp32.  Reductions are two-pass (partials + a final pass),
 * so results are deterministic run to run; scratch is caller-owned as elsewhere.
 * ====================================================================================== */

/* Attention forward that also writes the per-row log-sum-exp of the softmax, in the log2
 * domain: lse[(bw * heads + h) * N + q] = log2 sum_k exp2(S'_qk), S' = (scale q.k + bias) log2 e.
 * Same arguments as wf_window_attention_fwd otherwise; the workspace (qkv, then the
 * attention output o at the next 256-B boundary) is what the backward consumes.            */
int wf_window_attention_fwd_train(const float* x, const float* ln_w, const float* ln_b,
                                  float ln_eps, const uint16_t* wqkv_bf16x2, const float* bqkv,
                                  const float* bias, const uint16_t* wproj_bf16x2,
                                  const float* bproj, float* out, void* workspace, float* lse,
                                  int64_t B, int64_t C, int64_t D1, int64_t H1, int64_t W1,
                                  int64_t ws, int64_t heads, float scale, int precision,
                                  void* stream);

/* Backward of softmax(scale q k^T + bias) v per window and head (attention.py:92-101).
 * qkv (B*nW*N, 3C) and o (B*nW*N, C) window-major fp32 as saved by the forward, dout the
 * gradient of o (window-major), lse from wf_window_attention_fwd_train.
 * dqkv: (B*D1*H1*W1, 3C) in RASTER row order (the inverse of window_partition,
 * wave_helper.py:450-461), so the qkv weight gradient pairs it with the un-permuted input.
 * dbias: (heads, N, N), the bias gradient summed over all windows.  Every element of both is
 * written (no zeroing needed).  Deterministic (ABI 14): no atomics; the key-block partials of
 * dQ and the window-group partials of dbias live in `workspace`
 * (wf_window_attention_bwd_workspace_bytes) and are summed in index order.
 * head_dim in {16, 32, 48, 64}.                                                             */
int64_t wf_window_attention_bwd_workspace_bytes(int64_t B, int64_t C, int64_t D1, int64_t H1,
                                                int64_t W1, int64_t ws, int64_t heads);
int wf_window_attention_bwd_core(const float* qkv, const float* o, const float* dout,
                                 const float* bias, const float* lse, float* dqkv, float* dbias,
                                 void* workspace, int64_t B, int64_t C, int64_t D1, int64_t H1,
                                 int64_t W1, int64_t ws, int64_t heads, float scale,
                                 void* stream);

/* c[n][k] (+)= sum_m a[m][n] * b[m][k] -- dW = dY^T X of the training path's Linear / 1x1
 * conv / transposed-conv weights (ABI 14).  a (M, >= N) and b (M, >= K) fp32 row-major, lda /
 * ldb floats apart; c (N, K), ldc apart (accumulate = 1 adds to it).  fp32-faithful bf16x3
 * MFMAs, M dealt to many workgroups whose partials (workspace:
 * wf_gemm_tn_workspace_bytes(M, N, K) bytes) are summed in a fixed order: deterministic.    */
int64_t wf_gemm_tn_workspace_bytes(int64_t M, int64_t N, int64_t K);
int wf_gemm_tn(const float* a, int64_t lda, const float* b, int64_t ldb, float* c, int64_t ldc,
               int accumulate, void* workspace, int64_t M, int64_t N, int64_t K, void* stream);

/* dtable[r][h] = sum of dbias[h][i][j] over index[i][j] == r (the gather at
 * attention.py:94-97, adjoint), in ascending flat order: `perm` (N*N) lists the flat positions
 * i*N + j grouped by table row (a stable sort of the index), `offsets` (table_rows + 1) delimits
 * the groups.  Deterministic (ABI 14); every element of dtable (table_rows, heads) is written. */
int wf_rel_pos_bias_bwd(const float* dbias, const int64_t* perm, const int64_t* offsets,
                        float* dtable, int64_t N, int64_t heads, int64_t table_rows,
                        void* stream);

/* out[c] = sum_r in[r][c] * (row_scale ? row_scale[r / rows_per_scale] : 1): bias gradients.
 * partials: wf_colsum_parts(R) * N floats.                                                  */
int64_t wf_colsum_parts(int64_t R);
int wf_colsum(const float* in, int64_t R, int64_t N, const float* row_scale,
              int64_t rows_per_scale, float* partials, float* out, void* stream);

/* y = GELU?(LayerNorm(x)) over rows of N <= 1536 (w == NULL: no affine).  The LN -> GELU pairs
 * of CCF_FFN (wave_helper.py:278-286), Block.norm1/norm2, PatchMerging.norm and proj_out.    */
int wf_ln_act_fwd(const float* x, const float* w, const float* b, float eps, int gelu, float* y,
                  int64_t M, int64_t N, void* stream);
/* Backward of wf_ln_act_fwd: dx = [dadd +] dLN(dy * GELU'(z)); dw / db (when w != NULL) the
 * affine gradients.  partials: wf_ln_bwd_workspace_floats(M, N) floats.                     */
int64_t wf_ln_bwd_workspace_floats(int64_t M, int64_t N);
int wf_ln_act_bwd(const float* x, const float* w, const float* b, float eps, int gelu,
                  const float* dy, const float* dadd, float* dx, float* partials, float* dw,
                  float* db, int64_t M, int64_t N, void* stream);

/* Adjoint of wf_dwt3d_haar_fwd (without its fused LayerNorm): dx (B, D, H, W, C) channel-last
 * from the 8 band gradients dband[k] (NULL = zero), element (b, z, y, x, c) of band k at
 * dband[k][b*s[5k] + z*s[5k+1] + y*s[5k+2] + x*s[5k+3] + c*s[5k+4]].                        */
int wf_dwt3d_haar_bwd(const float* const* dband, const int64_t* strides, float* dx, int64_t B,
                      int64_t C, int64_t D, int64_t H, int64_t W, void* stream);

/* One Haar analysis level of an NCDHW tensor (the adjoint of one wf_idwt3d_haar level):
 * in (B, C, 2d, 2h, 2w), element (b, c, ...) at in + b*in_bstride + c*in_cstride, spatially
 * contiguous.  ll: (B, C, d, h, w) contiguous; det[k] (k = 0..6, key 'aad'..'ddd') element
 * (b, c, z, y, x) at det[k][b*s[0] + c*s[1] + z*s[2] + y*s[3] + x*s[4]].                    */
int wf_haar_analysis_ncdhw(const float* in, int64_t in_bstride, int64_t in_cstride, float* ll,
                           float* const* det, const int64_t* det_strides, int64_t B, int64_t C,
                           int64_t d, int64_t h, int64_t w, void* stream);

/* Adjoint of F.interpolate(trilinear, align_corners=False) along one axis
 * (wave_helper.py:500): in (outer, Lout, inner) -> out (outer, Lin, inner), optionally times
 * outer_scale[o / outer_per_scale] (the DropPath factor of the attention branch).           */
/* The same for align_corners=True (ProjectionUpsample's nn.Upsample, wave_helper.py:33-81):
 * three calls (x, y, z axes of a channel-last tensor) give the backward of upsample_cl.     */
int wf_interp_adjoint_axis_ac(const float* in, float* out, int64_t outer, int64_t Lout,
                              int64_t Lin, int64_t inner, void* stream);
int wf_interp_adjoint_axis(const float* in, float* out, int64_t outer, int64_t Lout,
                           int64_t Lin, int64_t inner, const float* outer_scale,
                           int64_t outer_per_scale, void* stream);

/* Depthwise 3^3 conv, channel-last, padding 1 (CCF_FFN.dwconv, wave_helper.py:285):
 * w (C, 27), bias (C) or NULL; flip != 0 convolves with the flipped kernel (the input
 * gradient).  C % 4 == 0.                                                                  */
int wf_dwconv3d_cl(const float* in, const float* w, const float* bias, int flip, float* out,
                   int64_t B, int64_t C, int64_t D, int64_t H, int64_t W, void* stream);
/* dw (C, 27) = sum over positions of dy[pos][c] x[pos + offset_k][c]: z-streaming LDS-tiled
 * for C % 32 == 0 (ABI 14), per-tile partials summed in a fixed order (deterministic).
 * partials: wf_dwconv_wgrad_ws_floats(B, C, D, H, W) floats.                                */
int64_t wf_dwconv_wgrad_ws_floats(int64_t B, int64_t C, int64_t D, int64_t H, int64_t W);
int wf_dwconv3d_wgrad(const float* dy, const float* x, float* partials, float* dw, int64_t B,
                      int64_t C, int64_t D, int64_t H, int64_t W, void* stream);

/* PatchMerging's 8-way sub-lattice gather (wave_helper.py:183-191, Q3 duplicates; v2 = the
 * itertools.product order of :154-156): merged (B, D/2, H/2, W/2, 8C).  The scatter is its
 * adjoint: dx sums every slot a position was gathered into (0, 1 or 2 under Q3).           */
int wf_patch_merging_gather(const float* x, int v2, float* merged, int64_t B, int64_t C,
                            int64_t D, int64_t H, int64_t W, void* stream);
int wf_patch_merging_scatter(const float* dmerged, int v2, float* dx, int64_t B, int64_t C,
                             int64_t D, int64_t H, int64_t W, void* stream);

/* PatchEmbed patches (patchembedding.py:214, Conv3d k=2 s=2): x NCDHW (B, Cin, 2D, 2H, 2W)
 * <-> rows (B*D*H*W, Cin*8) in the flattened weight order (ci, kz, ky, kx); dir 0 gathers x
 * into rows, dir 1 scatters rows into x.                                                    */
int wf_patchify(float* x, float* rows, int dir, int64_t B, int64_t Cin, int64_t D, int64_t H,
                int64_t W, void* stream);

/* (B, C, S) -> (B, S, C): the NCDHW -> channel-last transpose (proj_out's adjoint,
 * waveformer.py:289).                                                                       */
int wf_transpose_cs(const float* in, float* out, int64_t B, int64_t C, int64_t S, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* WAVEFORMER_HIP_H */
