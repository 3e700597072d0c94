/*
 * librfhip — C ABI of the MI355X-native RenderFormer inference path.
 *
 * Every entry point is stream-ordered and asynchronous (no device sync, no
 * allocation), takes plain device pointers, explicit sizes/strides (in
 * elements) and a hipStream_t passed as `void*`, and returns RF_OK or an
 * error code; rf_last_error() returns a thread-local message.  The caller
 * owns every buffer.  Tensors are row-major; "bf16" buffers hold raw
 * bfloat16 bits, "f32" buffers IEEE float.
 *
 * Reference interfaces replaced (paths relative to the reference checkout):
 *   rf_gemm_bf16       nn.Linear / aten mm+addmm in attention.py:51-57,95-100,121-125,202,342,361;
 *                      renderformer.py:49,63 (encoders); view_transformer.py:45 (ray encoder)
 *   rf_rmsnorm         nn.RMSNorm pre-norms attention.py:436-439,463,482 (+ kv_norm :508)
 *   rf_prenorm / rf_gemm_add_prenorm / rf_gemm_rownorm  the same pre-norms deferred into the GEMMs around them
 *                      (the residual GEMM's epilogue writes x * g and row sums of squares, the projection after
 *                      the norm scales its rows by 1 / rms): what rf_encoder_forward / rf_decoder_forward issue
 *   rf_qk_norm_rope    q/k RMSNorm over full width (attention.py:127-133) fused with the
 *                      triangle RoPE (rope.py:106-149 apply_rotary_emb_*cossin, :78-103, :315-333)
 *   rf_attn_fwd        flash_attn_varlen_qkvpacked_func / flash_attn_varlen_kvpacked_func
 *                      (attention.py:164-198) and the masked SDPA branch (attention.py:143-161);
 *                      rf_attn_combine / rf_attn_workspace_bytes belong to its split-KV mode
 *   rf_swin_attn_fwd   SwinSelfAttention roll + window_partition + masked SDPA + window_reverse
 *                      (attention.py:205-271, 316-370), with the roll done as index math
 *   rf_texture_pack    rendering_pipeline.py:67-68 (in-place log10 encode) + renderformer.py:145-147
 *                      flatten, with flash_attn.bert_padding.unpad_input-style compaction
 *   rf_texture_scan / rf_texture_linear  the texture encoder Linear (renderformer.py:145-147, 49) on
 *                      to_h5-format textures (scene_processor/to_h5.py:41-66: per-channel constant x fixed
 *                      patch mask) as a C-wide product with mask-summed weights, proven per call on the
 *                      device; rf_texture_pack_if / rf_gemm_bf16_if run the general path only when the
 *                      proof fails (device-side flag, no host round trip)
 *   rf_vn_encode       NeRFEncoding (nerf_encoding.py:63-84) on vertex normals, renderformer.py:139
 *   rf_ray_tokens      RayGenerator (ray_generator.py:13-50) + patchify rearrange (view_transformer.py:104-105)
 *   rf_patchify_rays   the patchify rearrange alone, for RenderFormer.forward callers (renderformer.py:171)
 *   rf_scene_pos       trans_to_cam_coord (transform.py:7-27) + process_tri_vpos_list (renderformer.py:103-124)
 *   rf_embed           token assembly renderformer.py:139-163, view_transformer.py:108 (RMSNorm eps=None)
 *   rf_hdr_output      ELU(1e-3) (view_transformer.py:86,122) + 10^x - 1 + permute (rendering_pipeline.py:119-123)
 *   rf_conv2d_bf16x3   DPT nn.Conv2d (dpt.py:44-52, 69-72, 124-125, 184-192, 208-213, 232-240; aten conv2d) with
 *                      the ResidualConvUnit SiLU/skip (dpt.py:86-92) and fusion sum (:141-143) fused; FINAL mode
 *                      also fuses output_conv2 SiLU + 1x1 (dpt.py:234-240), ELU and the log decode
 *   rf_conv2d_f16 / rf_deconv2d_f16  the same two DPT convolutions with fp16 operands (one MFMA per product)
 *   rf_conv1x1_f16_group  the four DPT tap projections (dpt.py:197-199, 244-249) as one launch
 *   rf_conv2d_f16_group   independent DPT convolutions / deconvolutions (resize layers, layer*_rn) as one launch
 *   rf_split_planes    (operand preparation for the above; no reference counterpart)
 *   rf_deconv2d_bf16x3 DPT nn.ConvTranspose2d kernel == stride (dpt.py:195-206; aten conv_transpose2d)
 *   rf_upsample_bilinear F.interpolate(bilinear, align_corners=True) (dpt.py:154-155, 269-270)
 *   rf_upsample_bilinear_h  the same resize on fp16 planes: refinenet1's output straight into output_conv1,
 *                      whose weights hold the folded 1x1 out_conv (dpt.py:157-159, 268-271; RF_CONV_BORDER_BIAS)
 *   rf_encoder_forward TransformerEncoder.forward (attention.py:579-590): the whole stage-1 stack in one call
 *   rf_decoder_forward TransformerDecoder.forward (attention.py:673-688) + the DPT taps (view_transformer.py:85)
 */
#ifndef RF_H
#define RF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RF_OK 0
#define RF_ERR_INVALID 1
#define RF_ERR_LAUNCH 2
#define RF_ERR_UNSUPPORTED 3
#define RF_ERR_DEVICE 4       /* an earlier launch reported a device-side error (see rf_device_error) */

#define RF_ABI_VERSION 16

/* GEMM epilogues */
#define RF_EPI_BF16 0       /* C(bf16)  = A W^T + bias                                   */
#define RF_EPI_F32 1        /* C(f32)   = A W^T + bias                                   */
#define RF_EPI_ADD_F32 2    /* C(f32)  += A W^T + bias   (residual stream update)         */
#define RF_EPI_SWIGLU 3     /* C(bf16)[M, N/2] = silu(A W1^T) * (A W3^T); W rows interleaved
                               in 16-row groups [w1[16g:16g+16]; w3[16g:16g+16]]            */
#define RF_EPI_F16 4        /* C(fp16)  = A W^T + bias                                   */
#define RF_EPI_SWIGLU_F16 5 /* RF_EPI_SWIGLU with an fp16 C                               */

/* 16-bit element types of an output (the *_dt / _sk entry points) */
#define RF_DT_BF16 0
#define RF_DT_F16 1

const char* rf_last_error(void);
int rf_abi_version(void);
/* Build flags: RF_BUILD_STUDY set in the study build (librfhip_study.so: the measured-slower alternatives and
 * ablation variants -- legacy split-KV attention, the one-wave-per-SIMD attention, the 4-wave GEMM, the 4-wave
 * conv -- kept for A/B studies); the production librfhip.so refuses them with RF_ERR_UNSUPPORTED. */
#define RF_BUILD_STUDY 1
int rf_build_flags(void);

/* Device-side error word.  A stream-K owner (GEMM or attention) whose partner's partial does not arrive within
 * the spin bound (env RF_SPIN_LIMIT polls, default 2^24; code 1 GEMM, 2 attention), a stream-K launch handed a
 * range table that does not cover its tiles (code 3) or rf_scene_pos given a set above max_tris (code 4)
 * stores a non-zero code into a host-mapped word instead
 * of failing silently; from then on every entry point returns RF_ERR_DEVICE (checked without a device sync)
 * until rf_clear_device_error(); the outputs of the reporting launch are invalid and the stream-K workspaces
 * must be re-zeroed.  rf_debug_raise_device_error launches a kernel that stores `code` (tests). */
int rf_device_error(void);
int rf_clear_device_error(void);
/* fp16 range flag.  Every writer of fp16 operands (RF_EPI_F16 / RF_EPI_SWIGLU_F16 GEMM outputs, rf_rmsnorm_f16,
 * fp16 attention / Swin O, fp16 DPT planes of the convolutions and rf_split_planes) stores a non-zero code (1 GEMM,
 * 2 RMSNorm, 4 attention, 8 DPT plane) into a second host-mapped word when it meets a value beyond fp16's range
 * (|x| > 65504, inf included; NaN operands are not flagged): the values it wrote are inf.  Read with
 * rf_f16_range_flag() (no device sync: read it after the launches in question have completed), reset with
 * rf_clear_f16_range_flag().  The model re-renders such a frame with bf16 operands (RenderFormer.range_check). */
int rf_f16_range_flag(void);
int rf_clear_f16_range_flag(void);
/* Per-render fp16 range words (ABI 14): one word per frame, so concurrent renders (other streams, other models,
 * other threads) never clear or inherit each other's overflow.  rf_range_word_new(&handle) allocates a zeroed
 * host-mapped word; rf_range_word_bind(handle) makes it the word every fp16 writer launched from the CALLING THREAD
 * raises, until the next bind (NULL: back to the process-wide word above); rf_range_word_read(handle) returns its
 * code (>= 0) with a plain host load, no device sync (read it once the frame's launches have completed);
 * rf_range_word_clear(handle) zeroes it; rf_range_word_free(handle) releases it (no launch that may still write it
 * can be in flight).  NULL handles address the process-wide word.  The model takes one word per render
 * (RenderFormer.range_check) and checks it when the frame's end event has completed. */
int rf_range_word_new(void** handle);
int rf_range_word_bind(void* handle);
int rf_range_word_read(void* handle);
int rf_range_word_clear(void* handle);
int rf_range_word_free(void* handle);
int rf_debug_raise_device_error(int code, void* stream);

/* Kernel timer (measurement only; bench.py's roofline).  rf_ktimer_arm() creates a start/stop event pair on the
 * current device and arms it for the calling thread: the NEXT kernel the library launches (the first kernel
 * of the next entry-point call) is dispatched with hipExtLaunchKernel, whose dispatch packet timestamps the
 * pair — the kernel's own duration, as a rocprofv3 kernel trace reports it, with no marker packets around it.
 * rf_ktimer_read() waits for every taken pair, writes up to max_n durations (ms, launch order), releases the
 * pairs and returns how many were taken. */
int rf_ktimer_arm(void);
int rf_ktimer_read(float* ms, int max_n);

/* workspace / ws_bytes of the GEMM and convolution entry points: optional (NULL = one block per
 * output tile), rf_gemm_workspace_bytes() bytes, zero-filled once when allocated, used by one stream at a
 * time; with it, launches whose output tiles cannot fill the CUs split the K loop stream-K style. */
/* C[M,N] (epilogue) A[M,K] * W[N,K]^T ; A, W bf16; K % 32 == 0, N % 128 == 0, 16-B aligned rows.
 * Every epilogue runs on the hand-written MFMA engine (gemm.hip; no vendor GEMM library is linked): the
 * tile shape (256x256 / 128x256 / 96x256 / 64x256 phased, 96x256 / 128x128 ring) is chosen per shape by a
 * measured cost model; RF_EPI_ADD_F32 accumulators start from the C tile (no read-modify-write epilogue).
 * workspace (optional, NULL = data-parallel tiles only): rf_gemm_workspace_bytes() bytes, zero-filled once
 * when allocated, used by one stream at a time; it enables the stream-K split for GEMMs whose tile count
 * would leave CUs idle. */
int rf_gemm_bf16(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc,
                 const float* bias, int m, int n, int k, int epilogue, void* workspace, int64_t ws_bytes,
                 void* stream);
int64_t rf_gemm_workspace_bytes(void);
/* rf_gemm_bf16 with fp16 operands A, W (fp16 MFMAs, the bf16 rate; 11-bit mantissa: the model's default operand
 * format, 6-7x less rounding error than bf16 end to end).  Every epilogue of rf_gemm_bf16 (RF_EPI_BF16 still
 * writes bf16, e.g. q/k/v for the attention kernels); RF_EPI_F16 / RF_EPI_SWIGLU_F16 write fp16 (the operand of
 * the next fp16 GEMM), also from rf_gemm_bf16. */
int rf_gemm_f16(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc,
                const float* bias, int m, int n, int k, int epilogue, void* workspace, int64_t ws_bytes,
                void* stream);
/* Deferred RMSNorm (ABI 15): the pre-norm of a transformer layer folded into the GEMMs on either side of it, with
 * no row kernel in between.  rmsnorm(x) W^T = ((x * g) W^T) / rms(x) row by row, rms(x) = sqrt(mean(x^2) + eps), so
 *   - the producer, rf_gemm_add_prenorm, runs rf_gemm_*(RF_EPI_ADD_F32) (x += A W^T, x fp32 [M, N]) and from the
 *     same epilogue also writes xg = x * g (16-bit: fp16 when operand_dtype is RF_DT_F16, else bf16; [M, N],
 *     row stride ldxg) and per row up to RF_PRENORM_SLOTS partial sums of x^2 (ss: [M][RF_PRENORM_SLOTS] floats,
 *     16-B aligned; one slot per output-column tile, unused slots 0);
 *   - the consumer, rf_gemm_rownorm, is rf_gemm_*(epilogue) of A = xg whose output rows are scaled by
 *     1 / sqrt(sum of the row's slots / norm_dim + eps) before the bias and the SwiGLU (epilogue RF_EPI_BF16 /
 *     RF_EPI_F16 / RF_EPI_SWIGLU / RF_EPI_SWIGLU_F16).
 * rf_prenorm writes xg and ss (slot 0 = the whole row's sum) from x directly: the first layer's norm, whose x comes
 * from a kernel that is not a GEMM.  N <= RF_PRENORM_SLOTS * 128 for the fused producer; above it
 * rf_gemm_add_prenorm runs the GEMM and then rf_prenorm.  Replaces the pair rf_rmsnorm* + GEMM of
 * AttentionLayer.forward's pre-norms (renderformer/layers/attention.py:509, 520) and the decoder's (:634-661):
 * same values up to rounding (xg rounds x * g where rf_rmsnorm rounds x * g / rms(x); the same relative error),
 * the sums of squares in a fixed order (bit-reproducible).  An fp16 xg beyond 65504 raises range code 2. */
#define RF_PRENORM_SLOTS 8
int rf_prenorm(const float* x, int64_t ldx, const float* norm_w, void* xg, int64_t ldxg, float* ss, int rows,
               int dim, int operand_dtype, void* stream);
int rf_gemm_add_prenorm(const void* a, int64_t lda, const void* w, int64_t ldw, float* x, int64_t ldx, int m, int n,
                        int k, const float* norm_w, void* xg, int64_t ldxg, float* ss, int operand_dtype,
                        void* workspace, int64_t ws_bytes, void* stream);
/* seg_ss (optional, NULL = none; RF_EPI_BF16 / RF_EPI_F16 only): also the partial sums of the squares of the
 * written (rounded) outputs per row for each of the first n_seg segments of seg_w columns (seg_w % 256 == 0,
 * <= RF_PRENORM_SLOTS * 128), [M][n_seg][RF_PRENORM_SLOTS] floats — the row sums a following full-width RMSNorm
 * of those segments needs (the Swin q/k norm folded into rf_swin_attn_fwd_qkn). */
int rf_gemm_rownorm(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int m, int n,
                    int k, int epilogue, const float* ss, int norm_dim, float eps, float* seg_ss, int seg_w,
                    int n_seg, int operand_dtype, void* workspace, int64_t ws_bytes, void* stream);
/* Positional encoding fused into the QK path (ABI 16).  The q/k RMSNorm + rotary encoding of an attention
 * (attention.py:127-141 q_norm / k_norm then apply_rotary_emb_*cossin, rope.py:106-149) split where each part is
 * cheapest, with no pass over q:
 *   - rf_gemm_qk_rope: rf_gemm_rownorm(RF_EPI_BF16) of a projection whose first n_seg segments of seg_w columns
 *     are q (and k).  Their rows of W must be PERMUTED per 128-wide head so that column 2 m + t holds dimension
 *     m + 64 t (the rotate-half pairs (m, m + 64) side by side; q and k permuted alike, so q.k is unchanged).  The
 *     epilogue writes bf16 rope(norm_w * y) (norm_w in the same permuted order, NULL = no norm; segment 0 also
 *     times q_scale) with angle m = pos[r / pos_div][m / n_freqs] * freqs[m % n_freqs] for m < 9 n_freqs (else 0), and, when
 *     norm_w is given, seg_ss[r][seg][RF_PRENORM_SLOTS] = partial sums of y^2 (y before the weight and rotation,
 *     f32) — the norm's 1 / rms is applied downstream (RoPE and the weight are linear per row).  ss / norm_dim /
 *     eps: the deferred pre-norm, as rf_gemm_rownorm (ss NULL: none).
 *   - rf_row_rms_scale: x[r] *= scale / sqrt(sum of ss[r * ld_ss + 0..7] / dim + eps) in place (bf16): the keys.
 *   - rf_attn_fwd_qn: rf_attn_fwd_dt (bf16 q/k/v) whose q rows are multiplied by q_scale / sqrt(sum of q_ss[r *
 *     ld_ss + 0..7] / q_dim + eps) as the stream-K kernel loads them (q_scale = softmax_scale * log2 e: the kernel
 *     runs on exp2 exponents). */
int rf_gemm_qk_rope(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int m, int n,
                    int k, const float* ss, int norm_dim, float eps, float* seg_ss, int seg_w, int n_seg,
                    const float* norm_w, const float* pos, int64_t ld_pos, int pos_div, const float* freqs,
                    int n_freqs, float q_scale, int operand_dtype, void* workspace, int64_t ws_bytes, void* stream);
int rf_row_rms_scale(void* x, int64_t ldx, int rows, int dim, const float* ss, int64_t ld_ss, float eps, float scale,
                     void* stream);
int rf_attn_fwd_qn(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv, void* o,
                   int64_t ldo, int o_dtype, const float* q_ss, int64_t ld_ss, int q_dim, float eps, float q_scale,
                   const int32_t* problems, int n_problems, int n_heads, int head_dim, void* workspace,
                   const int64_t* bounds, int grid, void* stream);
/* rf_gemm_bf16 on the HIP engine that does nothing unless *flag != 0 (read on the device when the launch
 * runs); stream-ordered after whatever wrote the flag. */
int rf_gemm_bf16_if(const int* flag, const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc,
                    const float* bias, int m, int n, int k, int epilogue, void* workspace, int64_t ws_bytes,
                    void* stream);

/* MX fp8 GEMM: C[M,N] (epilogue) A[M,K] * W[N,K]^T with OCP e4m3 operands (bytes, row strides lda/ldw in
 * bytes) and one E8M0 scale byte per 32 K-elements of every row (sa [M][ld_sa], sw [N][ld_sw]; value =
 * e4m3 * 2^(scale - 127)), fp32 accumulation on v_mfma_scale_f32_16x16x128_f8f6f4.  K % 128 == 0, N % 256 == 0.
 * Same epilogues as rf_gemm_bf16 (RF_EPI_ADD_F32 accumulates into C).  The stage-2 fp8 mode of the model
 * (RenderFormer(fp8=True)) runs its projections through this. */
int rf_gemm_mx8(const void* a, int64_t lda, const void* sa, int64_t ld_sa, const void* w, int64_t ldw, const void* sw,
                int64_t ld_sw, void* c, int64_t ldc, const float* bias, int m, int n, int k, int epilogue,
                void* stream);
/* bf16 rows x[rows][cols] -> e4m3 q[rows][ldq] + E8M0 scales[rows][ld_s] per 32-element block: scale
 * 2^ceil(log2(amax / 448)) (no saturation), round to nearest even. */
int rf_quant_mx8(const void* x, int64_t ldx, int rows, int cols, void* q, int64_t ldq, void* scales, int64_t ld_s,
                 void* stream);

/* out(bf16)[r, :] = x[r, :] * rsqrt(mean(x^2) + eps) * weight ; x f32. */
int rf_rmsnorm(const float* x, int64_t ldx, const float* weight, float eps, void* out, int64_t ldo,
               int rows, int dim, void* stream);
/* rf_rmsnorm with an fp16 out (the A operand of rf_gemm_f16). */
int rf_rmsnorm_f16(const float* x, int64_t ldx, const float* weight, float eps, void* out, int64_t ldo,
                   int rows, int dim, void* stream);

/* dst[r] = rope(rmsnorm(src[src_rows ? src_rows[r] : r]))  (bf16 -> bf16, may alias when src_rows == NULL)
 * over n_seg consecutive segments of width dim (q and k of one qkv row), each with its own full-width
 * RMSNorm weights norm_w[seg*dim ...] (norm_w may be NULL: no norm); pos may be NULL (no rope).
 * Segment 0 is additionally multiplied by seg0_scale (1 = none): passing softmax_scale * log2(e) for
 * the q segment lets rf_attn_fwd run with scale = ln 2 (no per-score multiply).
 * RoPE: head_dim 128, per head the half-split rotation with
 * angle[i] = pos[r / pos_div][i / n_freqs] * freqs[i % n_freqs] for i < 9*n_freqs, else 0. */
int rf_qk_norm_rope(const void* src, int64_t ld_src, void* dst, int64_t ld_dst, const int32_t* src_rows,
                    int rows, int dim, int n_heads, int n_seg, const float* norm_w, float eps, float seg0_scale,
                    const float* pos, int64_t ld_pos, int pos_div, const float* freqs, int n_freqs, void* stream);

/* rf_qk_norm_rope over n_groups column groups of the same rows in one launch: group g reads
 * src + g*src_gstride, writes dst + g*dst_gstride (elements) and uses norm_w + g*w_gstride; the rows,
 * src_rows and RoPE positions are shared.  The decoder's cross-attention keys of every layer
 * (attention.py:127-141 applied to the k projection of each decoder layer, with that layer's k_norm)
 * are rotated this way in one pass over the batched K/V projection.  Offsets must keep 16-B alignment. */
int rf_qk_norm_rope_groups(const void* src, int64_t ld_src, int64_t src_gstride, void* dst, int64_t ld_dst,
                           int64_t dst_gstride, const int32_t* src_rows, int rows, int dim, int n_heads, int n_seg,
                           int n_groups, const float* norm_w, int64_t w_gstride, float eps, float seg0_scale,
                           const float* pos, int64_t ld_pos, int pos_div, const float* freqs, int n_freqs,
                           void* stream);
/* rf_qk_norm_rope_groups on rows in rf_gemm_qk_rope's pair-interleaved column order (ABI 16): per head, column 2 m + t
 * is dimension m + 64 t, norm_w in the same order; the same angles and arithmetic (the stage-2 keys when the queries'
 * rotation runs in their projection's epilogue). */
int rf_qk_norm_rope_groups_ilv(const void* src, int64_t ld_src, int64_t src_gstride, void* dst, int64_t ld_dst,
                               int64_t dst_gstride, const int32_t* src_rows, int rows, int dim, int n_heads, int n_seg,
                               int n_groups, const float* norm_w, int64_t w_gstride, float eps, float seg0_scale,
                               const float* pos, int64_t ld_pos, int pos_div, const float* freqs, int n_freqs,
                               void* stream);

/* Variable-length multi-head attention, non-causal, head_dim 128, bf16 in/out, f32 softmax.
 * problems: int32[n_problems][5] = {q_start, q_len, k_start, k_len, v_start} (rows); k_len >= 1
 * wherever q_len >= 1.  For every problem p and head h: O[q_start+i, h*128:(h+1)*128] =
 *   softmax(scale * Q_i K_j^T, j < k_len) V_j .
 * scale = ln 2 means q already carries softmax_scale * log2(e) (rf_qk_norm_rope seg0_scale): the
 * scores are then used as exp2 exponents directly.
 * n_split == 0 (default mode): stream-K kernel, one workgroup per CU over the flattened
 *   (problem, head, 256-row block, 64-key tile) space; `workspace` = rf_attn_workspace_bytes(0, H, 0)
 *   bytes, ZEROED before its first use and reused as is afterwards (every launch uses fresh hand-off flag
 *   values); one launch at a time per workspace.  ws_rows is ignored.  Forward progress: a workgroup that
 *   merges a cut unit waits only on workgroups with a lower blockIdx (dispatched earlier) whose awaited piece
 *   is the first of their range, so launches drain with no co-residency assumption (two streams at once).
 * n_split >= 1: one workgroup per (problem, head, block, split); for n_split > 1 partials go to
 *   `workspace` (rf_attn_workspace_bytes(ws_rows, n_heads, n_split) bytes, ws_rows >= every output
 *   row + 1) and rf_attn_combine(rows = NULL, n_rows = ws_rows) writes O. */
int rf_attn_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                void* o, int64_t ldo, const int32_t* problems, int n_problems, int max_q_len, int n_heads,
                int head_dim, float scale, int n_split, void* workspace, int64_t ws_rows, void* stream);
int64_t rf_attn_workspace_bytes(int64_t rows, int n_heads, int n_split);
/* Cost-balanced stream-K ranges for the n_split == 0 kernel (host function, no device work): from the
 * HOST copy of `problems`, bounds[0..grid] (int64) = the first tile of each workgroup's range over the
 * flattened (problem, head, 256-row block, 64-key tile) space, chosen so every workgroup's prologues,
 * tiles, partial publishes and merges end together (equal tile counts leave the owners of units cut
 * three ways last).  grid = rf_attn_grid() (the device's CU count) for rf_attn_fwd_sched.
 * Replaces nothing in the reference (flash_attn schedules internally); a plan-time companion of
 * rf_attn_fwd, computed once per mask pattern like the problems table itself. */
int rf_attn_grid(void);
int rf_attn_schedule(const int32_t* problems_host, int n_problems, int n_heads, int grid, int64_t* bounds);
/* rf_attn_fwd (n_split == 0) with the workgroup ranges taken from `bounds` (device copy of the
 * rf_attn_schedule result; the grid is `grid` workgroups).  Same results up to the fp32 merge order.
 * The kernel checks the table against its own problems (bounds[0] == 0, monotone, bounds[grid] == the
 * launch's tile count, no unit across an XCD group) and reports RF_ERR_DEVICE (device error 3) instead of
 * reading past the problems when a table built for another launch is passed. */
int rf_attn_fwd_sched(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                      void* o, int64_t ldo, const int32_t* problems, int n_problems, int n_heads, int head_dim,
                      float scale, void* workspace, const int64_t* bounds, int grid, void* stream);
int rf_attn_combine(const void* workspace, int64_t ws_rows, int n_split, int n_heads, const int32_t* rows,
                    int n_rows, void* o, int64_t ldo, void* stream);
/* The stream-K attention (rf_attn_fwd_sched, or rf_attn_fwd n_split == 0 when bounds == NULL) with O written as
 * o_dtype: RF_DT_F16 when O is the A operand of an fp16 out-projection (rf_gemm_f16); q/k/v stay bf16. */
int rf_attn_fwd_sk(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                   void* o, int64_t ldo, int o_dtype, const int32_t* problems, int n_problems, int n_heads,
                   int head_dim, float scale, void* workspace, const int64_t* bounds, int grid, void* stream);
/* The stream-K attention with the q/k/v element type as an argument: qkv_dtype RF_DT_F16 runs fp16 operands on
 * v_mfma_f32_32x32x16_f16 (the bf16 rate; P is fp16 too), RF_DT_BF16 the bf16 kernel; O is o_dtype.  Replaces
 * flash_attn_varlen_qkvpacked_func / flash_attn_varlen_kvpacked_func (renderformer/layers/attention.py:166-172,
 * 193-195) for EITHER half type the reference hands them: its default torch_dtype=torch.float16
 * (rendering_pipeline.py:37, infer.py:37, batch_infer.py:65) makes q/k/v fp16, bf16 runs make them bf16.  bounds
 * NULL = equal ranges (then grid is ignored), else an rf_attn_schedule table for `grid` workgroups. */
int rf_attn_fwd_dt(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                   void* o, int64_t ldo, int qkv_dtype, int o_dtype, const int32_t* problems, int n_problems,
                   int n_heads, int head_dim, float scale, void* workspace, const int64_t* bounds, int grid,
                   void* stream);

/* Shifted-window attention over n_images patch grids [grid_h, grid_w] stored row-major (token
 * r = img*gh*gw + y*gw + x); windows of window x window tokens on the grid rolled by -shift,
 * Swin region mask when shift > 0.  Output written back to the un-rolled token positions. */
int rf_swin_attn_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                     void* o, int64_t ldo, int n_images, int grid_h, int grid_w, int window, int shift,
                     int n_heads, int head_dim, float scale, void* stream);
/* rf_swin_attn_fwd with O written as o_dtype (RF_DT_BF16 / RF_DT_F16). */
int rf_swin_attn_fwd_dt(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                        void* o, int64_t ldo, int o_dtype, int n_images, int grid_h, int grid_w, int window, int shift,
                        int n_heads, int head_dim, float scale, void* stream);
/* rf_swin_attn_fwd_dt with the full-width q/k RMSNorm folded into its loads (ABI 15): q, k as the projection wrote
 * them (rf_gemm_rownorm with seg_ss = qk_ss, seg_w = n_heads * 128, n_seg = 2), each q row scaled by
 * q_scale / rms(q row) * qk_norm_w[c] and each k row by 1 / rms(k row) * qk_norm_w[n_heads * 128 + c] before the
 * scores -- rf_qk_norm_rope(n_seg = 2, no RoPE, seg0_scale = q_scale)'s arithmetic without its pass over q and k
 * (reference SwinSelfAttention q/k norm, attention.py:345-359).  qk_norm_w and qk_ss are required (a model without q/k
 * norm weights runs rf_qk_norm_rope's scale-only form and rf_swin_attn_fwd_dt). */
int rf_swin_attn_fwd_qkn(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv, void* o,
                         int64_t ldo, int o_dtype, int n_images, int grid_h, int grid_w, int window, int shift,
                         int n_heads, int head_dim, float scale, const float* qk_ss, const float* qk_norm_w, float eps,
                         float q_scale, void* stream);

/* texture: f32 [n_rows, channels, patch_elems]; channels >= channels-log_channels are log10(x+1)
 * encoded IN PLACE for every row; rows with dst_row[r] >= 0 are written as bf16 to out[dst_row[r]]. */
int rf_texture_pack(float* texture, int64_t n_rows, int channels, int patch_elems, int log_channels,
                    const int32_t* dst_row, void* out, int64_t ldo, void* stream);
/* rf_texture_pack that does nothing unless *flag != 0. */
int rf_texture_pack_if(const int* flag, float* texture, int64_t n_rows, int channels, int patch_elems,
                       int log_channels, const int32_t* dst_row, void* out, int64_t ldo, void* stream);
/* One pass over texture f32 [n_rows, channels, 1024] (32x32 patches, channels <= 32): zeroes *flag, then
 * log10(x+1)-encodes channels >= channels-log_channels IN PLACE for every row (as rf_texture_pack), and for
 * rows with dst_row[r] >= 0 writes coef[dst_row[r]*ldc + c] = the row's channel-c constant and sets
 * *flag = 1 unless every texel equals that constant inside the to_h5 patch mask {(i, j): i + j <= 32}
 * (row-major i, j) and 0 outside it (exact compares; NaN fails). */
int rf_texture_scan(float* texture, int64_t n_rows, int channels, int patch_elems, int log_channels,
                    const int32_t* dst_row, float* coef, int64_t ldc, int* flag, void* stream);
/* rf_texture_scan with no reset launch: *flag must be 0 on entry and the kernel zeroes *flag_clear (a second
 * flag): alternating two flags by frame parity, frame i raises flags[i % 2] and clears flags[(i + 1) % 2]
 * (the reset otherwise costs a hipMemsetAsync blit kernel per frame).  n_rows >= 1. */
int rf_texture_scan2(float* texture, int64_t n_rows, int channels, int patch_elems, int log_channels,
                     const int32_t* dst_row, float* coef, int64_t ldc, int* flag, int* flag_clear, void* stream);
/* When *flag == 0: out f32 [rows, n] = bias + coef[rows, channels] * wsum[channels, n], with
 * wsum[c, o] = sum over the patch mask of W[o, c*1024 + e] (the texture Linear on scanned rows);
 * no-op otherwise.  channels <= 16, n % 4 == 0, 16-B aligned out/wsum/bias (bias may be NULL). */
int rf_texture_linear(const float* coef, int64_t ldc, int rows, int channels, const float* wsum,
                      const float* bias, float* out, int64_t ldo, int n, const int* flag, void* stream);

/* NeRF encoding (include_input) of vn f32 [n_rows, 9] into bf16 out[dst_row[r], 0:ldo] (zero padded). */
int rf_vn_encode(const float* vn, int64_t n_rows, const int32_t* dst_row, int n_freqs, void* out,
                 int64_t ldo, void* stream);
/* rf_vn_encode with out written as out_dtype (RF_DT_BF16 / RF_DT_F16: the operand of an fp16 GEMM). */
int rf_vn_encode_dt(const float* vn, int64_t n_rows, const int32_t* dst_row, int n_freqs, void* out,
                    int64_t ldo, int out_dtype, void* stream);

/* Pinhole rays for n_views cameras (c2w f32 [n_views,4,4], fov degrees [n_views]) at res x res,
 * normalised, patchified into bf16 tokens out[view*R + t, c*patch*patch + p1*patch + p2];
 * ray_pos[view, 9] = camera origin repeated 3x. */
int rf_ray_tokens(const float* c2w, const float* fov_deg, int n_views, int res, int patch, void* out,
                  float* ray_pos, void* stream);
/* rf_ray_tokens with out written as out_dtype (RF_DT_BF16 / RF_DT_F16). */
int rf_ray_tokens_dt(const float* c2w, const float* fov_deg, int n_views, int res, int patch, void* out,
                     float* ray_pos, int out_dtype, void* stream);

/* rays_d f32 [n_views, res, res, 3] (already generated) -> the same bf16 token layout as rf_ray_tokens. */
int rf_patchify_rays(const float* rays_d, int n_views, int res, int patch, void* out, void* stream);
/* rf_patchify_rays with out written as out_dtype (RF_DT_BF16 / RF_DT_F16). */
int rf_patchify_rays_dt(const float* rays_d, int n_views, int res, int patch, void* out, int out_dtype,
                        void* stream);

/* Triangle positions for RoPE.  tris f32 [*, 9]; valid_idx int32 [sum n_b] (rows into tris, grouped by
 * scene, offsets scene_off[B+1]).  For each set s (s = b when c2w == NULL, else s = b*n_views + v with the
 * camera transform p -> R^T (p - t)), writes n_reg centre rows then the n_b triangle rows to
 * pos_out[set_off[s] ...].  max_tris >= every n_b; partials: rf_scene_pos_partials(sets, max_tris) floats of
 * caller workspace (per-256-triangle sums, reduced in a fixed order: deterministic).  A set with n_b > max_tris
 * (the kernel sees scene_off on the device only) is clamped to its own partial slots and raises device error 4
 * (RF_ERR_DEVICE from the next call; its positions past ceil(max_tris/256)*256 are not written). */
int rf_scene_pos(const float* tris, const int32_t* valid_idx, const int32_t* scene_off, const float* c2w,
                 int n_scenes, int n_views, int n_reg, float* pos_out, const int32_t* set_off, int max_tris,
                 float* partials, int64_t partial_floats, void* stream);
int64_t rf_scene_pos_partials(int sets, int max_tris);

/* out[out_rows[r]] = base[r % base_rows] + sum_t rmsnorm(in_t[r]) * w_t   (f32; in_t / w_t may be NULL). */
int rf_embed(float* out, int64_t ldo, const int32_t* out_rows, int rows, int dim, const float* base,
             int base_rows, const float* in0, int64_t ld0, const float* w0, float eps0, const float* in1,
             int64_t ld1, const float* w1, float eps1, void* stream);

/* out = decode(elu(logits f32 [n, c, h, w], alpha)), decode = 10^x - 1 if log_decode; out is laid out
 * [n, h, w, c] when channels_last, else [n, c, h, w]. */
int rf_hdr_output(const float* logits, float* out, int n, int c, int h, int w, float elu_alpha, int log_decode,
                  int channels_last, void* stream);

/* DPT convolutions on the GEMM engine.  Activations are NHWC; a convolution reads its input as two
 * bf16 planes (hi = bf16(x), lo = bf16(x - hi); channel stride cin_pad, padded channels zero) and its
 * weights as bf16 hi/lo [cout_pad][kh][kw][cin_pad]; products are hi*hi + hi*lo + lo*hi with fp32
 * accumulation.  Epilogue: v = conv + bias + res1 + res2 (f32 NHWC, channel stride cout), then silu if
 * RF_CONV_SILU_OUT; v is stored to `out` (f32, may be NULL) and/or split into the output planes
 * p_hi/p_lo (channel stride p_ld), of silu(v) when RF_CONV_PLANE_SILU.
 * RF_CONV_FINAL (cout <= 64): out[pixel, f] = elu(sum_c silu(v_c) * w_fin[f, c] + b_fin[f], alpha),
 * then 10^x - 1 with RF_CONV_LOG_DECODE; [n, n_fin, h, w] layout with RF_CONV_NCHW_OUT.
 * RF_CONV_BORDER_BIAS (3x3, pad 1, stride 1, images of at least 2 x 2 pixels): `bias` holds 9 rows of cout, row 3 ry + rx with ry / rx = 0 on the
 * first image row / column, 2 on the last, 1 elsewhere: the bias of a convolution whose input carried a constant
 * that zero padding cuts at the border (an affine 1x1 folded into the 3x3 weights, dpt.py output_conv1). */
#define RF_CONV_PLANE_SILU 1
#define RF_CONV_SILU_OUT 2
#define RF_CONV_FINAL 4
#define RF_CONV_LOG_DECODE 8
#define RF_CONV_NCHW_OUT 16
#define RF_CONV_BORDER_BIAS 32
int rf_conv2d_bf16x3(const void* in_hi, const void* in_lo, int n_img, int hi, int wi, int cin_pad, const void* w_hi,
                     const void* w_lo, int cout, int cout_pad, int kh, int kw, int stride, int pad, const float* bias,
                     const float* res1, const float* res2, float* out, void* p_hi, void* p_lo, int p_ld, int flags,
                     const float* w_fin, const float* b_fin, int n_fin, float elu_alpha, void* workspace,
                     int64_t ws_bytes, void* stream);

/* ConvTranspose2d with kernel == stride == k: out[n, k y + dy, k x + dx, co] = sum_ci in[n, y, x, ci] *
 * W[ci, co, dy, dx] + bias[co]; input planes as above, weights bf16 hi/lo [(dy, dx, co)][cin_pad]. */
int rf_deconv2d_bf16x3(const void* in_hi, const void* in_lo, int n_img, int hi, int wi, int cin_pad, const void* w_hi,
                       const void* w_lo, int cout, int k, const float* bias, float* out, void* p_hi, void* p_lo,
                       int p_ld, void* workspace, int64_t ws_bytes, void* stream);

/* fp16-operand variants: one fp16 input plane (channel stride cin_pad), fp16 weights [cout_pad][kh][kw][cin_pad],
 * one MFMA per product with fp32 accumulation (11-bit operand mantissa: 9e-5 relative L2 on the large-proxy
 * DPT against 7e-4 for bf16 operands).  Same epilogue as above; the output plane p_out (may be NULL) is one
 * fp16 plane.  Values beyond fp16 range (|x| > 65504) become inf in the planes.  cout_pad: 64 (cout <= 64)
 * or a multiple of 128. */
int rf_conv2d_f16(const void* in, int n_img, int hi, int wi, int cin_pad, const void* w, int cout, int cout_pad, int kh,
                  int kw, int stride, int pad, const float* bias, const float* res1, const float* res2, float* out,
                  void* p_out, int p_ld, int flags, const float* w_fin, const float* b_fin, int n_fin, float elu_alpha,
                  void* workspace, int64_t ws_bytes, void* stream);
/* Up to 4 independent fp16 convolutions / deconvolutions (kernel == stride) as ONE launch on the 128 x 128
 * tile: the DPT's resize layers (dpt.py:195-216) and its layer*_rn convolutions (dpt.py:228-231), whose 64^2 /
 * 32^2 launches are latency-bound.  Member q is what rf_conv2d_f16 (deconv_k == 0: in, n_img, hi, wi, cin_pad,
 * w, cout, cout_pad, kh, kw, stride, pad, bias, out, p_out, p_ld, flags) or rf_deconv2d_f16 (deconv_k = k;
 * cout_pad, kh, kw, stride, pad and flags unused) computes, except RF_CONV_FINAL; output channels (cout_pad, or
 * k*k*cout) a multiple of 128. */
typedef struct {
    const void* in;
    const void* w;
    const float* bias;
    float* out;
    void* p_out;
    int n_img, hi, wi, cin_pad, cout, cout_pad, kh, kw, stride, pad, deconv_k, p_ld, flags;
} rf_conv_desc;
int rf_conv2d_f16_group(int n_conv, const rf_conv_desc* convs, void* stream);

/* Up to 4 independent 1x1 fp16 convolutions over images of the same n_img x hi x wi (the DPT's four tap
 * projections, dpt.py:197-199 / 244-249) in ONE launch: conv q reads in[q] (channel stride cin_pad[q]) and
 * writes out plane p_out[q] (channel stride p_ld[q]) = in . W_q^T + bias[q] (bias may be NULL, or any entry);
 * W_q fp16 [cout_pad[q]][cin_pad[q]], cout_pad a multiple of 128.  Same results as rf_conv2d_f16 per conv. */
int rf_conv1x1_f16_group(int n_conv, const void* const* in, const int* cin_pad, const void* const* w, const int* cout,
                         const int* cout_pad, const float* const* bias, void* const* p_out, const int* p_ld, int n_img,
                         int hi, int wi, void* stream);
int rf_deconv2d_f16(const void* in, int n_img, int hi, int wi, int cin_pad, const void* w, int cout, int k,
                    const float* bias, float* out, void* p_out, int p_ld, void* workspace, int64_t ws_bytes,
                    void* stream);

/* f32 rows x[r, 0:c] (row stride ldx) -> bf16 hi/lo planes (row stride p_ld), of silu(x) if silu_act.
 * p_lo == NULL: one fp16 plane in p_hi instead (input of rf_conv2d_f16 / rf_deconv2d_f16). */
int rf_split_planes(const float* x, int64_t rows, int c, int64_t ldx, void* p_hi, void* p_lo, int p_ld, int silu_act,
                    void* stream);

/* Bilinear resize, align_corners=True, NHWC fp32 (c % 4 == 0) into `out` and/or hi/lo planes
 * (p_lo == NULL: one fp16 plane, as rf_split_planes). */
int rf_upsample_bilinear(const float* in, int n_img, int hi, int wi, int c, float* out, int ho, int wo, void* p_hi,
                         void* p_lo, int p_ld, void* stream);

/* The same resize from one fp16 plane (channel stride in_ld, c % 8 == 0) into one fp16 plane (channel stride
 * p_ld): values widened to f32, blended as rf_upsample_bilinear, rounded once (F.interpolate of the plane's
 * values; dpt.py:268-271 with output_conv1's preceding 1x1 folded into its weights). */
int rf_upsample_bilinear_h(const void* in, int in_ld, int n_img, int hi, int wi, int c, int ho, int wo, void* p_out,
                           int p_ld, void* stream);

/* ---------------------------------------------------------------------------------------------------------------
 * Stage-level entry points: a whole transformer stack in one call (stage.cpp: host code that issues the unit entry
 * points above in the order the Python model does, so results are bit-identical to it).  Weight pointers are device
 * pointers in the operand type (RF_DT_F16 or RF_DT_BF16 = the model's `operands`), norm weights f32.  The struct
 * arrays themselves live in host memory.  Workspaces are caller-owned: `workspace` holds the stack's activations
 * (rf_*_workspace_bytes), gemm_ws / attn_ws are the GEMM / stream-K attention workspaces of the unit entry points.
 * --------------------------------------------------------------------------------------------------------------- */

/* One layer of TransformerEncoder (renderformer/layers/attention.py:579-590 -> AttentionLayer.forward :484-527,
 * MultiHeadAttention :115-202, FeedForwardSwiGLU :51-57). */
typedef struct {
    const float* attn_norm;  /* [D]   pre-norm of the attention block (norm1) */
    const void* w_qkv;       /* [3D, D] in-projection, rows q | k | v */
    const float* qk_norm;    /* [2D]  full-width q then k RMSNorm weights, or NULL (no q/k norm) */
    const void* w_out;       /* [D, D] out-projection */
    const float* ffn_norm;   /* [D]   pre-norm of the FFN block (norm2) */
    const void* w13;         /* [2F, D] w1 / w3 interleaved in 16-row groups (RF_EPI_SWIGLU layout) */
    const void* w2;          /* [D, F] */
} rf_encoder_layer;

typedef struct {
    int n_layers, rows, dim, n_heads, ffn_dim;  /* rows = packed tokens of the batch (registers + triangles) */
    int operand_dtype;                          /* RF_DT_F16 / RF_DT_BF16: weights and GEMM operands */
    float eps;                                  /* RMSNorm eps (1e-6) */
    const rf_encoder_layer* layers;             /* host array [n_layers] */
    const float* pos;                           /* [rows, 9] triangle vertex positions (RoPE), NULL = no RoPE */
    int64_t ld_pos;
    const float* freqs;                         /* RoPE frequencies [n_freqs] (rope.py:152-206) */
    int n_freqs;
    const int32_t* problems;                    /* device [n_problems][5] attention units (rf_attn_fwd), one per scene */
    int n_problems;
    const int64_t* bounds;                      /* rf_attn_schedule table (device) for `grid` workgroups, or NULL */
    int grid;
    void* workspace;                            /* rf_encoder_workspace_bytes() bytes (activations; no zeroing) */
    void* gemm_ws;                              /* rf_gemm_workspace_bytes() bytes, zeroed once (may be NULL) */
    int64_t gemm_ws_bytes;
    void* attn_ws;                              /* rf_attn_workspace_bytes(0, H, 0) bytes, zeroed once */
    int timer_attn;                             /* measurement: rf_ktimer_arm() before every attention launch */
    int qk_fused;                               /* 1: every layer's w_qkv q/k rows and qk_norm are in rf_gemm_qk_rope's
                                                   pair-interleaved order and the positional encoding runs fused into
                                                   the QK path (rf_gemm_qk_rope + rf_row_rms_scale + rf_attn_fwd_qn);
                                                   0: the standard layout (rf_gemm_rownorm + rf_qk_norm_rope) */
} rf_encoder_desc;

/* x[rows, dim] (f32 residual stream, row stride ldx) through the encoder stack in place: per layer
 * x += W_out attn(rope(qk_norm(W_qkv rmsnorm(x)))) ; x += W2 swiglu(W13 rmsnorm(x)).  Replaces
 * TransformerEncoder.forward (attention.py:579-590) on the packed, unpadded rows.  dim = n_heads * 128. */
int rf_encoder_forward(float* x, int64_t ldx, const rf_encoder_desc* desc, void* stream);
int64_t rf_encoder_workspace_bytes(int rows, int dim, int ffn_dim, int operand_dtype);

/* One layer of TransformerDecoder (attention.py:673-688 -> AttentionLayer.forward :484-527 with cross-attention,
 * :436-482): cross-attention rays -> triangles, self-attention between ray tokens (Swin windows :316-370 or full),
 * SwiGLU FFN, each pre-norm and residual. */
typedef struct {
    const float* query_norm;   /* [D] pre-norm of the cross-attention block */
    const void* w_q;           /* [D, D] */
    const float* q_norm;       /* [D] full-width q RMSNorm, or NULL */
    const float* kv_norm;      /* [Dc] context norm (per-layer K/V form only; unused with w_kv_all) */
    const void* w_kv;          /* [2D, Dc] K rows then V rows (per-layer K/V form only) */
    const float* k_norm;       /* [D] full-width k RMSNorm, or NULL (per-layer key form only) */
    const void* w_out;         /* [D, D] */
    const float* self_norm;    /* [D] pre-norm of the self-attention block; NULL = no self-attention */
    const void* w_self_in;     /* [3D, D] */
    const float* self_qk_norm; /* [2D] or NULL */
    const void* w_self_out;    /* [D, D] */
    const float* ffn_norm;     /* [D] */
    const void* w13;           /* [2F, D] (RF_EPI_SWIGLU layout) */
    const void* w2;            /* [D, F] */
} rf_decoder_layer;

/* A decoder output handed to the DPT head (view_transformer.py:85 out_layers): after layer `layer`, x is written
 * as operand planes (rf_split_planes: p_lo NULL = one fp16 plane) with channel stride p_ld. */
typedef struct {
    int layer, p_ld;
    void* p_hi;
    void* p_lo;
} rf_decoder_tap;

typedef struct {
    int n_layers, rows, dim, n_heads, ffn_dim;  /* rows = ray tokens of all (scene, view) images */
    int operand_dtype;
    float eps;
    const rf_decoder_layer* layers;             /* host array [n_layers] */
    /* context (the stage-1 output) and its K/V: one GEMM for every layer when w_kv_all != NULL (rows of layer i:
       K then V at 2*D*i; ctx_norm = unit weights, each layer's kv_norm folded into its rows), else per layer */
    const float* ctx;
    int64_t ld_ctx;
    int ctx_rows, ctx_dim;
    const float* ctx_norm;
    const void* w_kv_all;
    /* keys of each view: row r of the rotated keys reads context row kv_src_rows[r] with camera-frame triangle
       position kv_pos[r]; k_batch = 1 rotates every layer's keys in one launch (needs w_kv_all; k_norm_all =
       [n_layers * D] or NULL) */
    int kv_rows;
    const int32_t* kv_src_rows;
    const float* kv_pos;
    int64_t ld_kv_pos;
    int k_batch;
    const float* k_norm_all;
    const float* freqs;                         /* RoPE frequencies [n_freqs] */
    int n_freqs;
    const float* ray_pos;                       /* [images, 9] ray-origin positions, one per image (row / ray_pos_div) */
    int64_t ld_ray_pos;
    int ray_pos_div;                            /* ray tokens per image */
    const int32_t* cross_problems;              /* device [n_cross][5]: (q rows of an image, its scene's keys) */
    int n_cross;
    const int64_t* cross_bounds;                /* rf_attn_schedule table or NULL */
    int cross_grid;
    /* self-attention: Swin windows (swin = 1; shift on odd layers) or full attention over self_problems */
    int swin, n_images, grid_h, grid_w, window, shift;
    const int32_t* self_problems;
    int n_self;
    const rf_decoder_tap* taps;                 /* host array [n_taps], in layer order */
    int n_taps;
    void* workspace;                            /* rf_decoder_workspace_bytes(desc) bytes */
    void* gemm_ws;
    int64_t gemm_ws_bytes;
    void* attn_ws;
    int timer_cross;                            /* measurement: rf_ktimer_arm() before every cross-attention launch */
    int qk_fused;                               /* 1: w_q rows, q_norm, the K rows of w_kv / w_kv_all, k_norm and
                                                   k_norm_all in rf_gemm_qk_rope's pair-interleaved order: the query
                                                   rotation runs in the projection's epilogue (rf_gemm_qk_rope), the
                                                   keys' in rf_qk_norm_rope_groups_ilv, q's 1 / rms in rf_attn_fwd_qn */
} rf_decoder_desc;

/* x[rows, dim] (f32 ray-token residual stream) through the decoder stack in place; the DPT taps are written as
 * they are produced.  Replaces TransformerDecoder.forward (attention.py:673-688) on packed rows. */
int rf_decoder_forward(float* x, int64_t ldx, const rf_decoder_desc* desc, void* stream);
int64_t rf_decoder_workspace_bytes(const rf_decoder_desc* desc);

#ifdef __cplusplus
}
#endif
#endif /* RF_H */
