// Stage-level entry points: a whole transformer stack per call.
//
// rf_encoder_forward replaces TransformerEncoder.forward (renderformer/layers/attention.py:579-590), i.e. per layer
// AttentionLayer.forward (:484-527): pre-norm multi-head self-attention with full-width q/k RMSNorm and the
// triangle RoPE (MultiHeadAttention :115-202, rope.py:106-149) and the SwiGLU FFN (:51-57), both residual.  It is
// host code only: it issues the library's own unit entry points (rf_prenorm, rf_gemm_add_prenorm, rf_gemm_rownorm,
// rf_gemm_*, rf_qk_norm_rope, rf_attn_fwd_dt, or with qk_fused rf_gemm_qk_rope, rf_row_rms_scale, rf_attn_fwd_qn) on
// the caller's stream in exactly the order model.py::_stage1 does,
// so a stack run through here is bit-identical to the Python-orchestrated one, with one C call instead of 7 per
// layer from Python.  The pre-norms are deferred (rf.h): no RMSNorm row kernel after layer 0's first one.
#include <hip/hip_runtime.h>

#include <cmath>

#include "common.h"

namespace {
constexpr int64_t kAlign = 256;
int64_t align_up(int64_t b) { return (b + kAlign - 1) / kAlign * kAlign; }

// activation buffers of the encoder stack, carved from one caller-owned workspace
struct EncBufs {
    // byte offsets: h [T, D] half (x * g of the deferred RMSNorm), qkv [T, 3D] bf16, att [T, D] half, g [T, F] half,
    // ss [T, RF_PRENORM_SLOTS] f32 (the norm's partial sums of squares), qkss [T, 2, RF_PRENORM_SLOTS] f32 (the
    // fused QK path's q / k partial sums of squares, rf_gemm_qk_rope)
    int64_t h, qkv, att, g, ss, qkss, total;
};
EncBufs enc_layout(int rows, int dim, int ffn) {
    EncBufs b;
    const int64_t r = rows;
    b.h = 0;
    b.qkv = b.h + align_up(r * dim * 2);
    b.att = b.qkv + align_up(r * 3 * dim * 2);
    b.g = b.att + align_up(r * dim * 2);
    b.ss = b.g + align_up(r * (int64_t)ffn * 2);
    b.qkss = b.ss + align_up(r * RF_PRENORM_SLOTS * 4);
    b.total = b.qkss + align_up(r * 2 * RF_PRENORM_SLOTS * 4);
    return b;
}

// softmax scale * log2(e) for head_dim 128: q carries it (rf_qk_norm_rope seg0_scale), attention runs with scale ln 2
const float kLn2 = 0.69314718055994530942f;
const float kQLog2Scale = (float)(1.0 / std::sqrt(128.0) / 0.69314718055994530942);
}  // namespace

#define RF_CALL(expr)                     \
    do {                                  \
        const int rc_ = (expr);           \
        if (rc_ != RF_OK) return rc_;     \
    } while (0)

extern "C" int64_t rf_encoder_workspace_bytes(int rows, int dim, int ffn_dim, int operand_dtype) {
    (void)operand_dtype;  // both operand types are 2 bytes
    if (rows <= 0 || dim <= 0 || ffn_dim <= 0) return 0;
    return enc_layout(rows, dim, ffn_dim).total;
}

extern "C" int rf_encoder_forward(float* x, int64_t ldx, const rf_encoder_desc* d, void* stream) {
    RF_REQUIRE(d, "rf_encoder_forward: null descriptor");
    RF_REQUIRE(d->n_layers >= 0 && d->rows >= 0, "rf_encoder_forward: negative size");
    if (d->n_layers == 0 || d->rows == 0) return RF_OK;
    RF_REQUIRE(x && d->layers && d->workspace && d->attn_ws && d->problems, "rf_encoder_forward: null pointer");
    RF_REQUIRE(d->operand_dtype == RF_DT_F16 || d->operand_dtype == RF_DT_BF16,
               "rf_encoder_forward: operand_dtype must be RF_DT_F16 or RF_DT_BF16");
    RF_REQUIRE(d->n_heads >= 1 && d->dim == d->n_heads * 128,
               "rf_encoder_forward: dim (%d) must be n_heads (%d) * 128", d->dim, d->n_heads);
    RF_REQUIRE(d->ffn_dim > 0 && d->ffn_dim % 128 == 0, "rf_encoder_forward: ffn_dim must be a positive multiple of 128");
    RF_REQUIRE(ldx >= d->dim && ldx % 4 == 0, "rf_encoder_forward: ldx must be >= dim and 16-B aligned");
    RF_REQUIRE(!d->pos || (d->freqs && d->n_freqs > 0 && d->ld_pos >= 9),
               "rf_encoder_forward: pos needs freqs (and ld_pos >= 9)");
    RF_REQUIRE(d->n_problems >= 1, "rf_encoder_forward: no attention problems");
    RF_REQUIRE(((uintptr_t)d->workspace % kAlign) == 0, "rf_encoder_forward: workspace must be 256-B aligned");
    for (int i = 0; i < d->n_layers; ++i) {
        const rf_encoder_layer& L = d->layers[i];
        RF_REQUIRE(L.attn_norm && L.w_qkv && L.w_out && L.ffn_norm && L.w13 && L.w2,
                   "rf_encoder_forward: layer %d has a null weight", i);
    }
    const int T = d->rows, D = d->dim, H = d->n_heads, F = d->ffn_dim;
    const bool f16 = d->operand_dtype == RF_DT_F16;
    const EncBufs b = enc_layout(T, D, F);
    char* ws = static_cast<char*>(d->workspace);
    void* h = ws + b.h;                               // x * g (deferred RMSNorm): the next GEMM's A operand
    uint16_t* qkv = reinterpret_cast<uint16_t*>(ws + b.qkv);  // bf16 q | k | v (attention operands)
    void* att = ws + b.att;                           // attention O: the out-projection's A operand
    void* g = ws + b.g;                               // SwiGLU output: W2's A operand
    float* ss = reinterpret_cast<float*>(ws + b.ss);  // the pre-norm's partial sums of squares
    float* qkss = reinterpret_cast<float*>(ws + b.qkss);  // q / k partial sums of squares (fused QK path)
    auto gemm = f16 ? rf_gemm_f16 : rf_gemm_bf16;
    const int epi_swiglu = f16 ? RF_EPI_SWIGLU_F16 : RF_EPI_SWIGLU;
    const int o_dt = f16 ? RF_DT_F16 : RF_DT_BF16;
    const int dt = d->operand_dtype;
    void* gws = d->gemm_ws;
    const int64_t gwb = d->gemm_ws_bytes;
    // each pre-norm is deferred (rf.h): the residual GEMM before it writes x * g and the row sums of squares, the
    // projection after it scales its rows by 1 / rms; only layer 0's attention norm reads x in a row kernel
    RF_CALL(rf_prenorm(x, ldx, d->layers[0].attn_norm, h, D, ss, T, D, dt, stream));
    for (int i = 0; i < d->n_layers; ++i) {
        const rf_encoder_layer& L = d->layers[i];
        if (d->qk_fused) {
            // the positional encoding fused into the QK path (rf.h ABI 16): the projection's epilogue applies the
            // q/k norm weights and the triangle RoPE and writes the rows' sums of squares; k gets its 1 / rms in a
            // row pass, q as the attention loads it (with no q/k norm, the projection also applies q's softmax scale)
            const bool qkn = L.qk_norm != nullptr;
            RF_CALL(rf_gemm_qk_rope(h, D, L.w_qkv, D, qkv, 3 * D, T, 3 * D, D, ss, D, d->eps, qkn ? qkss : nullptr, D, 2,
                                    L.qk_norm, d->pos, d->ld_pos, 1, d->freqs, d->pos ? d->n_freqs : 0,
                                    qkn ? 1.0f : kQLog2Scale, dt, gws, gwb, stream));
            if (qkn) RF_CALL(rf_row_rms_scale(qkv + D, 3 * D, T, D, qkss + RF_PRENORM_SLOTS, 2 * RF_PRENORM_SLOTS, d->eps, 1.0f,
                                              stream));
            if (d->timer_attn) RF_CALL(rf_ktimer_arm());
            if (qkn)
                RF_CALL(rf_attn_fwd_qn(qkv, 3 * D, qkv + D, 3 * D, qkv + 2 * D, 3 * D, att, D, o_dt, qkss,
                                       2 * RF_PRENORM_SLOTS, D, d->eps, kQLog2Scale, d->problems, d->n_problems, H, 128,
                                       d->attn_ws, d->bounds, d->bounds ? d->grid : 0, stream));
            else
                RF_CALL(rf_attn_fwd_dt(qkv, 3 * D, qkv + D, 3 * D, qkv + 2 * D, 3 * D, att, D, RF_DT_BF16, o_dt,
                                       d->problems, d->n_problems, H, 128, kLn2, d->attn_ws, d->bounds,
                                       d->bounds ? d->grid : 0, stream));
        } else {
            RF_CALL(rf_gemm_rownorm(h, D, L.w_qkv, D, qkv, 3 * D, T, 3 * D, D, RF_EPI_BF16, ss, D, d->eps, nullptr, 0, 0, dt,
                                    gws, gwb, stream));
            RF_CALL(rf_qk_norm_rope(qkv, 3 * D, qkv, 3 * D, nullptr, T, D, H, 2, L.qk_norm, d->eps, kQLog2Scale, d->pos,
                                    d->ld_pos, 1, d->freqs, d->pos ? d->n_freqs : 0, stream));
            if (d->timer_attn) RF_CALL(rf_ktimer_arm());
            RF_CALL(rf_attn_fwd_dt(qkv, 3 * D, qkv + D, 3 * D, qkv + 2 * D, 3 * D, att, D, RF_DT_BF16, o_dt, d->problems,
                                   d->n_problems, H, 128, kLn2, d->attn_ws, d->bounds, d->bounds ? d->grid : 0, stream));
        }
        RF_CALL(rf_gemm_add_prenorm(att, D, L.w_out, D, x, ldx, T, D, D, L.ffn_norm, h, D, ss, dt, gws, gwb, stream));
        RF_CALL(rf_gemm_rownorm(h, D, L.w13, D, g, F, T, 2 * F, D, epi_swiglu, ss, D, d->eps, nullptr, 0, 0, dt, gws, gwb, stream));
        if (i + 1 < d->n_layers)
            RF_CALL(rf_gemm_add_prenorm(g, F, L.w2, F, x, ldx, T, D, F, d->layers[i + 1].attn_norm, h, D, ss, dt, gws,
                                        gwb, stream));
        else
            RF_CALL(gemm(g, F, L.w2, F, x, ldx, nullptr, T, D, F, RF_EPI_ADD_F32, gws, gwb, stream));
    }
    return RF_OK;
}

// ---------------------------------------------------------------------------------------------------------------
// rf_decoder_forward replaces TransformerDecoder.forward (attention.py:673-688): per layer the cross-attention of
// the ray tokens to their scene's triangles (K/V from the stage-1 output, keys rotated per view with the camera-
// frame triangle positions), the self-attention between ray tokens (Swin windows with the shift on odd layers,
// attention.py:604-605, or full attention), the SwiGLU FFN, and the DPT taps of view_transformer.py:85.  The same
// launches in the same order as model.py::_stage2 (bit-identical), one C call for the whole stack.
namespace {
struct DecBufs {
    int64_t h, q2, att, g, hc, kv, kview, qkv, ss, qkss, total;
};
DecBufs dec_layout(const rf_decoder_desc* d) {
    const int64_t T2 = d->rows, D = d->dim, F = d->ffn_dim, T1 = d->ctx_rows, L = d->n_layers;
    const bool kv_batch = d->w_kv_all != nullptr, k_batch = kv_batch && d->k_batch;
    DecBufs b;
    b.h = 0;
    b.q2 = b.h + align_up(T2 * D * 2);
    b.att = b.q2 + align_up(T2 * D * 2);
    b.g = b.att + align_up(T2 * D * 2);
    b.hc = b.g + align_up(T2 * F * 2);
    b.kv = b.hc + align_up(T1 * d->ctx_dim * 2);
    b.kview = b.kv + align_up(T1 * (kv_batch ? L : 1) * 2 * D * 2);
    b.qkv = b.kview + align_up((int64_t)d->kv_rows * (k_batch ? L : 1) * D * 2);
    b.ss = b.qkv + (d->layers && d->n_layers > 0 && d->layers[0].self_norm ? align_up(T2 * 3 * D * 2) : 0);
    b.qkss = b.ss + align_up(T2 * RF_PRENORM_SLOTS * 4);
    // (Swin's q/k row sums [T2][2][slots]; with qk_fused also the cross-attention q's [T2][1][slots], used earlier)
    b.total = b.qkss + align_up(T2 * (d->swin ? 2 : 1) * RF_PRENORM_SLOTS * 4);
    return b;
}
}  // namespace

extern "C" int64_t rf_decoder_workspace_bytes(const rf_decoder_desc* d) {
    if (!d || d->n_layers <= 0 || d->rows <= 0 || d->dim <= 0 || d->ffn_dim <= 0 || d->ctx_rows < 0 ||
        d->ctx_dim <= 0 || d->kv_rows < 0)
        return 0;
    return dec_layout(d).total;
}

extern "C" int rf_decoder_forward(float* x, int64_t ldx, const rf_decoder_desc* d, void* stream) {
    RF_REQUIRE(d, "rf_decoder_forward: null descriptor");
    RF_REQUIRE(d->n_layers >= 0 && d->rows >= 0, "rf_decoder_forward: negative size");
    if (d->n_layers == 0 || d->rows == 0) return RF_OK;
    RF_REQUIRE(x && d->layers && d->workspace && d->attn_ws && d->ctx && d->cross_problems && d->kv_src_rows,
               "rf_decoder_forward: null pointer");
    RF_REQUIRE(d->operand_dtype == RF_DT_F16 || d->operand_dtype == RF_DT_BF16,
               "rf_decoder_forward: operand_dtype must be RF_DT_F16 or RF_DT_BF16");
    RF_REQUIRE(d->n_heads >= 1 && d->dim == d->n_heads * 128,
               "rf_decoder_forward: dim (%d) must be n_heads (%d) * 128", d->dim, d->n_heads);
    RF_REQUIRE(d->ffn_dim > 0 && d->ffn_dim % 128 == 0, "rf_decoder_forward: ffn_dim must be a positive multiple of 128");
    RF_REQUIRE(ldx >= d->dim && ldx % 4 == 0, "rf_decoder_forward: ldx must be >= dim and 16-B aligned");
    RF_REQUIRE(d->ctx_rows > 0 && d->ctx_dim > 0 && d->ctx_dim % 64 == 0 && d->ld_ctx >= d->ctx_dim,
               "rf_decoder_forward: context [ctx_rows, ctx_dim] with ctx_dim % 64 == 0");
    RF_REQUIRE(d->kv_rows > 0 && d->n_cross >= 1, "rf_decoder_forward: no keys / cross-attention problems");
    RF_REQUIRE(!d->k_batch || d->w_kv_all, "rf_decoder_forward: k_batch needs the batched K/V (w_kv_all)");
    RF_REQUIRE(!d->kv_pos || (d->freqs && d->n_freqs > 0 && d->ld_kv_pos >= 9),
               "rf_decoder_forward: kv_pos needs freqs (and ld_kv_pos >= 9)");
    RF_REQUIRE(!d->ray_pos || (d->freqs && d->n_freqs > 0 && d->ld_ray_pos >= 9 && d->ray_pos_div >= 1),
               "rf_decoder_forward: ray_pos needs freqs, ld_ray_pos >= 9 and ray_pos_div >= 1");
    RF_REQUIRE(((uintptr_t)d->workspace % kAlign) == 0, "rf_decoder_forward: workspace must be 256-B aligned");
    RF_REQUIRE(d->n_taps >= 0 && (d->n_taps == 0 || d->taps), "rf_decoder_forward: taps");
    const bool self_attn = d->layers[0].self_norm != nullptr;
    for (int i = 0; i < d->n_layers; ++i) {
        const rf_decoder_layer& L = d->layers[i];
        RF_REQUIRE(L.query_norm && L.w_q && L.w_out && L.ffn_norm && L.w13 && L.w2,
                   "rf_decoder_forward: layer %d has a null weight", i);
        RF_REQUIRE(d->w_kv_all || (L.kv_norm && L.w_kv), "rf_decoder_forward: layer %d has no K/V weights", i);
        RF_REQUIRE((L.self_norm != nullptr) == self_attn && (!self_attn || (L.w_self_in && L.w_self_out)),
                   "rf_decoder_forward: layer %d: self-attention weights must be given for every layer or none", i);
    }
    if (self_attn && d->swin)
        RF_REQUIRE(d->n_images >= 1 && d->grid_h >= 1 && d->grid_w >= 1 && d->window >= 1 &&
                       (int64_t)d->n_images * d->grid_h * d->grid_w == d->rows,
                   "rf_decoder_forward: Swin grid n_images x grid_h x grid_w must cover the rows");
    if (self_attn && !d->swin) RF_REQUIRE(d->self_problems && d->n_self >= 1, "rf_decoder_forward: no self problems");
    for (int t = 0; t < d->n_taps; ++t)
        RF_REQUIRE(d->taps[t].p_hi && d->taps[t].p_ld >= d->dim && d->taps[t].layer >= 0 &&
                       d->taps[t].layer < d->n_layers && (t == 0 || d->taps[t].layer > d->taps[t - 1].layer),
                   "rf_decoder_forward: tap %d (layer order, planes, p_ld >= dim)", t);

    const int T2 = d->rows, D = d->dim, H = d->n_heads, F = d->ffn_dim, T1 = d->ctx_rows, NL = d->n_layers;
    const bool f16 = d->operand_dtype == RF_DT_F16;
    const bool kv_batch = d->w_kv_all != nullptr, k_batch = kv_batch && d->k_batch;
    const DecBufs b = dec_layout(d);
    char* ws = static_cast<char*>(d->workspace);
    void* h = ws + b.h;
    uint16_t* q2 = reinterpret_cast<uint16_t*>(ws + b.q2);
    void* att = ws + b.att;
    void* g = ws + b.g;
    void* hc = ws + b.hc;
    uint16_t* kv = reinterpret_cast<uint16_t*>(ws + b.kv);
    uint16_t* kview = reinterpret_cast<uint16_t*>(ws + b.kview);
    uint16_t* qkv = reinterpret_cast<uint16_t*>(ws + b.qkv);
    float* ss = reinterpret_cast<float*>(ws + b.ss);
    float* qkss = reinterpret_cast<float*>(ws + b.qkss);  // Swin q/k row sums (rf_swin_attn_fwd_qkn)
    const int dt = d->operand_dtype;
    const int64_t ld_kv = (kv_batch ? (int64_t)NL : 1) * 2 * D, ld_kview = (k_batch ? (int64_t)NL : 1) * D;
    auto rmsnorm = f16 ? rf_rmsnorm_f16 : rf_rmsnorm;
    auto gemm = f16 ? rf_gemm_f16 : rf_gemm_bf16;
    const int epi_swiglu = f16 ? RF_EPI_SWIGLU_F16 : RF_EPI_SWIGLU;
    const int o_dt = f16 ? RF_DT_F16 : RF_DT_BF16;
    void* gws = d->gemm_ws;
    const int64_t gwb = d->gemm_ws_bytes;
    const int nf = d->n_freqs;
    if (kv_batch) {  // every layer's K/V in one GEMM over the unit-normed context
        RF_CALL(rmsnorm(d->ctx, d->ld_ctx, d->ctx_norm, d->eps, hc, d->ctx_dim, T1, d->ctx_dim, stream));
        RF_CALL(gemm(hc, d->ctx_dim, d->w_kv_all, d->ctx_dim, kv, ld_kv, nullptr, T1, (int)ld_kv, d->ctx_dim,
                     RF_EPI_BF16, gws, gwb, stream));
    }
    // the keys' norm + rotation: the standard layout, or (qk_fused) the pair-interleaved order of the permuted weights
    auto k_rope = d->qk_fused ? rf_qk_norm_rope_groups_ilv : rf_qk_norm_rope_groups;
    if (k_batch)  // every layer's keys normed and rotated per view in one launch
        RF_CALL(k_rope(kv, ld_kv, 2 * D, kview, ld_kview, D, d->kv_src_rows, d->kv_rows, D, H, 1, NL, d->k_norm_all, D,
                       d->eps, 1.0f, d->kv_pos, d->ld_kv_pos, 1, d->freqs, d->kv_pos ? nf : 0, stream));
    int tap = 0;
    // the ray tokens' pre-norms are deferred as in the encoder (rf.h): only layer 0's query norm is a row kernel
    RF_CALL(rf_prenorm(x, ldx, d->layers[0].query_norm, h, D, ss, T2, D, dt, stream));
    for (int i = 0; i < NL; ++i) {
        const rf_decoder_layer& L = d->layers[i];
        // (i) cross-attention.  qk_fused: the query's norm weight and ray rotation in its projection's epilogue, its
        // 1 / rms in the attention's Q load (row sums in qkss, [T2][1][RF_PRENORM_SLOTS]; the Swin sums come later)
        const bool qf = d->qk_fused != 0, qn = qf && L.q_norm;
        if (qf)
            RF_CALL(rf_gemm_qk_rope(h, D, L.w_q, D, q2, D, T2, D, D, ss, D, d->eps, qn ? qkss : nullptr, D, 1, L.q_norm,
                                    d->ray_pos, d->ld_ray_pos, d->ray_pos ? d->ray_pos_div : 1, d->freqs,
                                    d->ray_pos ? nf : 0, qn ? 1.0f : kQLog2Scale, dt, gws, gwb, stream));
        else
            RF_CALL(rf_gemm_rownorm(h, D, L.w_q, D, q2, D, T2, D, D, RF_EPI_BF16, ss, D, d->eps, nullptr, 0, 0, dt, gws,
                                    gwb, stream));
        const uint16_t* kvi = kv_batch ? kv + (int64_t)2 * D * i : kv;
        if (!kv_batch) {
            RF_CALL(rmsnorm(d->ctx, d->ld_ctx, L.kv_norm, d->eps, hc, d->ctx_dim, T1, d->ctx_dim, stream));
            RF_CALL(gemm(hc, d->ctx_dim, L.w_kv, d->ctx_dim, kv, ld_kv, nullptr, T1, 2 * D, d->ctx_dim, RF_EPI_BF16,
                         gws, gwb, stream));
        }
        const uint16_t* ki = k_batch ? kview + (int64_t)D * i : kview;
        if (!qf)
            RF_CALL(rf_qk_norm_rope(q2, D, q2, D, nullptr, T2, D, H, 1, L.q_norm, d->eps, kQLog2Scale, d->ray_pos,
                                    d->ld_ray_pos, d->ray_pos ? d->ray_pos_div : 1, d->freqs, d->ray_pos ? nf : 0,
                                    stream));
        if (!k_batch)
            RF_CALL(k_rope(kvi, ld_kv, 0, kview, ld_kview, 0, d->kv_src_rows, d->kv_rows, D, H, 1, 1, L.k_norm, 0, d->eps,
                           1.0f, d->kv_pos, d->ld_kv_pos, 1, d->freqs, d->kv_pos ? nf : 0, stream));
        if (d->timer_cross) RF_CALL(rf_ktimer_arm());
        if (qn)
            RF_CALL(rf_attn_fwd_qn(q2, D, ki, ld_kview, kvi + D, ld_kv, att, D, o_dt, qkss, RF_PRENORM_SLOTS, D, d->eps,
                                   kQLog2Scale, d->cross_problems, d->n_cross, H, 128, d->attn_ws, d->cross_bounds,
                                   d->cross_bounds ? d->cross_grid : 0, stream));
        else
            RF_CALL(rf_attn_fwd_dt(q2, D, ki, ld_kview, kvi + D, ld_kv, att, D, RF_DT_BF16, o_dt, d->cross_problems,
                                   d->n_cross, H, 128, kLn2, d->attn_ws, d->cross_bounds,
                                   d->cross_bounds ? d->cross_grid : 0, stream));
        RF_CALL(rf_gemm_add_prenorm(att, D, L.w_out, D, x, ldx, T2, D, D, self_attn ? L.self_norm : L.ffn_norm, h, D,
                                    ss, dt, gws, gwb, stream));
        // (ii) self-attention between ray tokens
        if (self_attn) {
            // Swin: the full-width q/k norm folds into the attention's loads, fed by the projection's row sums
            // (rf_swin_attn_fwd_qkn); the per-op q/k norm pass remains for widths the segment sums do not cover
            const bool qkn = d->swin && L.self_qk_norm && D % 256 == 0 && D <= RF_PRENORM_SLOTS * 128;
            RF_CALL(rf_gemm_rownorm(h, D, L.w_self_in, D, qkv, 3 * D, T2, 3 * D, D, RF_EPI_BF16, ss, D, d->eps,
                                    qkn ? qkss : nullptr, D, 2, dt, gws, gwb, stream));
            if (qkn) {
                RF_CALL(rf_swin_attn_fwd_qkn(qkv, 3 * D, qkv + D, 3 * D, qkv + 2 * D, 3 * D, att, D, o_dt, d->n_images,
                                             d->grid_h, d->grid_w, d->window, i % 2 == 0 ? 0 : d->shift, H, 128, kLn2,
                                             qkss, L.self_qk_norm, d->eps, kQLog2Scale, stream));
            } else if (d->swin) {
                RF_CALL(rf_qk_norm_rope(qkv, 3 * D, qkv, 3 * D, nullptr, T2, D, H, 2, L.self_qk_norm, d->eps,
                                        kQLog2Scale, nullptr, 0, 1, nullptr, 0, stream));
                RF_CALL(rf_swin_attn_fwd_dt(qkv, 3 * D, qkv + D, 3 * D, qkv + 2 * D, 3 * D, att, D, o_dt, d->n_images,
                                            d->grid_h, d->grid_w, d->window, i % 2 == 0 ? 0 : d->shift, H, 128, kLn2,
                                            stream));
            } else {
                RF_CALL(rf_qk_norm_rope(qkv, 3 * D, qkv, 3 * D, nullptr, T2, D, H, 2, L.self_qk_norm, d->eps,
                                        kQLog2Scale, d->ray_pos, d->ld_ray_pos, d->ray_pos ? d->ray_pos_div : 1,
                                        d->freqs, d->ray_pos ? nf : 0, stream));
                RF_CALL(rf_attn_fwd_dt(qkv, 3 * D, qkv + D, 3 * D, qkv + 2 * D, 3 * D, att, D, RF_DT_BF16, o_dt,
                                       d->self_problems, d->n_self, H, 128, kLn2, d->attn_ws, nullptr, 0, stream));
            }
            RF_CALL(rf_gemm_add_prenorm(att, D, L.w_self_out, D, x, ldx, T2, D, D, L.ffn_norm, h, D, ss, dt, gws, gwb,
                                        stream));
        }
        // (iii) FFN
        RF_CALL(rf_gemm_rownorm(h, D, L.w13, D, g, F, T2, 2 * F, D, epi_swiglu, ss, D, d->eps, nullptr, 0, 0, dt, gws, gwb, stream));
        if (i + 1 < NL)
            RF_CALL(rf_gemm_add_prenorm(g, F, L.w2, F, x, ldx, T2, D, F, d->layers[i + 1].query_norm, h, D, ss, dt, gws,
                                        gwb, stream));
        else
            RF_CALL(gemm(g, F, L.w2, F, x, ldx, nullptr, T2, D, F, RF_EPI_ADD_F32, gws, gwb, stream));
        if (tap < d->n_taps && d->taps[tap].layer == i) {  // straight into the DPT projection's operand planes
            const rf_decoder_tap& t = d->taps[tap++];
            RF_CALL(rf_split_planes(x, T2, D, ldx, t.p_hi, t.p_lo, t.p_ld, 0, stream));
        }
    }
    return RF_OK;
}
