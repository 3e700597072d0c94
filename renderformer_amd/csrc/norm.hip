// Row-wise kernels: RMSNorm (f32 residual -> bf16 GEMM operand), full-width q/k
// RMSNorm fused with the triangle RoPE, and token-embedding assembly.
//
// All are HBM-bound streaming kernels: one wave64 per row, fp32 reductions with
// xor-shuffles, 8-16 B per lane accesses where the layout allows.
#include <math.h>
#include <stdlib.h>

#include "common.h"

namespace {

constexpr int ROWS_PER_BLOCK = 4;  // 4 waves, one row each

// ----------------------------------------------------------------------------- RMSNorm
// F16: the 16-bit output is fp16 (the A operand of an fp16 GEMM) instead of bf16
template <bool F16>
RF_DEV uint32_t pack_out(float lo, float hi) { return F16 ? pack_f16x2(lo, hi) : pack_bf16x2(lo, hi); }

template <bool F16>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const float* __restrict__ x, int64_t ldx,
                                                      const float* __restrict__ w, float eps,
                                                      bf16_t* __restrict__ out, int64_t ldo, int rows, int dim,
                                                      int* range) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float* xr = x + (int64_t)row * ldx;
    float ss = 0.f;
    for (int c = lane * 4; c < dim; c += 256) {
        const float4 v = *reinterpret_cast<const float4*>(xr + c);
        ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    ss = wave_sum(ss);
    const float inv = 1.0f / sqrtf(ss / (float)dim + eps);
    bf16_t* orow = out + (int64_t)row * ldo;
    float amax = 0.f;
    for (int c = lane * 4; c < dim; c += 256) {
        const float4 v = *reinterpret_cast<const float4*>(xr + c);
        const float4 g = *reinterpret_cast<const float4*>(w + c);
        const float o0 = v.x * inv * g.x, o1 = v.y * inv * g.y, o2 = v.z * inv * g.z, o3 = v.w * inv * g.w;
        if constexpr (F16) amax = amax3(amax3(amax, o0, o1), o2, o3);
        uint2 pk;
        pk.x = pack_out<F16>(o0, o1);
        pk.y = pack_out<F16>(o2, o3);
        *reinterpret_cast<uint2*>(orow + c) = pk;
    }
    if (F16 && range && !f16_in_range(amax)) report_f16_range(range, RF_RANGE_RMSNORM);
}

// dim = 256 * NV: the whole row and its weights are loaded up front (NV float4 per lane each, all in
// flight at once), so a row costs one memory round trip instead of one per 256 columns plus a re-read
template <int NV, bool F16>
__global__ __launch_bounds__(256) void rmsnorm_v_kernel(const float* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ w, float eps,
                                                        bf16_t* __restrict__ out, int64_t ldo, int rows,
                                                        int* range) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float* xr = x + (int64_t)row * ldx + 4 * lane;
    float4 v[NV], g[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = *reinterpret_cast<const float4*>(xr + 256 * i);
#pragma unroll
    for (int i = 0; i < NV; ++i) g[i] = *reinterpret_cast<const float4*>(w + 4 * lane + 256 * i);
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) ss += v[i].x * v[i].x + v[i].y * v[i].y + v[i].z * v[i].z + v[i].w * v[i].w;
    ss = wave_sum(ss);
    const float inv = 1.0f / sqrtf(ss / (float)(256 * NV) + eps);
    bf16_t* orow = out + (int64_t)row * ldo + 4 * lane;
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const float o0 = v[i].x * inv * g[i].x, o1 = v[i].y * inv * g[i].y;
        const float o2 = v[i].z * inv * g[i].z, o3 = v[i].w * inv * g[i].w;
        if constexpr (F16) amax = amax3(amax3(amax, o0, o1), o2, o3);
        uint2 pk;
        pk.x = pack_out<F16>(o0, o1);
        pk.y = pack_out<F16>(o2, o3);
        *reinterpret_cast<uint2*>(orow + 256 * i) = pk;
    }
    if (F16 && range && !f16_in_range(amax)) report_f16_range(range, RF_RANGE_RMSNORM);
}

// Deferred RMSNorm, row form (rf_prenorm): xg = 16-bit(x * g) and the row's sum of x^2 into slot 0 of its
// RF_PRENORM_SLOTS floats (slots 1.. zero), one pass over the row; the consumer GEMM (rf_gemm_rownorm) applies
// 1 / rms.  The first layer's pre-norm (x from the embedding, not from a GEMM) and the fallback of
// rf_gemm_add_prenorm above RF_PRENORM_SLOTS column tiles.
template <bool F16>
__global__ __launch_bounds__(256) void prenorm_kernel(const float* __restrict__ x, int64_t ldx,
                                                      const float* __restrict__ w, bf16_t* __restrict__ xg,
                                                      int64_t ldg, float* __restrict__ ss, int rows, int dim,
                                                      int* range) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float* xr = x + (int64_t)row * ldx;
    bf16_t* orow = xg + (int64_t)row * ldg;
    float s = 0.f, amax = 0.f;
    for (int c = lane * 4; c < dim; c += 256) {
        const float4 v = *reinterpret_cast<const float4*>(xr + c);
        const float4 g = *reinterpret_cast<const float4*>(w + c);
        s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        const float y0 = v.x * g.x, y1 = v.y * g.y, y2 = v.z * g.z, y3 = v.w * g.w;
        if constexpr (F16) amax = amax3(amax3(amax, y0, y1), y2, y3);
        uint2 pk;
        pk.x = pack_out<F16>(y0, y1);
        pk.y = pack_out<F16>(y2, y3);
        *reinterpret_cast<uint2*>(orow + c) = pk;
    }
    s = wave_sum(s);
    if (lane < RF_PRENORM_SLOTS / 4)
        reinterpret_cast<float4*>(ss + (int64_t)row * RF_PRENORM_SLOTS)[lane] =
            lane == 0 ? make_float4(s, 0.f, 0.f, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (F16 && range && !f16_in_range(amax)) report_f16_range(range, RF_RANGE_RMSNORM);
}

// ----------------------------------------------------------------------------- q/k norm + RoPE
// Work unit = (segment, head h, 8-element chunk j of the first half): it owns chunks j and
// j+8 of that head, i.e. the rotation pairs (8j+e, 8j+e+64), so the half-split rotation is
// done in registers and the row can be rewritten in place.  A wave owns a fixed unit set
// and walks rows grid-stride, so the norm weights are loaded into registers once.  The 64
// angles of a row are computed once (lane i -> angle i, accurate sincosf) and broadcast
// with cross-lane shuffles (all lanes active).  Segments (q and k of one qkv row) share
// the angles; each has its own full-width RMSNorm.
constexpr int MAX_UNITS = 256;  // segments * heads * 8

template <int UPL>
__global__ __launch_bounds__(256) void qk_norm_rope_kernel(const bf16_t* src, int64_t ld_src, bf16_t* dst,
                                                           int64_t ld_dst, const int32_t* __restrict__ src_rows,
                                                           int rows, int n_heads, int n_seg,
                                                           const float* __restrict__ norm_w, float eps,
                                                           float seg0_scale,
                                                           const float* __restrict__ pos, int64_t ld_pos, int pos_div,
                                                           const float* __restrict__ freqs, int n_freqs) {
    const int lane = threadIdx.x & 63;
    const int units = n_seg * n_heads * 8;
    const int dim = n_heads * 128;
    // unit -> (segment, head, chunk); column of the first chunk element
    int col[UPL];
    float wlo[UPL][8], whi[UPL][8];
#pragma unroll
    for (int u = 0; u < UPL; ++u) {
        const int unit = lane + 64 * u;
        const int seg = unit / (n_heads * 8), hj = unit % (n_heads * 8);
        col[u] = seg * dim + (hj >> 3) * 128 + 8 * (hj & 7);
        if (norm_w && unit < units) {
            const float4* wl = reinterpret_cast<const float4*>(norm_w + col[u]);
            const float4* wh = reinterpret_cast<const float4*>(norm_w + col[u] + 64);
            const float4 l0 = wl[0], l1 = wl[1], h0 = wh[0], h1 = wh[1];
            const float lv[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
            const float hv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                wlo[u][e] = lv[e];
                whi[u][e] = hv[e];
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) wlo[u][e] = whi[u][e] = 1.f;
        }
        // segment 0 (q) may carry the softmax scale * log2(e) for the attention kernel; RoPE is linear
        if (unit < n_heads * 8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                wlo[u][e] *= seg0_scale;
                whi[u][e] *= seg0_scale;
            }
        }
    }
    const int stride = gridDim.x * ROWS_PER_BLOCK;
    for (int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6); row < rows; row += stride) {
        const int srow = src_rows ? src_rows[row] : row;
        const bf16_t* s = src + (int64_t)srow * ld_src;
        // RoPE angle inputs are loaded with the row (one round trip), the sincos waits for them
        float ang = 0.f;
        if (pos && lane < 9 * n_freqs) ang = pos[(int64_t)(row / pos_div) * ld_pos + lane / n_freqs] * freqs[lane % n_freqs];
        u32x4 lo[UPL], hi[UPL];
        float ss[UPL];
#pragma unroll
        for (int u = 0; u < UPL; ++u) {
            ss[u] = 0.f;
            if (lane + 64 * u < units) {
                lo[u] = *reinterpret_cast<const u32x4*>(s + col[u]);
                hi[u] = *reinterpret_cast<const u32x4*>(s + col[u] + 64);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float a0 = __uint_as_float(lo[u][e] << 16), a1 = __uint_as_float(lo[u][e] & 0xffff0000u);
                    const float b0 = __uint_as_float(hi[u][e] << 16), b1 = __uint_as_float(hi[u][e] & 0xffff0000u);
                    ss[u] += a0 * a0 + a1 * a1 + b0 * b0 + b1 * b1;
                }
            }
        }
        // per-segment sum of squares: a segment spans n_heads*8 units = whole 64-lane groups when
        // n_heads*8 is a multiple of 64, otherwise a lane sub-range; reduce per segment explicitly.
        float inv[UPL];
#pragma unroll
        for (int u = 0; u < UPL; ++u) inv[u] = 1.f;
        if (norm_w) {
            const int upsg = n_heads * 8;
            for (int sg = 0; sg < n_seg; ++sg) {
                float part = 0.f;
#pragma unroll
                for (int u = 0; u < UPL; ++u) {
                    const int unit = lane + 64 * u;
                    part += (unit < units && unit / upsg == sg) ? ss[u] : 0.f;
                }
                const float tot = wave_sum(part);
                const float iv = 1.0f / sqrtf(tot / (float)dim + eps);
#pragma unroll
                for (int u = 0; u < UPL; ++u)
                    if ((lane + 64 * u) / upsg == sg) inv[u] = iv;
            }
        }
        float my_c = 1.f, my_s = 0.f;
        // hardware sin/cos: ~1e-6 absolute, far below the bf16 rounding of the rotated output
        if (pos && lane < 9 * n_freqs) __sincosf(ang, &my_s, &my_c);
        // every unit of this lane has chunk index j = lane & 7 (64 is a multiple of 8)
        float cs[8], sn[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            cs[k] = pos ? __shfl(my_c, 8 * (lane & 7) + k, 64) : 1.f;
            sn[k] = pos ? __shfl(my_s, 8 * (lane & 7) + k, 64) : 0.f;
        }
        bf16_t* d = dst + (int64_t)row * ld_dst;
#pragma unroll
        for (int u = 0; u < UPL; ++u) {
            if (lane + 64 * u < units) {
                u32x4 olo, ohi;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float ra[2], rb[2];
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const int i = 2 * e + t;
                        const float a = (t ? __uint_as_float(lo[u][e] & 0xffff0000u) : __uint_as_float(lo[u][e] << 16));
                        const float b = (t ? __uint_as_float(hi[u][e] & 0xffff0000u) : __uint_as_float(hi[u][e] << 16));
                        const float x0 = a * inv[u] * wlo[u][i], x1 = b * inv[u] * whi[u][i];
                        ra[t] = x0 * cs[i] - x1 * sn[i];  // rotate_half_hf: (-x2, x1)
                        rb[t] = x1 * cs[i] + x0 * sn[i];
                    }
                    olo[e] = pack_bf16x2(ra[0], ra[1]);
                    ohi[e] = pack_bf16x2(rb[0], rb[1]);
                }
                *reinterpret_cast<u32x4*>(d + col[u]) = olo;
                *reinterpret_cast<u32x4*>(d + col[u] + 64) = ohi;
            }
        }
    }
}

// One row per wave, no row loop (like rmsnorm_v_kernel): the row's q/k chunks are issued first, then the
// RoPE position and the norm weights, so every load of a wave is in flight in one round trip and the
// grid holds all rows at once (stage 1: 5,649 rows = 5,652 waves, 5.5 per SIMD).
// ILV: the pair-interleaved column order of rf_gemm_qk_rope (per head, column 2 m + t = dimension m + 64 t): a unit is
// 16 consecutive columns (rotation pairs 8 (unit & 7) .. + 7, the same angles as the half-split unit), lo / hi its
// two 16-B halves, each dword one (x1, x2) pair
template <int UPL, bool ILV = false>
__global__ __launch_bounds__(256) void qk_norm_rope_row_kernel(const bf16_t* src, int64_t ld_src, bf16_t* dst,
                                                               int64_t ld_dst, const int32_t* __restrict__ src_rows,
                                                               int rows, int n_heads, int n_seg,
                                                               const float* __restrict__ norm_w, float eps,
                                                               float seg0_scale,
                                                               const float* __restrict__ pos, int64_t ld_pos,
                                                               int pos_div, const float* __restrict__ freqs,
                                                               int n_freqs, int64_t src_gstride, int64_t dst_gstride,
                                                               int w_gstride, int split_qk) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    if (row >= rows) return;
    // group blockIdx.y: its own column block of src/dst and its own norm weights (same rows, same RoPE)
    src += blockIdx.y * src_gstride;
    dst += blockIdx.y * dst_gstride;
    if (norm_w) norm_w += blockIdx.y * w_gstride;
    constexpr int HOFF = ILV ? 8 : 64;  // column of the unit's second 16-B half
    const int upsg = n_heads * 8;
    const int units = n_seg * upsg;
    const int dim = n_heads * 128;
    const int srow = src_rows ? src_rows[row] : row;
    const bf16_t* s = src + (int64_t)srow * ld_src;
    int col[UPL];
    u32x4 lo[UPL], hi[UPL];
#pragma unroll
    for (int u = 0; u < UPL; ++u) {
        const int unit = lane + 64 * u;
        col[u] = (unit / upsg) * dim + ((unit % upsg) >> 3) * 128 + (ILV ? 16 : 8) * (unit & 7);
        if (unit < units) {
            lo[u] = *reinterpret_cast<const u32x4*>(s + col[u]);
            hi[u] = *reinterpret_cast<const u32x4*>(s + col[u] + HOFF);
        }
    }
    float ang = 0.f;
    if (pos && lane < 9 * n_freqs) ang = pos[(int64_t)(row / pos_div) * ld_pos + lane / n_freqs] * freqs[lane % n_freqs];
    float4 wl[UPL][2], wh[UPL][2];
#pragma unroll
    for (int u = 0; u < UPL; ++u) {
        if (norm_w && lane + 64 * u < units) {
            const float4* pl = reinterpret_cast<const float4*>(norm_w + col[u]);
            const float4* ph = reinterpret_cast<const float4*>(norm_w + col[u] + HOFF);
            wl[u][0] = pl[0];
            wl[u][1] = pl[1];
            wh[u][0] = ph[0];
            wh[u][1] = ph[1];
        } else {
            wl[u][0] = wl[u][1] = wh[u][0] = wh[u][1] = make_float4(1.f, 1.f, 1.f, 1.f);
        }
    }
    float ss[UPL];
#pragma unroll
    for (int u = 0; u < UPL; ++u) {
        ss[u] = 0.f;
        if (lane + 64 * u < units) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float a0 = __uint_as_float(lo[u][e] << 16), a1 = __uint_as_float(lo[u][e] & 0xffff0000u);
                const float b0 = __uint_as_float(hi[u][e] << 16), b1 = __uint_as_float(hi[u][e] & 0xffff0000u);
                ss[u] += a0 * a0 + a1 * a1 + b0 * b0 + b1 * b1;
            }
        }
    }
    float inv[UPL];
#pragma unroll
    for (int u = 0; u < UPL; ++u) inv[u] = 1.f;
    if (norm_w) {
        for (int sg = 0; sg < n_seg; ++sg) {
            float part = 0.f;
#pragma unroll
            for (int u = 0; u < UPL; ++u) {
                const int unit = lane + 64 * u;
                part += (unit < units && unit / upsg == sg) ? ss[u] : 0.f;
            }
            const float iv = 1.0f / sqrtf(wave_sum(part) / (float)dim + eps);
#pragma unroll
            for (int u = 0; u < UPL; ++u)
                if ((lane + 64 * u) / upsg == sg) inv[u] = iv;
        }
    }
    // segment 0 carries seg0_scale (RoPE is linear): folded into the row scale.  Every group's segment 0 (the
    // documented rf_qk_norm_rope_groups contract), except when the host split one two-segment (q, k) group into two
    // one-segment groups (split_qk): then group 1's segment 0 is k, which is not scaled
    if (!split_qk || blockIdx.y == 0) {
#pragma unroll
        for (int u = 0; u < UPL; ++u)
            if (lane + 64 * u < upsg) inv[u] *= seg0_scale;
    }
    float my_c = 1.f, my_s = 0.f;
    if (pos && lane < 9 * n_freqs) __sincosf(ang, &my_s, &my_c);
    float cs[8], sn[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        cs[k] = pos ? __shfl(my_c, 8 * (lane & 7) + k, 64) : 1.f;
        sn[k] = pos ? __shfl(my_s, 8 * (lane & 7) + k, 64) : 0.f;
    }
    bf16_t* d = dst + (int64_t)row * ld_dst;
#pragma unroll
    for (int u = 0; u < UPL; ++u) {
        if (lane + 64 * u < units) {
            const float wlo[8] = {wl[u][0].x, wl[u][0].y, wl[u][0].z, wl[u][0].w,
                                  wl[u][1].x, wl[u][1].y, wl[u][1].z, wl[u][1].w};
            const float whi[8] = {wh[u][0].x, wh[u][0].y, wh[u][0].z, wh[u][0].w,
                                  wh[u][1].x, wh[u][1].y, wh[u][1].z, wh[u][1].w};
            u32x4 olo, ohi;
            if constexpr (ILV) {  // dword e of lo: pair e, of hi: pair 4 + e, each (x1 low, x2 high)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const uint32_t wd = h ? hi[u][e] : lo[u][e];
                        const float* wv = h ? whi : wlo;
                        const int k = 4 * h + e;
                        const float x0 = __uint_as_float(wd << 16) * inv[u] * wv[2 * e];
                        const float x1 = __uint_as_float(wd & 0xffff0000u) * inv[u] * wv[2 * e + 1];
                        const uint32_t r = pack_bf16x2(x0 * cs[k] - x1 * sn[k], x1 * cs[k] + x0 * sn[k]);
                        if (h) ohi[e] = r;
                        else olo[e] = r;
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float ra[2], rb[2];
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const int i = 2 * e + t;
                        const float a = (t ? __uint_as_float(lo[u][e] & 0xffff0000u) : __uint_as_float(lo[u][e] << 16));
                        const float b = (t ? __uint_as_float(hi[u][e] & 0xffff0000u) : __uint_as_float(hi[u][e] << 16));
                        const float x0 = a * inv[u] * wlo[i], x1 = b * inv[u] * whi[i];
                        ra[t] = x0 * cs[i] - x1 * sn[i];  // rotate_half_hf: (-x2, x1)
                        rb[t] = x1 * cs[i] + x0 * sn[i];
                    }
                    olo[e] = pack_bf16x2(ra[0], ra[1]);
                    ohi[e] = pack_bf16x2(rb[0], rb[1]);
                }
            }
            *reinterpret_cast<u32x4*>(d + col[u]) = olo;
            *reinterpret_cast<u32x4*>(d + col[u] + HOFF) = ohi;
        }
    }
}

// ----------------------------------------------------------------------------- embedding assembly
__global__ __launch_bounds__(256) void embed_kernel(float* __restrict__ out, int64_t ldo,
                                                    const int32_t* __restrict__ out_rows, int rows, int dim,
                                                    const float* __restrict__ base, int base_rows,
                                                    const float* __restrict__ in0, int64_t ld0,
                                                    const float* __restrict__ w0, float eps0,
                                                    const float* __restrict__ in1, int64_t ld1,
                                                    const float* __restrict__ w1, float eps1) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    if (row >= rows) return;
    float s0 = 0.f, s1 = 0.f;
    const float* r0 = in0 ? in0 + (int64_t)row * ld0 : nullptr;
    const float* r1 = in1 ? in1 + (int64_t)row * ld1 : nullptr;
    if (r0) {
        float ss = 0.f;
        for (int c = lane; c < dim; c += 64) ss += r0[c] * r0[c];
        s0 = 1.0f / sqrtf(wave_sum(ss) / (float)dim + eps0);
    }
    if (r1) {
        float ss = 0.f;
        for (int c = lane; c < dim; c += 64) ss += r1[c] * r1[c];
        s1 = 1.0f / sqrtf(wave_sum(ss) / (float)dim + eps1);
    }
    const float* b = base ? base + (int64_t)(row % base_rows) * dim : nullptr;
    float* o = out + (int64_t)(out_rows ? out_rows[row] : row) * ldo;
    for (int c = lane; c < dim; c += 64) {
        // same association as the reference: (token + tex_emb) + vn_emb (renderformer.py:158)
        float v = b ? b[c] : 0.f;
        if (r0) v = v + r0[c] * s0 * w0[c];
        if (r1) v = v + r1[c] * s1 * w1[c];
        o[c] = v;
    }
}

// dim = 256 * NV, 16-B aligned rows: both encoder outputs and the base token row are loaded whole up front
// (NV float4 per lane each, one memory round trip per row), then normed and summed in registers
template <int NV>
__global__ __launch_bounds__(256) void embed_v_kernel(float* __restrict__ out, int64_t ldo,
                                                      const int32_t* __restrict__ out_rows, int rows,
                                                      const float* __restrict__ base, int base_rows,
                                                      const float* __restrict__ in0, int64_t ld0,
                                                      const float* __restrict__ w0, float eps0,
                                                      const float* __restrict__ in1, int64_t ld1,
                                                      const float* __restrict__ w1, float eps1) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int orow = out_rows ? out_rows[row] : row;
    float4 a[NV], b[NV], t[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        a[i] = in0 ? reinterpret_cast<const float4*>(in0 + (int64_t)row * ld0)[lane + 64 * i] : make_float4(0.f, 0.f, 0.f, 0.f);
        b[i] = in1 ? reinterpret_cast<const float4*>(in1 + (int64_t)row * ld1)[lane + 64 * i] : make_float4(0.f, 0.f, 0.f, 0.f);
        t[i] = base ? reinterpret_cast<const float4*>(base + (int64_t)(row % base_rows) * (256 * NV))[lane + 64 * i]
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        s0 += a[i].x * a[i].x + a[i].y * a[i].y + a[i].z * a[i].z + a[i].w * a[i].w;
        s1 += b[i].x * b[i].x + b[i].y * b[i].y + b[i].z * b[i].z + b[i].w * b[i].w;
    }
    s0 = in0 ? 1.0f / sqrtf(wave_sum(s0) / (float)(256 * NV) + eps0) : 0.f;
    s1 = in1 ? 1.0f / sqrtf(wave_sum(s1) / (float)(256 * NV) + eps1) : 0.f;
    float4* o = reinterpret_cast<float4*>(out + (int64_t)orow * ldo);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        // same association as the reference: (token + tex_emb) + vn_emb (renderformer.py:158)
        float4 v = t[i];
        if (in0) {
            const float4 g = reinterpret_cast<const float4*>(w0)[lane + 64 * i];
            v.x = v.x + a[i].x * s0 * g.x;
            v.y = v.y + a[i].y * s0 * g.y;
            v.z = v.z + a[i].z * s0 * g.z;
            v.w = v.w + a[i].w * s0 * g.w;
        }
        if (in1) {
            const float4 g = reinterpret_cast<const float4*>(w1)[lane + 64 * i];
            v.x = v.x + b[i].x * s1 * g.x;
            v.y = v.y + b[i].y * s1 * g.y;
            v.z = v.z + b[i].z * s1 * g.z;
            v.w = v.w + b[i].w * s1 * g.w;
        }
        o[lane + 64 * i] = v;
    }
}

}  // namespace

namespace {
template <bool F16>
int rmsnorm_launch(const float* x, int64_t ldx, const float* weight, float eps, void* out, int64_t ldo, int rows,
                   int dim, void* stream, const char* what) {
    RF_REQUIRE(x && weight && out, "%s: null pointer", what);
    RF_REQUIRE(dim % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0, "%s: dim/ld must be multiples of 4", what);
    if (rows <= 0) return RF_OK;
    const dim3 grid((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK);
    hipStream_t st = (hipStream_t)stream;
    const bool al = ((uintptr_t)x & 15) == 0 && ((uintptr_t)weight & 15) == 0 && ((uintptr_t)out & 7) == 0;
    static const bool generic = getenv("RF_RMSNORM_GENERIC") && atoi(getenv("RF_RMSNORM_GENERIC"));  // A/B only
    bf16_t* o = (bf16_t*)out;
    int* rg = F16 ? rf::range_word() : nullptr;  // fp16 out: raise the range flag on |x| > 65504 / NaN
    switch (al && !generic && dim % 256 == 0 ? dim / 256 : 0) {
        case 2: RF_LAUNCH((rmsnorm_v_kernel<2, F16>), grid, dim3(256), 0, st, x, ldx, weight, eps, o, ldo, rows, rg); break;
        case 3: RF_LAUNCH((rmsnorm_v_kernel<3, F16>), grid, dim3(256), 0, st, x, ldx, weight, eps, o, ldo, rows, rg); break;
        case 4: RF_LAUNCH((rmsnorm_v_kernel<4, F16>), grid, dim3(256), 0, st, x, ldx, weight, eps, o, ldo, rows, rg); break;
        case 6: RF_LAUNCH((rmsnorm_v_kernel<6, F16>), grid, dim3(256), 0, st, x, ldx, weight, eps, o, ldo, rows, rg); break;
        case 8: RF_LAUNCH((rmsnorm_v_kernel<8, F16>), grid, dim3(256), 0, st, x, ldx, weight, eps, o, ldo, rows, rg); break;
        default:
            RF_LAUNCH(rmsnorm_kernel<F16>, grid, dim3(256), 0, st, x, ldx, weight, eps, o, ldo, rows, dim, rg);
    }
    return rf::check_launch(what);
}
}  // namespace

extern "C" int rf_rmsnorm(const float* x, int64_t ldx, const float* weight, float eps, void* out, int64_t ldo,
                          int rows, int dim, void* stream) {
    return rmsnorm_launch<false>(x, ldx, weight, eps, out, ldo, rows, dim, stream, "rf_rmsnorm");
}

extern "C" int rf_rmsnorm_f16(const float* x, int64_t ldx, const float* weight, float eps, void* out, int64_t ldo,
                              int rows, int dim, void* stream) {
    return rmsnorm_launch<true>(x, ldx, weight, eps, out, ldo, rows, dim, stream, "rf_rmsnorm_f16");
}

extern "C" int rf_prenorm(const float* x, int64_t ldx, const float* norm_w, void* xg, int64_t ldxg, float* ss,
                          int rows, int dim, int operand_dtype, void* stream) {
    RF_REQUIRE(x && norm_w && xg && ss, "rf_prenorm: null pointer");
    RF_REQUIRE(operand_dtype == RF_DT_F16 || operand_dtype == RF_DT_BF16, "rf_prenorm: operand_dtype");
    RF_REQUIRE(dim > 0 && dim % 4 == 0 && ldx % 4 == 0 && ldxg % 4 == 0 && ldx >= dim && ldxg >= dim,
               "rf_prenorm: dim / ld must be multiples of 4 (ld >= dim)");
    RF_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)norm_w & 15) == 0 && ((uintptr_t)xg & 7) == 0 &&
                   ((uintptr_t)ss & 15) == 0,
               "rf_prenorm: x / norm_w / ss 16-B and xg 8-B aligned");
    if (rows <= 0) return RF_OK;
    const dim3 grid((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK);
    hipStream_t st = (hipStream_t)stream;
    if (operand_dtype == RF_DT_F16)
        RF_LAUNCH(prenorm_kernel<true>, grid, dim3(256), 0, st, x, ldx, norm_w, (bf16_t*)xg, ldxg, ss, rows, dim,
                  rf::range_word());
    else
        RF_LAUNCH(prenorm_kernel<false>, grid, dim3(256), 0, st, x, ldx, norm_w, (bf16_t*)xg, ldxg, ss, rows, dim,
                  nullptr);
    return rf::check_launch("rf_prenorm");
}

static int qk_norm_rope_groups(const void* src, int64_t ld_src, int64_t src_gstride, void* dst, int64_t ld_dst,
                               int64_t dst_gstride, const int32_t* src_rows, int rows, int dim, int n_heads, int n_seg,
                               int n_groups, const float* norm_w, int64_t w_gstride, float eps, float seg0_scale,
                               const float* pos, int64_t ld_pos, int pos_div, const float* freqs, int n_freqs,
                               void* stream, bool ilv);

extern "C" int rf_qk_norm_rope_groups(const void* src, int64_t ld_src, int64_t src_gstride, void* dst, int64_t ld_dst,
                                      int64_t dst_gstride, const int32_t* src_rows, int rows, int dim, int n_heads,
                                      int n_seg, int n_groups, const float* norm_w, int64_t w_gstride, float eps,
                                      float seg0_scale, const float* pos, int64_t ld_pos, int pos_div,
                                      const float* freqs, int n_freqs, void* stream) {
    return qk_norm_rope_groups(src, ld_src, src_gstride, dst, ld_dst, dst_gstride, src_rows, rows, dim, n_heads, n_seg,
                               n_groups, norm_w, w_gstride, eps, seg0_scale, pos, ld_pos, pos_div, freqs, n_freqs,
                               stream, false);
}

extern "C" int rf_qk_norm_rope_groups_ilv(const void* src, int64_t ld_src, int64_t src_gstride, void* dst,
                                          int64_t ld_dst, int64_t dst_gstride, const int32_t* src_rows, int rows,
                                          int dim, int n_heads, int n_seg, int n_groups, const float* norm_w,
                                          int64_t w_gstride, float eps, float seg0_scale, const float* pos,
                                          int64_t ld_pos, int pos_div, const float* freqs, int n_freqs, void* stream) {
    return qk_norm_rope_groups(src, ld_src, src_gstride, dst, ld_dst, dst_gstride, src_rows, rows, dim, n_heads, n_seg,
                               n_groups, norm_w, w_gstride, eps, seg0_scale, pos, ld_pos, pos_div, freqs, n_freqs,
                               stream, true);
}

static int qk_norm_rope_groups(const void* src, int64_t ld_src, int64_t src_gstride, void* dst, int64_t ld_dst,
                               int64_t dst_gstride, const int32_t* src_rows, int rows, int dim, int n_heads, int n_seg,
                               int n_groups, const float* norm_w, int64_t w_gstride, float eps, float seg0_scale,
                               const float* pos, int64_t ld_pos, int pos_div, const float* freqs, int n_freqs,
                               void* stream, bool ilv) {
    RF_REQUIRE(src && dst, "rf_qk_norm_rope: null pointer");
    RF_REQUIRE(dim == n_heads * 128 && n_seg >= 1 && n_seg * n_heads * 8 <= MAX_UNITS,
               "rf_qk_norm_rope: need head_dim 128 and n_seg*n_heads <= %d", MAX_UNITS / 8);
    RF_REQUIRE(ld_src % 8 == 0 && ld_dst % 8 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0,
               "rf_qk_norm_rope: rows must be 16-B aligned");
    RF_REQUIRE(n_groups >= 1 && n_groups <= 65535 && src_gstride % 8 == 0 && dst_gstride % 8 == 0 && w_gstride % 4 == 0,
               "rf_qk_norm_rope: bad group count/strides (16-B aligned group offsets)");
    RF_REQUIRE(!pos || (freqs && n_freqs > 0 && 9 * n_freqs <= 64 && pos_div > 0),
               "rf_qk_norm_rope: rope needs freqs with 9*n_freqs <= 64");
    if (rows <= 0) return RF_OK;
    RF_REQUIRE(!norm_w || ((uintptr_t)norm_w & 15) == 0, "rf_qk_norm_rope: norm weights must be 16-B aligned");
    const int blocks = (rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
    static const bool loop = getenv("RF_QKN_LOOP") && atoi(getenv("RF_QKN_LOOP"));  // A/B only
    int units = n_seg * n_heads * 8;
    hipStream_t st = (hipStream_t)stream;
    if (loop && !ilv) {  // the grid-stride kernel, one launch per group (standard layout only)
        const dim3 grid(blocks > 2048 ? 2048 : blocks);
        for (int g = 0; g < n_groups; ++g) {
            const bf16_t* s = (const bf16_t*)src + g * src_gstride;
            bf16_t* d = (bf16_t*)dst + g * dst_gstride;
            const float* w = norm_w ? norm_w + g * w_gstride : nullptr;
#define RF_QKL(U)                                                                                                 \
    RF_LAUNCH(qk_norm_rope_kernel<U>, grid, dim3(256), 0, st, s, ld_src, d, ld_dst, src_rows, rows,      \
                       n_heads, n_seg, w, eps, seg0_scale, pos, ld_pos, pos_div, freqs, n_freqs)
            if (units <= 64) RF_QKL(1);
            else if (units <= 128) RF_QKL(2);
            else RF_QKL(4);
#undef RF_QKL
        }
        return rf::check_launch("rf_qk_norm_rope");
    }
    // q and k of one row as two groups of one segment (grid.y = 2, the one-unit-per-lane kernel: 57 VGPRs, 8 waves per
    // SIMD) instead of one wave with both (95 VGPRs, 5 waves per SIMD: the stage-1 grid of 5,649 rows then needs a
    // second round); the per-segment sums and the arithmetic are the same, so the results are bit-identical.
    // RF_QKN_SPLIT=0 keeps the two-segment wave (A/B)
    const char* split_env = getenv("RF_QKN_SPLIT");
    int split_qk = 0;
    if (n_seg == 2 && n_groups == 1 && (!split_env || atoi(split_env) != 0)) {
        split_qk = 1;
        n_seg = 1;
        n_groups = 2;
        src_gstride = dst_gstride = dim;
        w_gstride = dim;
    }
    const dim3 grid(blocks, n_groups);
#define RF_QKN(U)                                                                                                 \
    if (ilv)                                                                                                      \
        RF_LAUNCH((qk_norm_rope_row_kernel<U, true>), grid, dim3(256), 0, st, (const bf16_t*)src, ld_src,          \
                  (bf16_t*)dst, ld_dst, src_rows, rows, n_heads, n_seg, norm_w, eps, seg0_scale, pos, ld_pos, pos_div, \
                  freqs, n_freqs, src_gstride, dst_gstride, (int)w_gstride, split_qk);                             \
    else                                                                                                          \
        RF_LAUNCH((qk_norm_rope_row_kernel<U, false>), grid, dim3(256), 0, st, (const bf16_t*)src, ld_src,         \
                  (bf16_t*)dst, ld_dst, src_rows, rows, n_heads, n_seg, norm_w, eps, seg0_scale, pos, ld_pos, pos_div, \
                  freqs, n_freqs, src_gstride, dst_gstride, (int)w_gstride, split_qk)
    units = n_seg * n_heads * 8;
    if (units <= 64) {
        RF_QKN(1);
    } else if (units <= 128) {
        RF_QKN(2);
    } else {
        RF_QKN(4);
    }
#undef RF_QKN
    return rf::check_launch("rf_qk_norm_rope");
}

extern "C" int rf_qk_norm_rope(const void* src, int64_t ld_src, void* dst, int64_t ld_dst, const int32_t* src_rows,
                               int rows, int dim, int n_heads, int n_seg, const float* norm_w, float eps,
                               float seg0_scale, const float* pos, int64_t ld_pos, int pos_div, const float* freqs, int n_freqs,
                               void* stream) {
    return rf_qk_norm_rope_groups(src, ld_src, 0, dst, ld_dst, 0, src_rows, rows, dim, n_heads, n_seg, 1, norm_w, 0, eps,
                                  seg0_scale, pos, ld_pos, pos_div, freqs, n_freqs, stream);
}

extern "C" int rf_embed(float* out, int64_t ldo, const int32_t* out_rows, int rows, int dim, const float* base,
                        int base_rows, const float* in0, int64_t ld0, const float* w0, float eps0, const float* in1,
                        int64_t ld1, const float* w1, float eps1, void* stream) {
    RF_REQUIRE(out, "rf_embed: null output");
    RF_REQUIRE((!in0 || w0) && (!in1 || w1), "rf_embed: input without norm weight");
    RF_REQUIRE(!base || base_rows > 0, "rf_embed: base_rows must be > 0");
    if (rows <= 0) return RF_OK;
    const dim3 grid((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK);
    hipStream_t st = (hipStream_t)stream;
    auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    const bool vec = dim % 256 == 0 && ldo % 4 == 0 && ld0 % 4 == 0 && ld1 % 4 == 0 && al(out) && al(base) &&
                     al(in0) && al(w0) && al(in1) && al(w1);
#define RF_EMB(NV)                                                                                                \
    RF_LAUNCH(embed_v_kernel<NV>, grid, dim3(256), 0, st, out, ldo, out_rows, rows, base, base_rows, in0, \
                       ld0, w0, eps0, in1, ld1, w1, eps1)
    switch (vec ? dim / 256 : 0) {
        case 3: RF_EMB(3); break;
        case 4: RF_EMB(4); break;
        case 6: RF_EMB(6); break;
        case 8: RF_EMB(8); break;
        default:
            RF_LAUNCH(embed_kernel, grid, dim3(256), 0, st, out, ldo, out_rows, rows, dim, base, base_rows,
                               in0, ld0, w0, eps0, in1, ld1, w1, eps1);
    }
#undef RF_EMB
    return rf::check_launch("rf_embed");
}

// ----------------------------------------------------------------------------- row RMS scale (rf.h)
// x[r][0:dim] *= scale / sqrt(sum_{s < 8} ss[r * ld_ss + s] / dim + eps), bf16 in place: the keys' 1 / rms after
// rf_gemm_qk_rope (which applied the norm weight and the rotation in its epilogue and wrote the row's partial sums
// of squares).  One row per wave, every load of the row issued before any use (one round trip).
template <int UPL>
__global__ __launch_bounds__(256) void row_rms_scale_kernel(bf16_t* x, int64_t ldx, int rows, int dim,
                                                            const float* __restrict__ ss, int64_t ld_ss, float eps,
                                                            float scale) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    if (row >= rows) return;
    bf16_t* r = x + (int64_t)row * ldx;
    u32x4 v[UPL];
#pragma unroll
    for (int u = 0; u < UPL; ++u)
        if (8 * (lane + 64 * u) < dim) v[u] = *reinterpret_cast<const u32x4*>(r + 8 * (lane + 64 * u));
    const float part = lane < 8 ? ss[(int64_t)row * ld_ss + lane] : 0.f;
    const float f = scale / sqrtf(wave_sum(part) / (float)dim + eps);
#pragma unroll
    for (int u = 0; u < UPL; ++u) {
        if (8 * (lane + 64 * u) < dim) {
            u32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                o[e] = pack_bf16x2(__uint_as_float(v[u][e] << 16) * f, __uint_as_float(v[u][e] & 0xffff0000u) * f);
            *reinterpret_cast<u32x4*>(r + 8 * (lane + 64 * u)) = o;
        }
    }
}

extern "C" int rf_row_rms_scale(void* x, int64_t ldx, int rows, int dim, const float* ss, int64_t ld_ss, float eps,
                                float scale, void* stream) {
    RF_REQUIRE(x && ss, "rf_row_rms_scale: null pointer");
    RF_REQUIRE(dim > 0 && dim % 8 == 0 && dim <= 4 * 512 && ldx >= dim && ldx % 8 == 0 && ((uintptr_t)x & 15) == 0,
               "rf_row_rms_scale: dim must be a multiple of 8 up to 2048 with 16-B aligned rows");
    RF_REQUIRE(ld_ss >= 8, "rf_row_rms_scale: ld_ss must be >= 8 (RF_PRENORM_SLOTS partial sums a row)");
    if (rows <= 0) return RF_OK;
    const int blocks = (rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
    hipStream_t st = (hipStream_t)stream;
    if (dim <= 512)
        RF_LAUNCH(row_rms_scale_kernel<1>, dim3(blocks), dim3(256), 0, st, (bf16_t*)x, ldx, rows, dim, ss, ld_ss, eps, scale);
    else if (dim <= 1024)
        RF_LAUNCH(row_rms_scale_kernel<2>, dim3(blocks), dim3(256), 0, st, (bf16_t*)x, ldx, rows, dim, ss, ld_ss, eps, scale);
    else
        RF_LAUNCH(row_rms_scale_kernel<4>, dim3(blocks), dim3(256), 0, st, (bf16_t*)x, ldx, rows, dim, ss, ld_ss, eps, scale);
    return rf::check_launch("rf_row_rms_scale");
}
