// DPT helpers around the GEMM engine: fp32 -> bf16 hi/lo activation planes and the
// align_corners bilinear resize (dpt.py:154-155), both NHWC.
//
// Activations consumed by a DPT convolution live as two bf16 planes hi = bf16(x),
// lo = bf16(x - hi) (optionally of silu(x): the ResidualConvUnit pre-activation,
// dpt.py:86-89, applied once per element instead of once per filter tap).  With p_lo == NULL the
// activation is stored as ONE fp16 plane in p_hi instead (the fp16-operand DPT mode).
#include <math.h>

#include "common.h"

namespace {


// returns max |value| written to an fp16 plane (0 for hi/lo planes): the range flag's input
RF_DEV float store_split4(bf16_t* p_hi, bf16_t* p_lo, int64_t off, float4 v, bool act) {
    float x[4] = {v.x, v.y, v.z, v.w};
    if (!p_lo) {
        if (act) {
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] = silu(x[e]);
        }
        *reinterpret_cast<uint2*>(p_hi + off) = make_uint2(pack_f16x2(x[0], x[1]), pack_f16x2(x[2], x[3]));
        return amax3(amax3(0.f, x[0], x[1]), x[2], x[3]);
    }
    uint32_t h[2], l[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        float a0 = x[2 * e], a1 = x[2 * e + 1];
        if (act) {
            a0 = silu(a0);
            a1 = silu(a1);
        }
        const bf16_t h0 = f32_to_bf16(a0), h1 = f32_to_bf16(a1);
        h[e] = (uint32_t)h0 | ((uint32_t)h1 << 16);
        l[e] = pack_bf16x2(a0 - bf16_to_f32(h0), a1 - bf16_to_f32(h1));
    }
    *reinterpret_cast<uint2*>(p_hi + off) = make_uint2(h[0], h[1]);
    *reinterpret_cast<uint2*>(p_lo + off) = make_uint2(l[0], l[1]);
    return 0.f;
}

__global__ __launch_bounds__(256) void split_kernel(const float* __restrict__ x, int rows, int c, int64_t ldx,
                                                    bf16_t* __restrict__ p_hi, bf16_t* __restrict__ p_lo, int p_ld,
                                                    int act, int* range) {
    const int c4 = c / 4;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;  // rows * c4 < 2^31 (host check)
    if (i >= rows * c4) return;
    const int r32 = i / c4;
    const int64_t r = r32;
    const int cc = (i - r32 * c4) * 4;
    const float am = store_split4(p_hi, p_lo, r * p_ld + cc, *reinterpret_cast<const float4*>(x + r * ldx + cc), act);
    // one fp16 plane (p_lo == NULL): the decoder taps cast to fp16 must fit its range
    if (range && !f16_in_range(am)) report_f16_range(range, RF_RANGE_CONV);
}

// bilinear, align_corners=True (torch upsample_bilinear2d); scale passed from the host.  One block row per
// output image row (blockIdx.y = img * ho + oy, uniform), threads over (ox, 4-channel group) with 32-bit
// index math (the flat 64-bit div/mod chain cost more than the memory traffic)
__global__ __launch_bounds__(256) void upsample_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                       bf16_t* __restrict__ p_hi, bf16_t* __restrict__ p_lo, int p_ld,
                                                       int hi, int wi, int c, int ho, int wo, float sh, float sw) {
    const int c4n = c >> 2;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= wo * c4n) return;
    const int row = blockIdx.y;  // img * ho + oy
    const int img = row / ho, oy = row - img * ho;
    const int ox = i / c4n;
    const int cc = (i - ox * c4n) * 4;
    const float fy = sh * (float)oy, fx = sw * (float)ox;
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = y0 + (y0 < hi - 1 ? 1 : 0), x1 = x0 + (x0 < wi - 1 ? 1 : 0);
    const float ly1 = fy - (float)y0, lx1 = fx - (float)x0;
    const float ly0 = 1.0f - ly1, lx0 = 1.0f - lx1;
    const float* base = in + (int64_t)img * hi * wi * c + cc;
    const float4 a = *reinterpret_cast<const float4*>(base + (int64_t)(y0 * wi + x0) * c);
    const float4 b = *reinterpret_cast<const float4*>(base + (int64_t)(y0 * wi + x1) * c);
    const float4 d = *reinterpret_cast<const float4*>(base + (int64_t)(y1 * wi + x0) * c);
    const float4 e = *reinterpret_cast<const float4*>(base + (int64_t)(y1 * wi + x1) * c);
    float4 r;
    r.x = ly0 * (lx0 * a.x + lx1 * b.x) + ly1 * (lx0 * d.x + lx1 * e.x);
    r.y = ly0 * (lx0 * a.y + lx1 * b.y) + ly1 * (lx0 * d.y + lx1 * e.y);
    r.z = ly0 * (lx0 * a.z + lx1 * b.z) + ly1 * (lx0 * d.z + lx1 * e.z);
    r.w = ly0 * (lx0 * a.w + lx1 * b.w) + ly1 * (lx0 * d.w + lx1 * e.w);
    const int64_t pix = (int64_t)row * wo + ox;
    if (out) *reinterpret_cast<float4*>(out + pix * c + cc) = r;
    if (p_hi) store_split4(p_hi, p_lo, pix * p_ld + cc, r, false);
}

// The same with 8 channels per thread (c % 8 == 0): 16-B fp16 plane stores and half the index math per
// output element; the arithmetic per channel is identical, so results are bit-identical to upsample_kernel
__global__ __launch_bounds__(256) void upsample8_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                        bf16_t* __restrict__ p_hi, bf16_t* __restrict__ p_lo, int p_ld,
                                                        int hi, int wi, int c, int ho, int wo, float sh, float sw) {
    const int c8n = c >> 3;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= wo * c8n) return;
    const int row = blockIdx.y;  // img * ho + oy
    const int img = row / ho, oy = row - img * ho;
    const int ox = i / c8n;
    const int cc = (i - ox * c8n) * 8;
    const float fy = sh * (float)oy, fx = sw * (float)ox;
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = y0 + (y0 < hi - 1 ? 1 : 0), x1 = x0 + (x0 < wi - 1 ? 1 : 0);
    const float ly1 = fy - (float)y0, lx1 = fx - (float)x0;
    const float ly0 = 1.0f - ly1, lx0 = 1.0f - lx1;
    const float* base = in + (int64_t)img * hi * wi * c + cc;
    const float4* pa = reinterpret_cast<const float4*>(base + (int64_t)(y0 * wi + x0) * c);
    const float4* pb = reinterpret_cast<const float4*>(base + (int64_t)(y0 * wi + x1) * c);
    const float4* pd = reinterpret_cast<const float4*>(base + (int64_t)(y1 * wi + x0) * c);
    const float4* pe = reinterpret_cast<const float4*>(base + (int64_t)(y1 * wi + x1) * c);
    float4 a[2], b[2], d[2], e[2], r[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        a[h] = pa[h];
        b[h] = pb[h];
        d[h] = pd[h];
        e[h] = pe[h];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        r[h].x = ly0 * (lx0 * a[h].x + lx1 * b[h].x) + ly1 * (lx0 * d[h].x + lx1 * e[h].x);
        r[h].y = ly0 * (lx0 * a[h].y + lx1 * b[h].y) + ly1 * (lx0 * d[h].y + lx1 * e[h].y);
        r[h].z = ly0 * (lx0 * a[h].z + lx1 * b[h].z) + ly1 * (lx0 * d[h].z + lx1 * e[h].z);
        r[h].w = ly0 * (lx0 * a[h].w + lx1 * b[h].w) + ly1 * (lx0 * d[h].w + lx1 * e[h].w);
    }
    const int64_t pix = (int64_t)row * wo + ox;
    if (out) {
        float4* o = reinterpret_cast<float4*>(out + pix * c + cc);
        o[0] = r[0];
        o[1] = r[1];
    }
    if (p_hi && !p_lo) {
        *reinterpret_cast<uint4*>(p_hi + pix * p_ld + cc) =
            make_uint4(pack_f16x2(r[0].x, r[0].y), pack_f16x2(r[0].z, r[0].w), pack_f16x2(r[1].x, r[1].y),
                       pack_f16x2(r[1].z, r[1].w));
    } else if (p_hi) {
        store_split4(p_hi, p_lo, pix * p_ld + cc, r[0], false);
        store_split4(p_hi, p_lo, pix * p_ld + cc + 4, r[1], false);
    }
}

// fp16 plane in (channel stride in_ld) -> fp16 plane out, 8 channels per thread, the blend of upsample8_kernel
__global__ __launch_bounds__(256) void upsample8h_kernel(const uint16_t* __restrict__ in, int in_ld,
                                                         uint16_t* __restrict__ p_out, int p_ld, int hi, int wi, int c,
                                                         int ho, int wo, float sh, float sw) {
    const int c8n = c >> 3;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= wo * c8n) return;
    const int row = blockIdx.y;  // img * ho + oy
    const int img = row / ho, oy = row - img * ho;
    const int ox = i / c8n;
    const int cc = (i - ox * c8n) * 8;
    const float fy = sh * (float)oy, fx = sw * (float)ox;
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = y0 + (y0 < hi - 1 ? 1 : 0), x1 = x0 + (x0 < wi - 1 ? 1 : 0);
    const float ly1 = fy - (float)y0, lx1 = fx - (float)x0;
    const float ly0 = 1.0f - ly1, lx0 = 1.0f - lx1;
    const uint16_t* base = in + (int64_t)img * hi * wi * in_ld + cc;
    const uint4 qa = *reinterpret_cast<const uint4*>(base + (int64_t)(y0 * wi + x0) * in_ld);
    const uint4 qb = *reinterpret_cast<const uint4*>(base + (int64_t)(y0 * wi + x1) * in_ld);
    const uint4 qd = *reinterpret_cast<const uint4*>(base + (int64_t)(y1 * wi + x0) * in_ld);
    const uint4 qe = *reinterpret_cast<const uint4*>(base + (int64_t)(y1 * wi + x1) * in_ld);
    const uint32_t wa[4] = {qa.x, qa.y, qa.z, qa.w}, wb[4] = {qb.x, qb.y, qb.z, qb.w};
    const uint32_t wd[4] = {qd.x, qd.y, qd.z, qd.w}, we[4] = {qe.x, qe.y, qe.z, qe.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float r[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float a = f16_bits_to_f32((uint16_t)(wa[k] >> (16 * h))), b = f16_bits_to_f32((uint16_t)(wb[k] >> (16 * h)));
            const float d = f16_bits_to_f32((uint16_t)(wd[k] >> (16 * h))), e = f16_bits_to_f32((uint16_t)(we[k] >> (16 * h)));
            r[h] = ly0 * (lx0 * a + lx1 * b) + ly1 * (lx0 * d + lx1 * e);
        }
        o[k] = pack_f16x2(r[0], r[1]);
    }
    *reinterpret_cast<uint4*>(p_out + ((int64_t)row * wo + ox) * p_ld + cc) = make_uint4(o[0], o[1], o[2], o[3]);
}

}  // namespace

extern "C" int rf_upsample_bilinear_h(const void* in, int in_ld, int n_img, int hi, int wi, int c, int ho, int wo,
                                      void* p_out, int p_ld, void* stream) {
    RF_REQUIRE(in && p_out, "rf_upsample_bilinear_h: null pointer");
    RF_REQUIRE(c % 8 == 0 && in_ld % 8 == 0 && p_ld % 8 == 0 && in_ld >= c && p_ld >= c,
               "rf_upsample_bilinear_h: bad widths (c, in_ld, p_ld multiples of 8)");
    RF_REQUIRE(((uintptr_t)in & 15) == 0 && ((uintptr_t)p_out & 15) == 0, "rf_upsample_bilinear_h: 16-B alignment");
    if ((int64_t)n_img * ho * wo <= 0) return RF_OK;
    RF_REQUIRE((int64_t)wo * (c / 8) < (1 << 30) && (int64_t)n_img * ho < 65536 && (int64_t)hi * wi < (1 << 30),
               "rf_upsample_bilinear_h: image too large");
    const float sh = ho > 1 ? (float)(hi - 1) / (float)(ho - 1) : 0.f;
    const float sw = wo > 1 ? (float)(wi - 1) / (float)(wo - 1) : 0.f;
    const dim3 grid((unsigned)((wo * (c / 8) + 255) / 256), (unsigned)(n_img * ho));
    RF_LAUNCH(upsample8h_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const uint16_t*)in, in_ld,
              (uint16_t*)p_out, p_ld, hi, wi, c, ho, wo, sh, sw);
    return rf::check_launch("rf_upsample_bilinear_h");
}

extern "C" int rf_split_planes(const float* x, int64_t rows, int c, int64_t ldx, void* p_hi, void* p_lo, int p_ld,
                               int silu_act, void* stream) {
    RF_REQUIRE(x && p_hi, "rf_split_planes: null pointer");
    RF_REQUIRE(c % 4 == 0 && ldx % 4 == 0 && p_ld % 4 == 0 && p_ld >= c, "rf_split_planes: bad widths");
    const int64_t n = rows * (c / 4);
    if (n <= 0) return RF_OK;
    RF_REQUIRE(n < (1ll << 31) - 256, "rf_split_planes: too many elements");
    RF_LAUNCH(split_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, (int)rows, c,
                       ldx, (bf16_t*)p_hi, (bf16_t*)p_lo, p_ld, silu_act, p_lo ? nullptr : rf::range_word());
    return rf::check_launch("rf_split_planes");
}

extern "C" int rf_upsample_bilinear(const float* in, int n_img, int hi, int wi, int c, float* out, int ho, int wo,
                                    void* p_hi, void* p_lo, int p_ld, void* stream) {
    RF_REQUIRE(in && (out || p_hi), "rf_upsample_bilinear: null pointer");
    RF_REQUIRE(c % 4 == 0 && (!p_hi || (p_ld % 4 == 0 && p_ld >= c)), "rf_upsample_bilinear: bad widths");
    const int64_t total = (int64_t)n_img * ho * wo * (c / 4);
    if (total <= 0) return RF_OK;
    RF_REQUIRE((int64_t)wo * (c / 4) < (1 << 30) && (int64_t)n_img * ho < 65536 && (int64_t)hi * wi < (1 << 30),
               "rf_upsample_bilinear: image too large");
    // scale computed on the host with IEEE float division, as aten's area_pixel_compute_scale<float>
    const float sh = ho > 1 ? (float)(hi - 1) / (float)(ho - 1) : 0.f;
    const float sw = wo > 1 ? (float)(wi - 1) / (float)(wo - 1) : 0.f;
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (c % 8 == 0 && (!p_hi || p_ld % 8 == 0) && al16(in) && al16(out) && al16(p_hi) && al16(p_lo)) {
        const dim3 grid((unsigned)((wo * (c / 8) + 255) / 256), (unsigned)(n_img * ho));
        RF_LAUNCH(upsample8_kernel, grid, dim3(256), 0, (hipStream_t)stream, in, out, (bf16_t*)p_hi,
                           (bf16_t*)p_lo, p_ld, hi, wi, c, ho, wo, sh, sw);
    } else {
        const dim3 grid((unsigned)((wo * (c / 4) + 255) / 256), (unsigned)(n_img * ho));
        RF_LAUNCH(upsample_kernel, grid, dim3(256), 0, (hipStream_t)stream, in, out, (bf16_t*)p_hi,
                           (bf16_t*)p_lo, p_ld, hi, wi, c, ho, wo, sh, sw);
    }
    return rf::check_launch("rf_upsample_bilinear");
}
