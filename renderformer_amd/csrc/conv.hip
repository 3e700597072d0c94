// DPT decode convolutions for gfx950: NHWC implicit-GEMM on bf16 MFMA with a
// three-term bf16 split ("bf16x3") so the head keeps fp32-level accuracy.
//
// The DPT head must stay at fp32 precision (a plain bf16 DPT costs 2.0e-3
// relative L2 on its own, SURVEY Appendix C, over the 1e-3 budget).  Exact fp32
// MFMA runs at 1/16 of the bf16 rate; instead every fp32 operand x is split into
// hi = bf16(x) and lo = bf16(x - hi) and a.b ~= ah.bh + ah.bl + al.bh (the dropped
// al.bl term is ~2^-16 relative), i.e. three bf16 MFMAs per product, 5.3x the
// fp32-MFMA rate at ~1e-5 relative error per dot product.  Weights are split once
// on the host; activations are split while staging the A tile (fused with the
// RCU pre-activation SiLU).
//
// GEMM view: M = output pixels (img, oy, ox), N = output channels, K = (ky, kx, ci)
// with ci padded to a multiple of 64 so a 64-wide K step is one filter tap.
// Epilogues fuse bias, up to two residual adds (RCU skip + fusion-block sum),
// SiLU, the ConvTranspose k=s pixel scatter, and — for the last 3x3 conv — the
// SiLU -> 1x1 (32 -> 3) -> ELU(1e-3) -> 10^x - 1 head so the 32-channel
// full-resolution tensor never reaches HBM.
//
// Tile BM=128 pixels x BN (128 or 32) channels x BK=64, 256 threads, one LDS
// buffer (64 KiB at BN=128) with register staging: the next K step's loads are
// issued before this step's MFMAs and written after the barrier.
#include <math.h>

#include "common.h"

namespace {

constexpr int BM = 128, BK = 64, THREADS = 256;

struct ConvArgs {
    const float* in;
    const bf16_t* w_hi;
    const bf16_t* w_lo;
    const float* bias;
    const float* res1;
    const float* res2;
    float* out;
    const float* w_fin;
    const float* b_fin;
    int n_img, hi, wi, cin, cin_pad;
    int ho, wo, kw, stride, pad;
    int cout, m, k, deconv;  // deconv > 0: ConvTranspose with kernel = stride = deconv (1x1 GEMM + scatter)
    int flags, n_fin;
    float elu_alpha;
};

RF_DEV int swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

RF_DEV float silu(float x) { return x / (1.0f + expf(-x)); }

RF_DEV void split_store(char* hi_tile, char* lo_tile, int row, int col4, float4 v) {
    // col4 = index of a 4-channel group in the 64-wide K step: 16-B chunk col4/2, half col4&1
    const float x[4] = {v.x, v.y, v.z, v.w};
    uint32_t h[2], l[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const bf16_t h0 = f32_to_bf16(x[2 * e]), h1 = f32_to_bf16(x[2 * e + 1]);
        const float r0 = x[2 * e] - bf16_to_f32(h0), r1 = x[2 * e + 1] - bf16_to_f32(h1);
        h[e] = (uint32_t)h0 | ((uint32_t)h1 << 16);
        l[e] = pack_bf16x2(r0, r1);
    }
    const int off = swz(row, col4 >> 1) + (col4 & 1) * 8;
    *reinterpret_cast<uint2*>(hi_tile + off) = make_uint2(h[0], h[1]);
    *reinterpret_cast<uint2*>(lo_tile + off) = make_uint2(l[0], l[1]);
}

template <int BN>
__global__ __launch_bounds__(THREADS, 2) void conv_bf16x3_kernel(ConvArgs p) {
    constexpr int WN = BN >= 64 ? BN / 64 : 1;       // waves along N
    constexpr int WM = 4 / WN;                         // waves along M
    constexpr int MW = BM / WM, NW = BN / WN;          // per-wave tile
    constexpr int TI = MW / 16, TJ = NW / 16;
    constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
    constexpr int A_F4 = BM * BK / 4 / THREADS;        // float4 per thread per K step (8)
    constexpr int B_CH = BN * BK / 8 / THREADS;        // 16-B chunks per thread per operand (4 or 1)
    static_assert(B_CH >= 1, "BN too small");
    __shared__ __attribute__((aligned(16))) char smem[2 * A_BYTES + 2 * B_BYTES];
    char* a_hi = smem;
    char* a_lo = smem + A_BYTES;
    char* b_hi = smem + 2 * A_BYTES;
    char* b_lo = b_hi + B_BYTES;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int tiles_m = (p.m + BM - 1) / BM;
    const int tm = blockIdx.x % tiles_m, tn = blockIdx.x / tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const bool silu_in = p.flags & RF_CONV_SILU_IN;

    // per-thread A rows (fixed across K steps): row = i*16 + tid/16, 4-channel group = tid%16
    int a_img[A_F4], a_iy[A_F4], a_ix[A_F4];
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
        int m = m0 + i * 16 + (tid >> 4);
        const bool ok = m < p.m;
        m = ok ? m : p.m - 1;
        const int ox = m % p.wo, t = m / p.wo;
        const int oy = t % p.ho;
        a_img[i] = ok ? t / p.ho : -1;
        a_iy[i] = oy * p.stride - p.pad;
        a_ix[i] = ox * p.stride - p.pad;
    }
    const int c4 = (tid & 15) * 4;

    float4 areg[A_F4];
    u32x4 bhreg[B_CH], blreg[B_CH];
    auto load = [&](int kt) {
        const int k0 = kt * BK;
        const int tap = k0 / p.cin_pad, cbase = k0 % p.cin_pad;
        const int ky = tap / p.kw, kx = tap % p.kw;
        const int c = cbase + c4;
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            const int iy = a_iy[i] + ky, ix = a_ix[i] + kx;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (a_img[i] >= 0 && iy >= 0 && iy < p.hi && ix >= 0 && ix < p.wi && c < p.cin)
                v = *reinterpret_cast<const float4*>(p.in + (((int64_t)a_img[i] * p.hi + iy) * p.wi + ix) * p.cin + c);
            areg[i] = v;
        }
#pragma unroll
        for (int i = 0; i < B_CH; ++i) {
            const int ch = i * THREADS + tid;
            const int row = ch >> 3, kc = ch & 7;
            const int64_t off = (int64_t)(n0 + row) * p.k + k0 + kc * 8;
            bhreg[i] = *reinterpret_cast<const u32x4*>(p.w_hi + off);
            blreg[i] = *reinterpret_cast<const u32x4*>(p.w_lo + off);
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            float4 v = areg[i];
            if (silu_in) {
                v.x = silu(v.x);
                v.y = silu(v.y);
                v.z = silu(v.z);
                v.w = silu(v.w);
            }
            split_store(a_hi, a_lo, i * 16 + (tid >> 4), tid & 15, v);
        }
#pragma unroll
        for (int i = 0; i < B_CH; ++i) {
            const int ch = i * THREADS + tid;
            const int off = swz(ch >> 3, ch & 7);
            *reinterpret_cast<u32x4*>(b_hi + off) = bhreg[i];
            *reinterpret_cast<u32x4*>(b_lo + off) = blreg[i];
        }
    };

    f32x4 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = p.k / BK;
    load(0);
    store();
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) load(kt + 1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int kc = ks * 4 + (lane >> 4);
            bf16x8 ah[TI], al[TI], bh[TJ], bl[TJ];
#pragma unroll
            for (int i = 0; i < TI; ++i) {
                const int r = wm * MW + i * 16 + (lane & 15);
                ah[i] = *reinterpret_cast<const bf16x8*>(a_hi + swz(r, kc));
                al[i] = *reinterpret_cast<const bf16x8*>(a_lo + swz(r, kc));
            }
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int r = wn * NW + j * 16 + (lane & 15);
                bh[j] = *reinterpret_cast<const bf16x8*>(b_hi + swz(r, kc));
                bl[j] = *reinterpret_cast<const bf16x8*>(b_lo + swz(r, kc));
            }
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                }
        }
        __syncthreads();
        if (kt + 1 < nk) {
            store();
            __syncthreads();
        }
    }

    // ------------------------------------------------------------------ epilogue
    const int col_l = lane & 15, row_q = (lane >> 4) * 4;
    if (p.flags & RF_CONV_FINAL) {
        // SiLU -> 1x1 (BN=cout channels -> n_fin) -> ELU -> optional 10^x - 1; one pixel row spans the
        // 16 lanes sharing lane>>4 times TJ column tiles.
        for (int f = 0; f < p.n_fin; ++f) {
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    float s = 0.f;
#pragma unroll
                    for (int j = 0; j < TJ; ++j) {
                        const int col = n0 + wn * NW + j * 16 + col_l;
                        if (col < p.cout) {
                            float v = acc[i][j][rr] + (p.bias ? p.bias[col] : 0.f);
                            v = silu(v);
                            s += v * p.w_fin[f * p.cout + col];
                        }
                    }
                    s += __shfl_xor(s, 1, 64);
                    s += __shfl_xor(s, 2, 64);
                    s += __shfl_xor(s, 4, 64);
                    s += __shfl_xor(s, 8, 64);
                    const int m = m0 + wm * MW + i * 16 + row_q + rr;
                    if (col_l == 0 && m < p.m) {
                        float y = s + p.b_fin[f];
                        y = y > 0.f ? y : p.elu_alpha * expm1f(y);
                        if (p.flags & RF_CONV_LOG_DECODE) y = powf(10.0f, y) - 1.0f;
                        const int hw = p.ho * p.wo;
                        const int64_t o = (p.flags & RF_CONV_NCHW_OUT)
                                              ? ((int64_t)(m / hw) * p.n_fin + f) * hw + (m % hw)
                                              : (int64_t)m * p.n_fin + f;
                        p.out[o] = y;
                    }
                }
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
        const int col = n0 + wn * NW + j * 16 + col_l;
        const int nreal = p.deconv ? p.cout * p.deconv * p.deconv : p.cout;
        if (col >= nreal) continue;
        const int co = p.deconv ? col % p.cout : col;
        const float b = p.bias ? p.bias[co] : 0.f;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int m = m0 + wm * MW + i * 16 + row_q + rr;
                if (m >= p.m) continue;
                int64_t o;
                if (p.deconv) {
                    const int kk = p.deconv;
                    const int tap = col / p.cout, dy = tap / kk, dx = tap % kk;
                    const int x = m % p.wo, t = m / p.wo, y = t % p.ho, img = t / p.ho;
                    o = (((int64_t)img * p.ho * kk + y * kk + dy) * (p.wo * kk) + x * kk + dx) * p.cout + co;
                } else {
                    o = (int64_t)m * p.cout + co;
                }
                float v = acc[i][j][rr] + b;
                if (p.res1) v += p.res1[o];
                if (p.res2) v += p.res2[o];
                if (p.flags & RF_CONV_SILU_OUT) v = silu(v);
                p.out[o] = v;
            }
    }
}

// bilinear, align_corners=True, NHWC fp32 (torch upsample_bilinear2d semantics)
__global__ __launch_bounds__(256) void upsample_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                       int n_img, int hi, int wi, int c, int ho, int wo) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int c4n = c / 4;
    const int64_t total = (int64_t)n_img * ho * wo * c4n;
    if (idx >= total) return;
    const int cc = (int)(idx % c4n) * 4;
    int64_t t = idx / c4n;
    const int ox = (int)(t % wo);
    t /= wo;
    const int oy = (int)(t % ho);
    const int img = (int)(t / ho);
    const float sh = ho > 1 ? (float)(hi - 1) / (float)(ho - 1) : 0.f;
    const float sw = wo > 1 ? (float)(wi - 1) / (float)(wo - 1) : 0.f;
    const float fy = sh * (float)oy, fx = sw * (float)ox;
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = y0 + (y0 < hi - 1 ? 1 : 0), x1 = x0 + (x0 < wi - 1 ? 1 : 0);
    const float ly1 = fy - (float)y0, lx1 = fx - (float)x0;
    const float ly0 = 1.0f - ly1, lx0 = 1.0f - lx1;
    const float* base = in + (int64_t)img * hi * wi * c + cc;
    const float4 a = *reinterpret_cast<const float4*>(base + ((int64_t)y0 * wi + x0) * c);
    const float4 b = *reinterpret_cast<const float4*>(base + ((int64_t)y0 * wi + x1) * c);
    const float4 d = *reinterpret_cast<const float4*>(base + ((int64_t)y1 * wi + x0) * c);
    const float4 e = *reinterpret_cast<const float4*>(base + ((int64_t)y1 * wi + x1) * c);
    float4 r;
    r.x = ly0 * (lx0 * a.x + lx1 * b.x) + ly1 * (lx0 * d.x + lx1 * e.x);
    r.y = ly0 * (lx0 * a.y + lx1 * b.y) + ly1 * (lx0 * d.y + lx1 * e.y);
    r.z = ly0 * (lx0 * a.z + lx1 * b.z) + ly1 * (lx0 * d.z + lx1 * e.z);
    r.w = ly0 * (lx0 * a.w + lx1 * b.w) + ly1 * (lx0 * d.w + lx1 * e.w);
    *reinterpret_cast<float4*>(out + idx * 4) = r;
}

int launch_conv(const ConvArgs& a, int n_cols, void* stream, const char* what) {
    const int tiles_m = (a.m + BM - 1) / BM;
    hipStream_t s = (hipStream_t)stream;
    if (n_cols <= 32) {
        hipLaunchKernelGGL(conv_bf16x3_kernel<32>, dim3(tiles_m * ((n_cols + 31) / 32)), dim3(THREADS), 0, s, a);
    } else {
        hipLaunchKernelGGL(conv_bf16x3_kernel<128>, dim3(tiles_m * ((n_cols + 127) / 128)), dim3(THREADS), 0, s, a);
    }
    return rf::check_launch(what);
}

}  // namespace

extern "C" int rf_conv2d_bf16x3(const float* in, int n_img, int hi, int wi, int cin, const void* w_hi,
                                const void* w_lo, int cin_pad, int cout, int cout_pad, int kh, int kw, int stride,
                                int pad, const float* bias, const float* res1, const float* res2, float* out,
                                int flags, const float* w_fin, const float* b_fin, int n_fin, float elu_alpha,
                                void* stream) {
    RF_REQUIRE(in && w_hi && w_lo && out, "rf_conv2d_bf16x3: null pointer");
    RF_REQUIRE(cin % 4 == 0 && cin_pad % BK == 0 && cin_pad >= cin, "rf_conv2d_bf16x3: cin %d / cin_pad %d", cin,
               cin_pad);
    RF_REQUIRE(((uintptr_t)in & 15) == 0, "rf_conv2d_bf16x3: input must be 16-B aligned");
    const int bn = cout <= 32 ? 32 : 128;
    RF_REQUIRE(cout_pad % bn == 0 && cout_pad >= cout, "rf_conv2d_bf16x3: cout_pad %d must be a multiple of %d",
               cout_pad, bn);
    RF_REQUIRE(!(flags & RF_CONV_FINAL) || (cout <= 32 && w_fin && b_fin && n_fin > 0),
               "rf_conv2d_bf16x3: final head needs cout <= 32 and w_fin/b_fin");
    ConvArgs a{};
    a.in = in;
    a.w_hi = (const bf16_t*)w_hi;
    a.w_lo = (const bf16_t*)w_lo;
    a.bias = bias;
    a.res1 = res1;
    a.res2 = res2;
    a.out = out;
    a.w_fin = w_fin;
    a.b_fin = b_fin;
    a.n_img = n_img;
    a.hi = hi;
    a.wi = wi;
    a.cin = cin;
    a.cin_pad = cin_pad;
    a.ho = (hi + 2 * pad - kh) / stride + 1;
    a.wo = (wi + 2 * pad - kw) / stride + 1;
    a.kw = kw;
    a.stride = stride;
    a.pad = pad;
    a.cout = cout;
    a.m = n_img * a.ho * a.wo;
    a.k = kh * kw * cin_pad;
    a.deconv = 0;
    a.flags = flags;
    a.n_fin = n_fin;
    a.elu_alpha = elu_alpha;
    if (a.m <= 0) return RF_OK;
    return launch_conv(a, cout_pad, stream, "rf_conv2d_bf16x3");
}

extern "C" int rf_deconv2d_bf16x3(const float* in, int n_img, int hi, int wi, int cin, const void* w_hi,
                                  const void* w_lo, int cin_pad, int cout, int k, const float* bias, float* out,
                                  void* stream) {
    RF_REQUIRE(in && w_hi && w_lo && out, "rf_deconv2d_bf16x3: null pointer");
    RF_REQUIRE(cin % 4 == 0 && cin_pad % BK == 0 && cin_pad >= cin, "rf_deconv2d_bf16x3: bad cin/cin_pad");
    RF_REQUIRE((k * k * cout) % 128 == 0, "rf_deconv2d_bf16x3: k*k*cout must be a multiple of 128");
    ConvArgs a{};
    a.in = in;
    a.w_hi = (const bf16_t*)w_hi;
    a.w_lo = (const bf16_t*)w_lo;
    a.bias = bias;
    a.out = out;
    a.n_img = n_img;
    a.hi = hi;
    a.wi = wi;
    a.cin = cin;
    a.cin_pad = cin_pad;
    a.ho = hi;
    a.wo = wi;
    a.kw = 1;
    a.stride = 1;
    a.pad = 0;
    a.cout = cout;
    a.m = n_img * hi * wi;
    a.k = cin_pad;
    a.deconv = k;
    if (a.m <= 0) return RF_OK;
    return launch_conv(a, k * k * cout, stream, "rf_deconv2d_bf16x3");
}

extern "C" int rf_upsample_bilinear(const float* in, int n_img, int hi, int wi, int c, float* out, int ho, int wo,
                                    void* stream) {
    RF_REQUIRE(in && out, "rf_upsample_bilinear: null pointer");
    RF_REQUIRE(c % 4 == 0, "rf_upsample_bilinear: channels must be a multiple of 4");
    const int64_t total = (int64_t)n_img * ho * wo * (c / 4);
    if (total <= 0) return RF_OK;
    hipLaunchKernelGGL(upsample_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, in,
                       out, n_img, hi, wi, c, ho, wo);
    return rf::check_launch("rf_upsample_bilinear");
}
