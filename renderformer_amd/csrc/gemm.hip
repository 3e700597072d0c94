// MFMA GEMM engine for gfx950: every projection of both transformer stages and
// every DPT convolution runs through this one kernel template.
//
//   C[M,N] (epilogue) A[M,K] * W[N,K]^T
//
// * Operands are K-contiguous bf16 (nn.Linear weight layout [out, in]); the A
//   rows are either dense (a + m*lda) or gathered (DPT convolutions: im2col of an
//   NHWC activation plane, one 32-wide K step = one filter tap, out-of-image rows
//   point at a zero row) — no im2col buffer is ever materialised.
// * NTERM = 3 evaluates fp32-accurate products from bf16 hi/lo splits of both
//   operands: a.b ~= ah.bh + ah.bl + al.bh  (DPT head, see dpt.py).
// * Tile 128x128x32, 256 threads = 2x2 waves of 64x64 (4x4 v_mfma_f32_16x16x32_bf16).
//   Both operands go global->LDS with global_load_lds_dwordx4 (no VGPR staging)
//   through a 3-deep LDS ring: at step kt the wave waits (counted vmcnt) only for
//   tile kt, one raw s_barrier both publishes tile kt and retires the reads of the
//   buffer tile kt+2 overwrites, and tile kt+2's loads then fly under the MFMAs of
//   tile kt.  LDS image: 64-B rows, 16-B chunk index XOR ((row >> 1) & 3) on the
//   source address (LDS-DMA writes lane-linearly) and on the ds_read_b128 address,
//   conflict-free for the fragment reads (tools/banks.py).
// * The MFMA is issued with the W fragment as the first operand, so each lane's
//   accumulator holds 4 consecutive output COLUMNS of one row: epilogue stores,
//   residual loads and SwiGLU pairs are 8-16 B vectors per lane.
// * blockIdx is remapped so each XCD walks a contiguous band of tiles (T1).
#include <math.h>

#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, THREADS = 256, STAGES = 3;
constexpr int TILE = BM * BK * 2;  // 8 KiB per operand plane per stage

enum Epi { E_BF16 = RF_EPI_BF16, E_F32 = RF_EPI_F32, E_ADD = RF_EPI_ADD_F32, E_SWIGLU = RF_EPI_SWIGLU, E_CONV = 16 };

struct EngineArgs {
    const bf16_t* a;
    const bf16_t* a_lo;
    int64_t lda;
    const bf16_t* w;
    const bf16_t* w_lo;
    int64_t ldw;
    int m, n, k;
    // gathered A (convolution): NHWC plane [img][hi][wi][cin_pad]
    int gather, hi, wi, cin_pad, ho, wo, kw, stride, pad;
    const bf16_t* zero;
    // epilogue
    void* c;
    int64_t ldc;
    const float* bias;
    const float* res1;
    const float* res2;
    bf16_t* p_hi;
    bf16_t* p_lo;
    int p_ld;
    int cout, deconv, flags, n_fin;
    const float* w_fin;
    const float* b_fin;
    float elu_alpha;
};

RF_DEV int lds_off(int row, int ch) { return row * 64 + ((ch ^ ((row >> 1) & 3)) << 4); }

RF_DEV float silu(float x) { return x / (1.0f + expf(-x)); }

template <int EPI, int NTERM, bool GATHER>
__global__ __launch_bounds__(THREADS, 2) void engine_kernel(EngineArgs p) {
    constexpr int PLANES = NTERM == 3 ? 4 : 2;  // A, W (+ A_lo, W_lo)
    constexpr int STAGE_BYTES = PLANES * TILE;
    __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE_BYTES];

    const int tiles_n = p.n / BN;
    const int tiles_m = (p.m + BM - 1) / BM;
    const int nwg = tiles_n * tiles_m;
    const int hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    const int tm = wg % tiles_m, tn = wg / tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;

    // ---- per-lane staging geometry: piece pc (0..1) of this wave covers rows (wave*2+pc)*16 .. +16
    int row_of[2], lc_of[2];
#pragma unroll
    for (int pc = 0; pc < 2; ++pc) {
        const int row = (wave * 2 + pc) * 16 + (lane >> 2);
        row_of[pc] = row;
        lc_of[pc] = (lane & 3) ^ ((row >> 1) & 3);
    }
    int g_img[2] = {0, 0}, g_iy[2] = {0, 0}, g_ix[2] = {0, 0};
    const bf16_t* a_row_ptr[2];
    const bf16_t* a_row_ptr_lo[2];
#pragma unroll
    for (int pc = 0; pc < 2; ++pc) {
        int m = m0 + row_of[pc];
        const bool ok = m < p.m;
        m = ok ? m : p.m - 1;
        if constexpr (GATHER) {
            const int ox = m % p.wo, t = m / p.wo;
            g_img[pc] = ok ? t / p.ho : -1;
            g_iy[pc] = (t % p.ho) * p.stride - p.pad;
            g_ix[pc] = ox * p.stride - p.pad;
        }
        a_row_ptr[pc] = p.a + (int64_t)m * p.lda;
        a_row_ptr_lo[pc] = NTERM == 3 ? p.a_lo + (int64_t)m * p.lda : nullptr;
    }

    auto issue = [&](int kt, int buf) {
        char* st = smem + buf * STAGE_BYTES;
        const int k0 = kt * BK;
        int tap = 0, cb = k0, ky = 0, kx = 0;
        if constexpr (GATHER) {
            tap = k0 / p.cin_pad;
            cb = k0 - tap * p.cin_pad;
            ky = tap / p.kw;
            kx = tap - ky * p.kw;
        }
#pragma unroll
        for (int pc = 0; pc < 2; ++pc) {
            const int piece = wave * 2 + pc;
            const int kofs = lc_of[pc] * 8;
            const bf16_t* sa;
            const bf16_t* sa_lo = nullptr;
            if constexpr (GATHER) {
                const int iy = g_iy[pc] + ky, ix = g_ix[pc] + kx;
                const bool ok = g_img[pc] >= 0 && iy >= 0 && iy < p.hi && ix >= 0 && ix < p.wi;
                const int64_t off = (((int64_t)g_img[pc] * p.hi + iy) * p.wi + ix) * p.cin_pad + cb + kofs;
                sa = ok ? p.a + off : p.zero;
                if constexpr (NTERM == 3) sa_lo = ok ? p.a_lo + off : p.zero;
            } else {
                sa = a_row_ptr[pc] + k0 + kofs;
                if constexpr (NTERM == 3) sa_lo = a_row_ptr_lo[pc] + k0 + kofs;
            }
            const bf16_t* sw = p.w + (int64_t)(n0 + row_of[pc]) * p.ldw + k0 + kofs;
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, sa), LDS_PTR(void, st + piece * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, sw), LDS_PTR(void, st + TILE + piece * 1024), 16, 0, 0);
            if constexpr (NTERM == 3) {
                const bf16_t* sw_lo = p.w_lo + (int64_t)(n0 + row_of[pc]) * p.ldw + k0 + kofs;
                __builtin_amdgcn_global_load_lds(GLB_PTR(void, sa_lo), LDS_PTR(void, st + 2 * TILE + piece * 1024),
                                                 16, 0, 0);
                __builtin_amdgcn_global_load_lds(GLB_PTR(void, sw_lo), LDS_PTR(void, st + 3 * TILE + piece * 1024),
                                                 16, 0, 0);
            }
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = p.k / BK;
    issue(0, 0);
    if (nk > 1) issue(1, 1);
    const int frag_row = lane & 15, frag_ch = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        // tile kt landed for this wave: leave only tile kt+1's loads in flight
        if (kt + 1 < nk) {
            if constexpr (NTERM == 3)
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt + 2 < nk) issue(kt + 2, (kt + 2) % STAGES);
        const char* st = smem + (kt % STAGES) * STAGE_BYTES;
        bf16x8 fa[4], fw[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(st + lds_off(wm * 64 + i * 16 + frag_row, frag_ch));
#pragma unroll
        for (int j = 0; j < 4; ++j)
            fw[j] = *reinterpret_cast<const bf16x8*>(st + TILE + lds_off(wn * 64 + j * 16 + frag_row, frag_ch));
        if constexpr (NTERM == 3) {
            bf16x8 fal[4], fwl[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                fal[i] = *reinterpret_cast<const bf16x8*>(st + 2 * TILE + lds_off(wm * 64 + i * 16 + frag_row, frag_ch));
#pragma unroll
            for (int j = 0; j < 4; ++j)
                fwl[j] = *reinterpret_cast<const bf16x8*>(st + 3 * TILE + lds_off(wn * 64 + j * 16 + frag_row, frag_ch));
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fwl[j], fa[i], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[j], fal[i], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[j], fa[i], acc[i][j], 0, 0, 0);
                }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[j], fa[i], acc[i][j], 0, 0, 0);
        }
    }

    // ------------------------------------------------------------------ epilogue
    // acc[i][j][e] = C[row][col + e], row = m0 + wm*64 + i*16 + (lane & 15),
    //                                  col = n0 + wn*64 + j*16 + 4*(lane >> 4)
    const int rl = lane & 15, cq = 4 * (lane >> 4);
    if constexpr (EPI == E_SWIGLU) {
        bf16_t* c = reinterpret_cast<bf16_t*>(p.c);
#pragma unroll
        for (int pair = 0; pair < 2; ++pair) {
            const int gcol = n0 + wn * 64 + pair * 32;  // 32-row interleave group: [w1 x16 | w3 x16]
            const int ocol = (gcol >> 5) * 16 + cq;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = m0 + wm * 64 + i * 16 + rl;
                if (row < p.m) {
                    float o[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float g = acc[i][2 * pair][e], u = acc[i][2 * pair + 1][e];
                        if (p.bias) {
                            g += p.bias[gcol + cq + e];
                            u += p.bias[gcol + 16 + cq + e];
                        }
                        o[e] = silu(g) * u;
                    }
                    *reinterpret_cast<uint2*>(c + (int64_t)row * p.ldc + ocol) =
                        make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
                }
            }
        }
        return;
    } else if constexpr (EPI == E_CONV) {
        if (p.flags & RF_CONV_FINAL) {
            // SiLU -> 1x1 (cout <= 32 channels -> n_fin) -> ELU -> [10^x - 1]; pixel row = lane & 15,
            // its channels spread over j tiles, e and the four lane>>4 groups.
            for (int f = 0; f < p.n_fin; ++f) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float s = 0.f;
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int col = n0 + wn * 64 + j * 16 + cq + e;
                            if (col < p.cout) {
                                const float v = silu(acc[i][j][e] + (p.bias ? p.bias[col] : 0.f));
                                s += v * p.w_fin[f * p.cout + col];
                            }
                        }
                    s += __shfl_xor(s, 16, 64);
                    s += __shfl_xor(s, 32, 64);
                    const int m = m0 + wm * 64 + i * 16 + rl;
                    if (lane < 16 && wn == 0 && m < p.m) {
                        float y = s + p.b_fin[f];
                        y = y > 0.f ? y : p.elu_alpha * expm1f(y);
                        if (p.flags & RF_CONV_LOG_DECODE) y = powf(10.0f, y) - 1.0f;
                        const int hwp = p.ho * p.wo;
                        const int64_t o = (p.flags & RF_CONV_NCHW_OUT) ? ((int64_t)(m / hwp) * p.n_fin + f) * hwp + (m % hwp)
                                                                      : (int64_t)m * p.n_fin + f;
                        reinterpret_cast<float*>(p.c)[o] = y;
                    }
                }
            }
            return;
        }
        const int kk = p.deconv;
        const int nreal = kk ? p.cout * kk * kk : p.cout;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = m0 + wm * 64 + i * 16 + rl;
            if (m >= p.m) continue;
            // output pixel base for the (deconv) scatter
            int img = 0, y = 0, x = 0;
            if (kk) {
                x = m % p.wo;
                const int t = m / p.wo;
                y = t % p.ho;
                img = t / p.ho;
            }
            float4 r1[4], r2[4];
            int64_t obase[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = n0 + wn * 64 + j * 16 + cq;
                int64_t pix = m;
                int co = col;
                if (kk) {
                    const int tap = col / p.cout, dy = tap / kk, dx = tap % kk;
                    co = col - tap * p.cout;
                    pix = ((int64_t)img * p.ho * kk + y * kk + dy) * (p.wo * kk) + x * kk + dx;
                }
                obase[j] = pix * 65536 + co;  // packed (pixel, channel)
                if (col < nreal) {
                    r1[j] = p.res1 ? *reinterpret_cast<const float4*>(p.res1 + pix * p.cout + co) : float4{0, 0, 0, 0};
                    r2[j] = p.res2 ? *reinterpret_cast<const float4*>(p.res2 + pix * p.cout + co) : float4{0, 0, 0, 0};
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = n0 + wn * 64 + j * 16 + cq;
                if (col >= nreal) continue;
                const int64_t pix = obase[j] >> 16;
                const int co = (int)(obase[j] & 65535);
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                const float rr1[4] = {r1[j].x, r1[j].y, r1[j].z, r1[j].w};
                const float rr2[4] = {r2[j].x, r2[j].y, r2[j].z, r2[j].w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (p.bias) v[e] += p.bias[co + e];
                    v[e] = (v[e] + rr1[e]) + rr2[e];
                    if (p.flags & RF_CONV_SILU_OUT) v[e] = silu(v[e]);
                }
                if (p.c)
                    *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.c) + pix * p.cout + co) =
                        make_float4(v[0], v[1], v[2], v[3]);
                if (p.p_hi) {
                    uint32_t h[2], l[2];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        float a0 = v[2 * e], a1 = v[2 * e + 1];
                        if (p.flags & RF_CONV_PLANE_SILU) {
                            a0 = silu(a0);
                            a1 = silu(a1);
                        }
                        const bf16_t h0 = f32_to_bf16(a0), h1 = f32_to_bf16(a1);
                        h[e] = (uint32_t)h0 | ((uint32_t)h1 << 16);
                        l[e] = pack_bf16x2(a0 - bf16_to_f32(h0), a1 - bf16_to_f32(h1));
                    }
                    *reinterpret_cast<uint2*>(p.p_hi + pix * p.p_ld + co) = make_uint2(h[0], h[1]);
                    *reinterpret_cast<uint2*>(p.p_lo + pix * p.p_ld + co) = make_uint2(l[0], l[1]);
                }
            }
        }
        return;
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = m0 + wm * 64 + i * 16 + rl;
            if (row >= p.m) continue;
            float4 old[4];
            if constexpr (EPI == E_ADD) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    old[j] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.c) + (int64_t)row * p.ldc +
                                                              n0 + wn * 64 + j * 16 + cq);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = n0 + wn * 64 + j * 16 + cq;
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                if (p.bias) {
                    const float4 b = *reinterpret_cast<const float4*>(p.bias + col);
                    v[0] += b.x;
                    v[1] += b.y;
                    v[2] += b.z;
                    v[3] += b.w;
                }
                const int64_t o = (int64_t)row * p.ldc + col;
                if constexpr (EPI == E_BF16) {
                    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.c) + o) =
                        make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
                } else if constexpr (EPI == E_F32) {
                    *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.c) + o) = make_float4(v[0], v[1], v[2], v[3]);
                } else {
                    *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.c) + o) =
                        make_float4(old[j].x + v[0], old[j].y + v[1], old[j].z + v[2], old[j].w + v[3]);
                }
            }
        }
    }
}

template <int EPI, int NTERM, bool GATHER = false>
int launch(const EngineArgs& a, void* stream, const char* what) {
    const int nwg = (a.n / BN) * ((a.m + BM - 1) / BM);
    hipLaunchKernelGGL((engine_kernel<EPI, NTERM, GATHER>), dim3(nwg), dim3(THREADS), 0, (hipStream_t)stream, a);
    return rf::check_launch(what);
}

__device__ __attribute__((aligned(16))) bf16_t g_zero_row[64];  // stays zero: source of padded conv taps

}  // namespace

extern "C" int rf_gemm_bf16(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc,
                            const float* bias, int m, int n, int k, int epilogue, void* stream) {
    RF_REQUIRE(a && w && c, "rf_gemm_bf16: null pointer");
    RF_REQUIRE(m > 0 && n > 0 && k > 0, "rf_gemm_bf16: empty problem m=%d n=%d k=%d", m, n, k);
    RF_REQUIRE(k % BK == 0, "rf_gemm_bf16: K=%d must be a multiple of %d", k, BK);
    RF_REQUIRE(n % BN == 0, "rf_gemm_bf16: N=%d must be a multiple of %d", n, BN);
    RF_REQUIRE(lda % 8 == 0 && ldw % 8 == 0 && lda >= k && ldw >= k, "rf_gemm_bf16: lda/ldw must be >=K and 16-B aligned");
    RF_REQUIRE(((uintptr_t)a & 15) == 0 && ((uintptr_t)w & 15) == 0, "rf_gemm_bf16: operands must be 16-B aligned");
    RF_REQUIRE(epilogue >= RF_EPI_BF16 && epilogue <= RF_EPI_SWIGLU, "rf_gemm_bf16: bad epilogue %d", epilogue);
    RF_REQUIRE(ldc >= (epilogue == RF_EPI_SWIGLU ? n / 2 : n) && ldc % 4 == 0, "rf_gemm_bf16: ldc too small/unaligned");
    RF_REQUIRE(((uintptr_t)c & 7) == 0, "rf_gemm_bf16: output must be 8-B aligned");
    EngineArgs p{};
    p.a = (const bf16_t*)a;
    p.lda = lda;
    p.w = (const bf16_t*)w;
    p.ldw = ldw;
    p.m = m;
    p.n = n;
    p.k = k;
    p.c = c;
    p.ldc = ldc;
    p.bias = bias;
    switch (epilogue) {
        case RF_EPI_BF16: return launch<E_BF16, 1>(p, stream, "rf_gemm_bf16");
        case RF_EPI_F32: return launch<E_F32, 1>(p, stream, "rf_gemm_bf16");
        case RF_EPI_ADD_F32: return launch<E_ADD, 1>(p, stream, "rf_gemm_bf16");
        default: return launch<E_SWIGLU, 1>(p, stream, "rf_gemm_bf16");
    }
}

static int conv_common(EngineArgs& p, const void* w_hi, const void* w_lo, int cout, int cout_pad, float* out,
                       const float* bias, const float* res1, const float* res2, void* p_hi, void* p_lo, int p_ld,
                       int flags, const float* w_fin, const float* b_fin, int n_fin, float elu_alpha, void* stream,
                       const char* what) {
    RF_REQUIRE(w_hi && w_lo, "%s: null weights", what);
    RF_REQUIRE(cout % 4 == 0, "%s: cout must be a multiple of 4", what);
    RF_REQUIRE(out || p_hi, "%s: no output", what);
    RF_REQUIRE(!p_hi || (p_lo && p_ld % 4 == 0 && p_ld >= cout), "%s: bad plane output", what);
    RF_REQUIRE(!(flags & RF_CONV_FINAL) || (cout <= 64 && w_fin && b_fin && n_fin > 0 && out),
               "%s: final head needs cout <= 64 and w_fin/b_fin", what);
    static void* z = nullptr;  // device address of the zero row (per process; single device per process)
    if (!z && hipGetSymbolAddress(&z, HIP_SYMBOL(g_zero_row)) != hipSuccess) {
        z = nullptr;
        rf::set_error("%s: zero row symbol", what);
        return RF_ERR_LAUNCH;
    }
    p.zero = (const bf16_t*)z;
    p.w = (const bf16_t*)w_hi;
    p.w_lo = (const bf16_t*)w_lo;
    p.n = cout_pad;
    p.c = out;
    p.bias = bias;
    p.res1 = res1;
    p.res2 = res2;
    p.p_hi = (bf16_t*)p_hi;
    p.p_lo = (bf16_t*)p_lo;
    p.p_ld = p_ld;
    p.cout = cout;
    p.flags = flags;
    p.w_fin = w_fin;
    p.b_fin = b_fin;
    p.n_fin = n_fin;
    p.elu_alpha = elu_alpha;
    if (p.m <= 0) return RF_OK;
    return p.gather ? launch<E_CONV, 3, true>(p, stream, what) : launch<E_CONV, 3, false>(p, stream, what);
}

extern "C" int rf_conv2d_bf16x3(const void* in_hi, const void* in_lo, int n_img, int hi, int wi, int cin_pad,
                                const void* w_hi, const void* w_lo, int cout, int cout_pad, int kh, int kw, int stride,
                                int pad, const float* bias, const float* res1, const float* res2, float* out,
                                void* p_hi, void* p_lo, int p_ld, int flags, const float* w_fin, const float* b_fin,
                                int n_fin, float elu_alpha, void* stream) {
    RF_REQUIRE(in_hi && in_lo, "rf_conv2d_bf16x3: null input");
    RF_REQUIRE(cin_pad % BK == 0, "rf_conv2d_bf16x3: cin_pad %d must be a multiple of %d", cin_pad, BK);
    RF_REQUIRE(cout_pad % BN == 0 && cout_pad >= cout, "rf_conv2d_bf16x3: cout_pad %d must be a multiple of %d",
               cout_pad, BN);
    EngineArgs p{};
    p.a = (const bf16_t*)in_hi;
    p.a_lo = (const bf16_t*)in_lo;
    p.gather = 1;
    p.hi = hi;
    p.wi = wi;
    p.cin_pad = cin_pad;
    p.ho = (hi + 2 * pad - kh) / stride + 1;
    p.wo = (wi + 2 * pad - kw) / stride + 1;
    p.kw = kw;
    p.stride = stride;
    p.pad = pad;
    p.m = n_img * p.ho * p.wo;
    p.k = kh * kw * cin_pad;
    p.ldw = p.k;
    return conv_common(p, w_hi, w_lo, cout, cout_pad, out, bias, res1, res2, p_hi, p_lo, p_ld, flags, w_fin, b_fin,
                       n_fin, elu_alpha, stream, "rf_conv2d_bf16x3");
}

extern "C" int rf_deconv2d_bf16x3(const void* in_hi, const void* in_lo, int n_img, int hi, int wi, int cin_pad,
                                  const void* w_hi, const void* w_lo, int cout, int k, const float* bias, float* out,
                                  void* p_hi, void* p_lo, int p_ld, void* stream) {
    RF_REQUIRE(in_hi && in_lo, "rf_deconv2d_bf16x3: null input");
    RF_REQUIRE(cin_pad % BK == 0, "rf_deconv2d_bf16x3: cin_pad must be a multiple of %d", BK);
    RF_REQUIRE((k * k * cout) % BN == 0 && cout < 65536, "rf_deconv2d_bf16x3: k*k*cout must be a multiple of %d", BN);
    EngineArgs p{};
    p.a = (const bf16_t*)in_hi;
    p.a_lo = (const bf16_t*)in_lo;
    p.lda = cin_pad;
    p.ho = hi;
    p.wo = wi;
    p.m = n_img * hi * wi;
    p.k = cin_pad;
    p.ldw = cin_pad;
    p.deconv = k;
    return conv_common(p, w_hi, w_lo, cout, k * k * cout, out, bias, nullptr, nullptr, p_hi, p_lo, p_ld, 0, nullptr,
                       nullptr, 0, 0.f, stream, "rf_deconv2d_bf16x3");
}
