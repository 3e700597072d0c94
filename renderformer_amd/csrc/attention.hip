// Flash-style attention forward for gfx950, head_dim 128, bf16 operands, fp32
// online softmax.  Two front-ends share one wave-level body:
//
//   * varlen (rf_attn_fwd): per problem p a query row range and a key/value row
//     range — this one kernel covers stage-1 triangle self-attention over
//     unpadded scenes (flash_attn_varlen_qkvpacked_func, attention.py:164-173)
//     and stage-2 ray->triangle cross-attention where K is per view and V is
//     shared by every view of a scene (flash_attn_varlen_kvpacked_func,
//     attention.py:183-198).  Padding never reaches the kernel: the host packs
//     valid tokens, so the key mask is just "j < k_len" on the last tile.
//   * swin (rf_swin_attn_fwd): one 64-token window per block; the cyclic roll
//     and window partition/reverse (attention.py:205-234, 333-368) are pure row
//     index math on load/store and the shift mask (attention.py:237-271) is
//     computed from region labels in registers.
//
// Wave layout (each wave owns 32 query rows, the whole workgroup streams the
// same K/V tiles of 64 keys through LDS):
//   S^T[key][q] = K Q^T with v_mfma_f32_32x32x16_bf16, K from LDS as the A
//   operand, Q held in registers as the B operand.  The accumulator has the
//   query on the lane and 16 keys in registers, so the row max/sum need one
//   cross-half exchange only, and the probabilities feed the next MFMA
//   (O^T = V^T P^T) as its B operand without any lane movement; V^T comes
//   straight from the row-major V tile with ds_read_b64_tr_b16.
// LDS images use the 256-B-row XOR swizzle off(row, ch) = 256 row +
// 16 (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))), conflict-free for both the
// K ds_read_b128 and the V transposed reads (checked with the bank model in
// tools/banks.py).  K/V tiles are register-staged with the issue-early /
// write-late split: the next tile's global loads fly under this tile's MFMAs.
#include "common.h"

namespace {

constexpr int HD = 128;
constexpr int KT = 64;                 // keys per tile
constexpr int TILE_BYTES = KT * HD * 2;  // 16 KiB
constexpr float NEG = -1.0e30f;

struct AttnArgs {
    const bf16_t* q;
    const bf16_t* k;
    const bf16_t* v;
    bf16_t* o;
    int64_t ldq, ldk, ldv, ldo;
    const int32_t* problems;  // varlen: [P][5]
    float c;                  // softmax scale * log2(e)
    // swin
    int gh, gw, shift, window;
};

RF_DEV int swz_off(int row, int ch) { return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4); }

RF_DEV int region(int c, int g, int window, int shift) { return c < g - window ? 0 : (c < g - shift ? 1 : 2); }

template <bool SWIN, int NW>
__global__ __launch_bounds__(NW * 64, 2) void attn_fwd_kernel(AttnArgs p) {
    constexpr int T = NW * 64;
    constexpr int CPT = (KT * HD / 8) / T;  // 16-B chunks per thread per tile (per operand)
    constexpr int NBUF = SWIN ? 1 : 2;
    __shared__ __attribute__((aligned(16))) char smem[NBUF * 2 * TILE_BYTES];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int half = lane >> 5;
    const int h = blockIdx.y;
    const int hoff = h * HD;

    int q_start = 0, q_len = 0, k_start = 0, k_len = 0, v_start = 0, q0 = 0;
    int img_row0 = 0, wy = 0, wx = 0;
    if constexpr (SWIN) {
        const int nwx = p.gw / p.window;
        wy = blockIdx.x / nwx;
        wx = blockIdx.x % nwx;
        img_row0 = blockIdx.z * p.gh * p.gw;
        q_len = k_len = KT;
    } else {
        const int32_t* d = p.problems + blockIdx.z * 5;
        q_start = d[0];
        q_len = d[1];
        k_start = d[2];
        k_len = d[3];
        v_start = d[4];
        q0 = blockIdx.x * (NW * 32);
        if (q0 >= q_len) return;
    }

    // window-local token -> global row (swin) ; query/key index -> row (varlen)
    auto swin_row = [&](int i) {
        const int hs = wy * p.window + i / p.window;
        const int ws = wx * p.window + i % p.window;
        int hy = hs + p.shift, wxx = ws + p.shift;
        hy -= hy >= p.gh ? p.gh : 0;
        wxx -= wxx >= p.gw ? p.gw : 0;
        return img_row0 + hy * p.gw + wxx;
    };
    auto swin_label = [&](int i) {
        const int hs = wy * p.window + i / p.window;
        const int ws = wx * p.window + i % p.window;
        return region(hs, p.gh, p.window, p.shift) * 3 + region(ws, p.gw, p.window, p.shift);
    };

    // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[q][16 s + 8 half + 0..7]
    const int qi = wave * 32 + (lane & 31);  // query index within block
    int qrow;
    if constexpr (SWIN) {
        qrow = swin_row(qi);
    } else {
        const int qq = q0 + qi;
        qrow = q_start + (qq < q_len ? qq : q_len - 1);
    }
    bf16x8 qf[8];
    {
        const bf16_t* src = p.q + (int64_t)qrow * p.ldq + hoff + 8 * half;
#pragma unroll
        for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(src + 16 * s);
    }
    int qlabel = 0;
    if constexpr (SWIN) qlabel = p.shift > 0 ? swin_label(qi) : 0;

    // ---- K/V staging (register-staged; rows clamped, tail masked later)
    u32x4 kreg[CPT], vreg[CPT];
    auto load_tile = [&](int kt) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int c = i * T + tid;
            const int row = c >> 4, ch = c & 15;
            int kr, vr;
            if constexpr (SWIN) {
                kr = vr = swin_row(row);
            } else {
                int j = kt * KT + row;
                j = j < k_len ? j : k_len - 1;
                kr = k_start + j;
                vr = v_start + j;
            }
            kreg[i] = *reinterpret_cast<const u32x4*>(p.k + (int64_t)kr * p.ldk + hoff + ch * 8);
            vreg[i] = *reinterpret_cast<const u32x4*>(p.v + (int64_t)vr * p.ldv + hoff + ch * 8);
        }
    };
    auto write_tile = [&](int buf) {
        char* kb = smem + buf * 2 * TILE_BYTES;
        char* vb = kb + TILE_BYTES;
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int c = i * T + tid;
            const int off = swz_off(c >> 4, c & 15);
            *reinterpret_cast<u32x4*>(kb + off) = kreg[i];
            *reinterpret_cast<u32x4*>(vb + off) = vreg[i];
        }
    };

    f32x16 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_run = NEG, l_run = 0.f;

    const int nt = (k_len + KT - 1) / KT;
    load_tile(0);
    write_tile(0);
    __syncthreads();

    // tr-read lane geometry (ds_read_b64_tr_b16): group g = lane>>4, lane 4qq+pp of the group
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;

    for (int kt = 0; kt < nt; ++kt) {
        const int cur = SWIN ? 0 : (kt & 1);
        if (!SWIN && kt + 1 < nt) load_tile(kt + 1);
        const char* kb = smem + cur * 2 * TILE_BYTES;
        const char* vb = kb + TILE_BYTES;

        // ---- S^T = K Q^T for two 32-key sub-blocks
        f32x16 s[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[b][r] = 0.f;
#pragma unroll
            for (int st = 0; st < 8; ++st) {
                const bf16x8 a = *reinterpret_cast<const bf16x8*>(kb + swz_off(b * 32 + (lane & 31), 2 * st + half));
                s[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[st], s[b], 0, 0, 0);
            }
        }

        // ---- scale, mask, online softmax (query on the lane; keys split across lane halves)
        float mt = NEG;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int key = b * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                float val = s[b][r] * p.c;
                if constexpr (SWIN) {
                    if (p.shift > 0 && swin_label(key) != qlabel) val = NEG;
                } else {
                    if (kt * KT + key >= k_len) val = NEG;
                }
                s[b][r] = val;
                mt = fmaxf(mt, val);
            }
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        const float m_new = fmaxf(m_run, mt);
        const float alpha = exp2f(m_run - m_new);
        m_run = m_new;
        float ls = 0.f;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float pv = exp2f(s[b][r] - m_new);
                s[b][r] = pv;
                ls += pv;
            }
        l_run = l_run * alpha + ls;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;

        // ---- O^T += V^T P^T : P (accumulator layout) is the B operand as-is
        bf16x8 pf[2][2];
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int sp = 0; sp < 2; ++sp)
#pragma unroll
                for (int j = 0; j < 8; ++j) pf[b][sp][j] = (__bf16)s[b][8 * sp + j];

#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            const int col = dt * 32 + 16 * (g & 1) + 4 * pp;
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int sp = 0; sp < 2; ++sp) {
                    const int row = b * 32 + 16 * sp + 4 * (g >> 1) + qq;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        LDS_PTR(s16x4, vb + swz_off(row, col >> 3) + (col & 7) * 2));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        LDS_PTR(s16x4, vb + swz_off(row + 8, col >> 3) + (col & 7) * 2));
                    const auto a16 = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                    const bf16x8 a = __builtin_bit_cast(bf16x8, a16);
                    o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pf[b][sp], o[dt], 0, 0, 0);
                }
        }

        if (!SWIN && kt + 1 < nt) write_tile(cur ^ 1);
        __syncthreads();
    }

    // ---- normalise and store: lane owns query (lane & 31), d = dt*32 + 8 gq + 4 half + 0..3
    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = l_tot > 0.f ? 1.0f / l_tot : 0.f;
    int orow;
    if constexpr (SWIN) {
        orow = swin_row(qi);
    } else {
        const int qq2 = q0 + qi;
        if (qq2 >= q_len) return;
        orow = q_start + qq2;
    }
    bf16_t* dst = p.o + (int64_t)orow * p.ldo + hoff;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            uint2 pk;
            pk.x = pack_bf16x2(o[dt][4 * gq + 0] * inv, o[dt][4 * gq + 1] * inv);
            pk.y = pack_bf16x2(o[dt][4 * gq + 2] * inv, o[dt][4 * gq + 3] * inv);
            *reinterpret_cast<uint2*>(dst + dt * 32 + 8 * gq + 4 * half) = pk;
        }
}

constexpr float LOG2E = 1.4426950408889634f;

}  // namespace

extern "C" int rf_attn_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                           void* o, int64_t ldo, const int32_t* problems, int n_problems, int max_q_len, int n_heads,
                           int head_dim, float scale, void* stream) {
    RF_REQUIRE(q && k && v && o && problems, "rf_attn_fwd: null pointer");
    RF_REQUIRE(head_dim == HD, "rf_attn_fwd: head_dim must be 128 (got %d)", head_dim);
    RF_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0, "rf_attn_fwd: strides must be 16-B aligned");
    RF_REQUIRE(n_problems < 65536 && n_heads < 65536, "rf_attn_fwd: grid too large");
    if (n_problems <= 0 || max_q_len <= 0) return RF_OK;
    AttnArgs a{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, ldq, ldk, ldv, ldo, problems,
               scale * LOG2E, 0, 0, 0, 8};
    constexpr int NW = 4;
    dim3 grid((max_q_len + NW * 32 - 1) / (NW * 32), n_heads, n_problems);
    hipLaunchKernelGGL((attn_fwd_kernel<false, NW>), grid, dim3(NW * 64), 0, (hipStream_t)stream, a);
    return rf::check_launch("rf_attn_fwd");
}

extern "C" int rf_swin_attn_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                                void* o, int64_t ldo, int n_images, int grid_h, int grid_w, int window, int shift,
                                int n_heads, int head_dim, float scale, void* stream) {
    RF_REQUIRE(q && k && v && o, "rf_swin_attn_fwd: null pointer");
    RF_REQUIRE(head_dim == HD, "rf_swin_attn_fwd: head_dim must be 128");
    RF_REQUIRE(window == 8, "rf_swin_attn_fwd: window must be 8 (64-token tiles)");
    RF_REQUIRE(grid_h % window == 0 && grid_w % window == 0, "rf_swin_attn_fwd: grid %dx%d not divisible by window",
               grid_h, grid_w);
    RF_REQUIRE(shift >= 0 && shift < window, "rf_swin_attn_fwd: bad shift");
    RF_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0, "rf_swin_attn_fwd: strides must be 16-B aligned");
    if (n_images <= 0) return RF_OK;
    AttnArgs a{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, ldq, ldk, ldv, ldo, nullptr,
               scale * LOG2E, grid_h, grid_w, shift, window};
    dim3 grid((grid_h / window) * (grid_w / window), n_heads, n_images);
    hipLaunchKernelGGL((attn_fwd_kernel<true, 2>), grid, dim3(128), 0, (hipStream_t)stream, a);
    return rf::check_launch("rf_swin_attn_fwd");
}
