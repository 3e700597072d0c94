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
// Wave layout (each wave owns 32 query rows, the workgroup streams the same
// K/V tiles of 64 keys through LDS):
//   S^T[key][q] = K Q^T with v_mfma_f32_32x32x16_bf16, K from LDS as the A
//   operand, Q held in registers as the B operand.  The accumulator has the
//   query on the lane and 16 keys in registers, so the row max/sum need one
//   cross-half exchange only, and the probabilities feed the next MFMA
//   (O^T = V^T P^T) as its B operand without any lane movement; V^T comes
//   straight from the row-major V tile with ds_read_b64_tr_b16.
// VALU diet (the loop is VALU-bound otherwise): the softmax scale is folded into
// one FMA feeding v_exp_f32 directly, the key mask only runs on the tail tile,
// row maxima use max3, and the O rescale is deferred until a row max grows by
// more than 2^8 (guide T13).  The next tile's global loads are issued after the
// QK^T MFMAs (issuing them earlier makes hipcc's loop-carried vmcnt waits stall
// the QK^T on them) and land under the softmax and PV.
// Long key ranges are split over several workgroups (flash-decoding style) when a
// launch would otherwise leave CUs idle; rf_attn_combine merges the partials.
// LDS images use the 256-B-row XOR swizzle off(row, ch) = 256 row +
// 16 (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))), conflict-free for both the
// K ds_read_b128 and the V transposed reads (tools/banks.py).  K/V tiles are
// register-staged with the issue-early / write-late split, double-buffered.
// Workgroups are mapped so that every XCD processes a contiguous range of
// (problem, head, split, q-block): the q-blocks sharing one K/V stream sit on one
// XCD and read it from that XCD's L2.
#include <math.h>
#include <stdio.h>
#include <algorithm>
#include <atomic>
#include <vector>

#include <type_traits>

#include "common.h"

#define RF_CONST __attribute__((address_space(4)))  // read-only for the launch: scalar loads

namespace {

constexpr int HD = 128;
constexpr int KT = 64;                   // keys per tile
constexpr int TILE_BYTES = KT * HD * 2;  // 16 KiB
constexpr float NEG = -1.0e30f;
constexpr int QB5_ = 256;  // query rows per stream-K unit (= QB5 of attn_sk_kernel / 4 x 64 of attn_p4_kernel)
constexpr float RESCALE_LOG2 = 8.0f;  // legacy kernels: row-max growth (log2 units) that forces a rescale
constexpr float SUM_THR_LOG2 = 12.0f;  // stream-K kernel: half-row tile sum (log2) that forces a rescale

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
    // varlen grid decomposition
    int n_qblk, n_heads, n_split, n_total;
    // split partials: O [split][rows][D] f32, M/L [split][rows][H] f32
    float* part_o;
    float* part_ml;
    int64_t part_rows;
    // stream-K
    int n_problems;
    int* flag;
    float thr;  // deferred-rescale threshold (log2 units; RF_ATTN_THR, default 8)
    int* err;   // device error word (rf::device_error_word): stream-K hand-off timeouts
    int spin;   // stream-K hand-off spin bound (polls)
    // stream-K range boundaries [grid + 1] by LOGICAL block index (common.h SkLayout; rf_attn_schedule:
    // cost-balanced, group-aligned); null = equal tile counts per group
    const int64_t* bounds;
    int epoch;  // hand-off flag value of this launch (> 0, new every launch: no re-arm, stale flags never match)
    int o_f16;  // output O as fp16 (the A operand of an fp16 out-projection) instead of bf16
    int* range; // o_f16: the mapped fp16 range flag (|O| > 65504), else null
    int ascend; // diagnostic (RF_SK_ASCEND=1): ascending blockIdx order inside a group (the round-2 layout), A/B only
    // Swin with the q/k norm folded in (rf_swin_attn_fwd_qkn): q and k arrive as the projection wrote them and are
    // normalised on load over the full width (qk_dim columns per segment) from the projection's per-row partial sums
    // of squares (qk_ss [row][2][PRENORM_SLOTS]: q, k), weighted by qk_w [2 * qk_dim] (null: no norm) and, for q,
    // scaled by qk_scale (softmax scale * log2 e) -- rf_qk_norm_rope's arithmetic, without its HBM round trip
    const float* qk_ss;
    const float* qk_w;
    float qk_eps, qk_scale;
    int qk_dim;
    // stream-K kernel (rf_attn_fwd_qn): q arrives normed-by-weight and rotated (rf_gemm_qk_rope) but not divided by
    // its rms: row r of q is multiplied by qk_scale / sqrt(sum_{s < 8} qk_ss[r * qk_ld + s] / qk_dim + qk_eps) when
    // the piece loads it (qk_ss null: q already final)
    int64_t qk_ld;
};

// two f32 -> the 16-bit output pair: fp16 (OF16) or bf16, RNE
template <bool OF16>
RF_DEV uint32_t pack_o(float lo, float hi) { return OF16 ? pack_f16x2(lo, hi) : pack_bf16x2(lo, hi); }

// Stream-K ranges in the forward-progress layout (common.h SkLayout): the launch's units (head x q-block of
// every problem that has keys) in G contiguous chunks, one per XCD group, each chunk's tiles over the group's
// blocks in descending blockIdx order.  The stream-K kernels read their ranges from a table by LOGICAL block
// index, bounds[L] = first tile of logical block L (bounds[grid] = total): the cost-balanced host table
// (rf_attn_schedule), or the equal split written on the device by attn_equal_bounds_kernel.  The kernels check
// the table against the launch instead of trusting it.
RF_DEV void sk_attn_count(const AttnArgs& p, int64_t& total, int64_t& units) {
    total = 0;
    units = 0;
    for (int i = 0; i < p.n_problems; ++i) {
        const int32_t* d = p.problems + 5 * i;
        const int64_t nt = (d[3] + KT - 1) / KT, nu = nt > 0 ? (int64_t)p.n_heads * ((d[1] + QB5_ - 1) / QB5_) : 0;
        total += nu * nt;
        units += nu;
    }
}
RF_DEV int64_t sk_unit_tile(const AttnArgs& p, int64_t u, int64_t total) {  // first tile of unit u (u = units: total)
    int64_t t = 0;
    for (int i = 0; i < p.n_problems; ++i) {
        const int32_t* d = p.problems + 5 * i;
        const int64_t nt = (d[3] + KT - 1) / KT, nu = nt > 0 ? (int64_t)p.n_heads * ((d[1] + QB5_ - 1) / QB5_) : 0;
        if (u < nu) return t + u * nt;
        u -= nu;
        t += nu * nt;
    }
    return total;
}
// equal tile counts per block inside each group (no host schedule): one workgroup writes the table
__global__ __launch_bounds__(64) void attn_equal_bounds_kernel(AttnArgs p, int nwg, int64_t* out) {
    int64_t total, units;
    sk_attn_count(p, total, units);
    const SkLayout lay(nwg, units);
    for (int g = 0; g < lay.G; ++g) {
        const int64_t t0 = sk_unit_tile(p, units * g / lay.G, total), t1 = sk_unit_tile(p, units * (g + 1) / lay.G, total);
        const int nb = lay.size(g), b0 = lay.base(g);
        for (int li = threadIdx.x; li < nb; li += 64) out[b0 + li] = t0 + (t1 - t0) * li / nb;
    }
    if (threadIdx.x == 0) out[nwg] = total;
}
// this block's logical index and its group's end (partners of an owner lie in (L, gend)); -1 = bad table
RF_DEV int sk_attn_block(const AttnArgs& p, int hw, int nwg, int& gend) {
    int64_t total, units;
    sk_attn_count(p, total, units);
    const SkLayout lay(nwg, units);
    int g = 0;
    int L = lay.logical(hw, &g);
    gend = lay.base(g) + lay.size(g);
    if (p.ascend) L = lay.base(g) + gend - 1 - L;  // A/B diagnostic only (RF_SK_ASCEND=1): round-2 order, no progress guarantee
    const int64_t b = p.bounds[L], e = p.bounds[L + 1];
    const bool bad = b < 0 || e < b || e > total || (L == 0 && b != 0) || (L == nwg - 1 && e != total);
    return bad ? -1 : L;
}

RF_DEV int swz_off(int row, int ch) { return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4); }

RF_DEV int region(int c, int g, int window, int shift) { return c < g - window ? 0 : (c < g - shift ? 1 : 2); }

RF_DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

RF_DEV float max3(float a, float b, float c) { return __builtin_fmaxf(__builtin_fmaxf(a, b), c); }

// 1 / rms of row `row`'s segment `seg` from its RF_PRENORM_SLOTS partial sums, in slot order (as rf_gemm_rownorm)
RF_DEV float qk_inv_rms(const AttnArgs& p, int64_t row, int seg) {
    const float4* q = reinterpret_cast<const float4*>(p.qk_ss + (row * 2 + seg) * RF_PRENORM_SLOTS);
    const float4 a = q[0], b = q[1];
    const float sum = ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
    return 1.0f / sqrtf(sum / (float)p.qk_dim + p.qk_eps);
}

// 8 bf16 values x -> bf16(x * s * w[e]) (rf_qk_norm_rope's order: row scale first, then the weight)
RF_DEV u32x4 qk_scale8(u32x4 x, float s, const float* w) {
    const float4 w0 = *reinterpret_cast<const float4*>(w), w1 = *reinterpret_cast<const float4*>(w + 4);
    const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    u32x4 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float a = __uint_as_float(x[e] << 16) * s * wv[2 * e];
        const float b = __uint_as_float(x[e] & 0xffff0000u) * s * wv[2 * e + 1];
        r[e] = pack_bf16x2(a, b);
    }
    return r;
}

template <bool SWIN, int NW, bool OF16 = false, bool QKN = false>
__global__ __launch_bounds__(NW * 64, NW == 8 ? 1 : 2) void attn_fwd_kernel(AttnArgs p) {
    constexpr int T = NW * 64;
    constexpr int CPT = (KT * HD / 8) / T;  // 16-B chunks per thread per tile (per operand)
    constexpr int NBUF = SWIN ? 1 : 2;
    // QKN (Swin with the q/k norm folded in): after the K/V tile, 1 / rms of the window's 64 key rows and the q / k
    // norm weights of this head (128 floats each), staged once per workgroup
    constexpr int QKN_BYTES = QKN ? (KT + 2 * HD) * 4 : 0;
    __shared__ __attribute__((aligned(16))) char smem[NBUF * 2 * TILE_BYTES + QKN_BYTES];
    float* const qkn_inv = reinterpret_cast<float*>(smem + NBUF * 2 * TILE_BYTES);
    float* const qkn_gq = qkn_inv + KT;
    float* const qkn_gk = qkn_gq + HD;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int half = lane >> 5;

    int h, q_start = 0, q_len = 0, k_start = 0, k_len = 0, v_start = 0, q0 = 0;
    int split = 0, t_begin = 0, t_end = 0;
    int img_row0 = 0, wy = 0, wx = 0;
    if constexpr (SWIN) {
        const int nwx = p.gw >> 3;  // window == 8 (host-checked)
        h = blockIdx.y;
        wy = blockIdx.x / nwx;
        wx = blockIdx.x % nwx;
        img_row0 = blockIdx.z * p.gh * p.gw;
        q_len = k_len = KT;
        t_end = 1;
    } else {
        // XCD-aware bijective remap: hardware ids round-robin over 8 XCDs; hand each XCD a
        // contiguous range of logical ids ordered (problem, head, split, q-block).
        const int nwg = p.n_total, hwid = blockIdx.x;
        const int xcd = hwid & 7, qq = nwg >> 3, rr = nwg & 7;
        int id = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (hwid >> 3);
        const int qb = id % p.n_qblk;
        id /= p.n_qblk;
        split = id % p.n_split;
        id /= p.n_split;
        h = id % p.n_heads;
        const int prob = id / p.n_heads;
        const int32_t* d = p.problems + prob * 5;
        q_start = d[0];
        q_len = d[1];
        k_start = d[2];
        k_len = d[3];
        v_start = d[4];
        q0 = qb * (NW * 32);
        if (q0 >= q_len) return;
        const int nt_all = (k_len + KT - 1) / KT;
        const int per = (nt_all + p.n_split - 1) / p.n_split;
        t_begin = split * per;
        t_end = min(nt_all, t_begin + per);
    }
    const int hoff = h * HD;

    // Swin windows are 8 x 8 tokens (the host requires window == 8: one 64-key tile), so the row / label math is
    // shifts and compile-time constants instead of run-time divisions (the shifted layers' mask computes a label
    // for each of a lane's 32 keys)
    constexpr int SW = 8;
    auto swin_row = [&](int i) {
        const int hs = wy * SW + (i >> 3);  // i >= 0
        const int ws = wx * SW + (i & 7);
        int hy = hs + p.shift, wxx = ws + p.shift;
        hy -= hy >= p.gh ? p.gh : 0;
        wxx -= wxx >= p.gw ? p.gw : 0;
        return img_row0 + hy * p.gw + wxx;
    };
    auto swin_label = [&](int i) {
        const int hs = wy * SW + (i >> 3);  // i >= 0
        const int ws = wx * SW + (i & 7);
        return region(hs, p.gh, SW, p.shift) * 3 + region(ws, p.gw, SW, p.shift);
    };

    // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[q][16 s + 8 half + 0..7]
    const int qi = wave * 32 + (lane & 31);
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

    // ---- K/V staging (register-staged; rows clamped, tail masked later).  Thread tid stages 16-B chunk
    // (tid & 15) of rows (tid >> 4) + 16 i, i < CPT; its K/V row pointers advance by one tile per step
    // and only a tile that crosses k_len takes the clamped slow path.
    u32x4 kreg[CPT], vreg[CPT];
    const int srow = tid >> 4, sch = tid & 15;
    const bf16_t* kbase;
    const bf16_t* vbase;
    if constexpr (SWIN) {
        kbase = p.k + hoff + sch * 8;
        vbase = p.v + hoff + sch * 8;
    } else {
        kbase = p.k + (int64_t)(k_start + t_begin * KT + srow) * p.ldk + hoff + sch * 8;
        vbase = p.v + (int64_t)(v_start + t_begin * KT + srow) * p.ldv + hoff + sch * 8;
    }
    const int64_t k16 = (int64_t)(T / 16) * p.ldk, v16 = (int64_t)(T / 16) * p.ldv;
    auto load_tile = [&](int kt) {
        if constexpr (SWIN) {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int r = swin_row(srow + i * (T / 16));
                kreg[i] = *reinterpret_cast<const u32x4*>(kbase + (int64_t)r * p.ldk);
                vreg[i] = *reinterpret_cast<const u32x4*>(vbase + (int64_t)r * p.ldv);
            }
        } else if ((kt + 1) * KT <= k_len) {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                kreg[i] = *reinterpret_cast<const u32x4*>(kbase + i * k16);
                vreg[i] = *reinterpret_cast<const u32x4*>(vbase + i * v16);
            }
        } else {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int over = kt * KT + srow + i * (T / 16) - (k_len - 1);
                const int64_t back = over > 0 ? over : 0;
                kreg[i] = *reinterpret_cast<const u32x4*>(kbase + i * k16 - back * p.ldk);
                vreg[i] = *reinterpret_cast<const u32x4*>(vbase + i * v16 - back * p.ldv);
            }
        }
        kbase += KT * p.ldk;
        vbase += KT * p.ldv;
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
    float m_run = NEG, l_run = 0.f;  // m_run in raw score units (before * c)
    const float c = p.c;

    if constexpr (QKN) {
        // the fused full-width q/k RMSNorm (rf_qk_norm_rope's arithmetic: row scale, then weight; q also carries
        // the softmax scale): every load is issued before any is used (q and the K/V tile above/here, then the
        // row sums and weights), the key rows' 1 / rms and both weight vectors go through LDS once, and the
        // transforms are branch-free (qk_w is never null on this path)
        load_tile(t_begin);
        float sq = 0.f, sk = 0.f, gq = 0.f, gk = 0.f;
        sq = qk_inv_rms(p, qrow, 0) * p.qk_scale;
        if (tid < KT) sk = qk_inv_rms(p, swin_row(tid), 1);
        if (tid < HD) {
            gq = p.qk_w[hoff + tid];
            gk = p.qk_w[p.qk_dim + hoff + tid];
        }
        if (tid < KT) qkn_inv[tid] = sk;
        if (tid < HD) {
            qkn_gq[tid] = gq;
            qkn_gk[tid] = gk;
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < 8; ++s)
            qf[s] = __builtin_bit_cast(bf16x8, qk_scale8(__builtin_bit_cast(u32x4, qf[s]), sq,
                                                           qkn_gq + 16 * s + 8 * half));
#pragma unroll
        for (int i = 0; i < CPT; ++i) kreg[i] = qk_scale8(kreg[i], qkn_inv[srow + i * (T / 16)], qkn_gk + sch * 8);
        write_tile(0);
    } else if (t_begin < t_end) {
        load_tile(t_begin);
        write_tile(0);
    }
    __syncthreads();

    // tr-read lane geometry (ds_read_b64_tr_b16): group g = lane>>4, lane 4qq+pp of the group
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;

    for (int kt = t_begin; kt < t_end; ++kt) {
        const int cur = SWIN ? 0 : ((kt - t_begin) & 1);
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

        // next tile's K/V loads fly under the softmax and the PV MFMAs (written to LDS after them)
        if (!SWIN && kt + 1 < t_end) load_tile(kt + 1);

        // ---- mask (tail tile / swin regions only), row max
        bool masked;
        if constexpr (SWIN) {
            masked = p.shift > 0;
        } else {
            masked = (kt + 1) * KT > k_len;
        }
        if (masked) {
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = b * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                    bool drop;
                    if constexpr (SWIN) {
                        drop = swin_label(key) != qlabel;
                    } else {
                        drop = kt * KT + key >= k_len;
                    }
                    s[b][r] = drop ? NEG : s[b][r];
                }
        }
        float mt = max3(s[0][0], s[0][1], s[0][2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) mt = max3(mt, s[0][r], s[0][r + 1]);
        mt = max3(mt, s[0][15], s[1][0]);
#pragma unroll
        for (int r = 1; r < 15; r += 2) mt = max3(mt, s[1][r], s[1][r + 1]);
        mt = __builtin_fmaxf(mt, s[1][15]);
        mt = __builtin_fmaxf(mt, __shfl_xor(mt, 32, 64));
        // deferred rescale (guide T13): keep the running max unless some row of the wave grew by
        // more than RESCALE_LOG2 (in log2 units); probabilities are then bounded by 2^RESCALE_LOG2,
        // harmless for the fp32 sums and for bf16 P (relative precision is scale-free).
        if (__any((mt - m_run) * c > RESCALE_LOG2)) {
            const float m_new = __builtin_fmaxf(m_run, mt);
            const float alpha = fast_exp2((m_run - m_new) * c);
            l_run *= alpha;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
            m_run = m_new;
        }
        const float mc = m_run * c;
        float ls = 0.f;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float pv = fast_exp2(__builtin_fmaf(s[b][r], c, -mc));
                s[b][r] = pv;
                ls += pv;
            }
        l_run += ls;

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

        if (!SWIN && kt + 1 < t_end) write_tile(cur ^ 1);
        __syncthreads();
    }

    // ---- epilogue: lane owns query (lane & 31), d = dt*32 + 8 gq + 4 half + 0..3
    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
    int orow;
    if constexpr (SWIN) {
        orow = swin_row(qi);
    } else {
        const int qq2 = q0 + qi;
        if (qq2 >= q_len) return;
        orow = q_start + qq2;
    }
    if (!SWIN && p.n_split > 1) {
        // unnormalised partials for rf_attn_combine (rows indexed like the output)
        float* po = p.part_o + ((int64_t)split * p.part_rows + orow) * (p.n_heads * HD) + hoff;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int gq = 0; gq < 4; ++gq)
                *reinterpret_cast<float4*>(po + dt * 32 + 8 * gq + 4 * half) =
                    make_float4(o[dt][4 * gq], o[dt][4 * gq + 1], o[dt][4 * gq + 2], o[dt][4 * gq + 3]);
        if (half == 0) {
            float* pm = p.part_ml + (((int64_t)split * p.part_rows + orow) * p.n_heads + h) * 2;
            pm[0] = m_run * c;
            pm[1] = l_tot;
        }
        return;
    }
    const float inv = l_tot > 0.f ? 1.0f / l_tot : 0.f;
    bf16_t* dst = p.o + (int64_t)orow * p.ldo + hoff;
    if constexpr (OF16) {  // fp16 O (Swin): range flag as in the stream-K epilogue
        float amax = 0.f;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int r = 0; r < 16; r += 2) amax = amax3(amax, o[dt][r] * inv, o[dt][r + 1] * inv);
        if (p.range && !f16_in_range(amax)) report_f16_range(p.range, RF_RANGE_ATTN);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            uint2 pk;
            pk.x = pack_o<OF16>(o[dt][4 * gq + 0] * inv, o[dt][4 * gq + 1] * inv);
            pk.y = pack_o<OF16>(o[dt][4 * gq + 2] * inv, o[dt][4 * gq + 3] * inv);
            *reinterpret_cast<uint2*>(dst + dt * 32 + 8 * gq + 4 * half) = pk;
        }
}

// ---------------------------------------------------------------------------------------------
// Varlen kernel (rf_attn_fwd): 8 waves x 32 query rows per workgroup, K/V tiles streamed
// global->LDS by DMA (global_load_lds, no VGPR staging) through a 3-stage ring, and the loop
// software-pipelined inside each wave: S(t+1) = K(t+1) Q^T is issued in the same basic block as
// the softmax of S(t), so the exp/convert VALU work of one tile runs under the QK^T MFMAs of the
// next one (the loop was VALU-bound when the two phases were serial).  One barrier per tile.
// The per-tile row max is taken per lane half only (no cross-lane exchange on the common path):
// the running max m is shared by both halves and only moves, with one exchange, in the rare
// deferred-rescale branch.
constexpr int NW3 = 8;
constexpr int QBLK3 = NW3 * 32;
constexpr int NST3 = 3;

template <int N>
RF_DEV void attn_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

#ifdef RF_STUDY  // the legacy per-unit split-KV kernel: study build only (make study)
__global__ __launch_bounds__(NW3 * 64, 1) void attn_v3_kernel(AttnArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[NST3 * 2 * TILE_BYTES];  // 96 KiB

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int half = lane >> 5;

    // XCD-aware bijective remap (see attn_fwd_kernel)
    const int nwg = p.n_total, hwid = blockIdx.x;
    const int xcd = hwid & 7, qd = nwg >> 3, rm = nwg & 7;
    int id = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + (hwid >> 3);
    const int qb = id % p.n_qblk;
    id /= p.n_qblk;
    const int split = id % p.n_split;
    id /= p.n_split;
    const int h = id % p.n_heads;
    const int prob = id / p.n_heads;
    const int32_t* d = p.problems + prob * 5;
    const int q_start = d[0], q_len = d[1], k_start = d[2], k_len = d[3], v_start = d[4];
    const int q0 = qb * QBLK3;
    if (q0 >= q_len) return;
    const int nt_all = (k_len + KT - 1) / KT;
    const int per = (nt_all + p.n_split - 1) / p.n_split;
    const int t_begin = split * per;
    const int t_end = min(nt_all, t_begin + per);
    const int nt = t_end - t_begin;
    const int hoff = h * HD;

    // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[q][16 s + 8 half + 0..7]
    const int qi = wave * 32 + (lane & 31);
    bf16x8 qf[8];
    {
        const int qq = q0 + qi;
        const int qrow = q_start + (qq < q_len ? qq : q_len - 1);
        const bf16_t* src = p.q + (int64_t)qrow * p.ldq + hoff + 8 * half;
#pragma unroll
        for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(src + 16 * s);
    }

    // ---- DMA geometry: a 1-KiB piece is 4 tile rows; wave w fills K and V pieces 2w and 2w+1.
    // Lane l writes LDS bytes piece*1024 + 16 l, i.e. row 4 piece + (l >> 4), physical chunk l & 15,
    // so it fetches the logical chunk that the swizzle maps there.
    const int r_a = 8 * wave + (lane >> 4), r_b = r_a + 4;
    const int lc_a = (lane & 15) ^ (((r_a & 3) << 2) | ((r_a >> 2) & 3));
    const int lc_b = (lane & 15) ^ (((r_b & 3) << 2) | ((r_b >> 2) & 3));
    const bf16_t* ka = p.k + (int64_t)(k_start + t_begin * KT + r_a) * p.ldk + hoff + lc_a * 8;
    const bf16_t* kb = p.k + (int64_t)(k_start + t_begin * KT + r_b) * p.ldk + hoff + lc_b * 8;
    const bf16_t* va = p.v + (int64_t)(v_start + t_begin * KT + r_a) * p.ldv + hoff + lc_a * 8;
    const bf16_t* vb = p.v + (int64_t)(v_start + t_begin * KT + r_b) * p.ldv + hoff + lc_b * 8;
    const int64_t kstep = KT * p.ldk, vstep = KT * p.ldv;
    auto issue = [&](int kt, int stage) {  // called for kt = t_begin, t_begin + 1, ... in order
        char* kd = smem + stage * 2 * TILE_BYTES + wave * 2048;
        char* vd = kd + TILE_BYTES;
        if ((kt + 1) * KT <= k_len) {
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, ka), LDS_PTR(void, kd), 16, 0, 0);
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, kb), LDS_PTR(void, kd + 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, va), LDS_PTR(void, vd), 16, 0, 0);
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, vb), LDS_PTR(void, vd + 1024), 16, 0, 0);
        } else {  // tail tile: rows past k_len re-read row k_len - 1 (masked out of the softmax)
            const int oa = kt * KT + r_a - (k_len - 1), ob = kt * KT + r_b - (k_len - 1);
            const int64_t ba = oa > 0 ? oa : 0, bb = ob > 0 ? ob : 0;
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, ka - ba * p.ldk), LDS_PTR(void, kd), 16, 0, 0);
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, kb - bb * p.ldk), LDS_PTR(void, kd + 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, va - ba * p.ldv), LDS_PTR(void, vd), 16, 0, 0);
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, vb - bb * p.ldv), LDS_PTR(void, vd + 1024), 16, 0, 0);
        }
        ka += kstep;
        kb += kstep;
        va += vstep;
        vb += vstep;
    };

    f32x16 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_run = NEG, l_run = 0.f;  // m_run in raw score units, identical in both lane halves
    const float c = p.c;
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;  // ds_read_b64_tr_b16 lane geometry

    auto qk = [&](const char* kt_lds, f32x16* s) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[b][r] = 0.f;
#pragma unroll
            for (int st = 0; st < 8; ++st) {
                const bf16x8 a =
                    *reinterpret_cast<const bf16x8*>(kt_lds + swz_off(b * 32 + (lane & 31), 2 * st + half));
                s[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[st], s[b], 0, 0, 0);
            }
        }
    };

    if (nt > 0) {
        issue(t_begin, 0);
        if (nt > 1) {
            issue(t_begin + 1, 1);
            attn_wait_vm<4>();
        } else {
            attn_wait_vm<0>();
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    }
    f32x16 s[2];
    if (nt > 0) qk(smem, s);
    int cur = 0, nxt = 1, fre = 2;

    for (int i = 0; i < nt; ++i) {
        const int kt = t_begin + i;
        // tile kt+1 (the only DMA in flight) landed for every wave, and every wave is done with
        // tile kt-1, whose stage now takes tile kt+2
        __builtin_amdgcn_sched_barrier(0);
        attn_wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (i + 2 < nt) issue(kt + 2, fre);

        if ((kt + 1) * KT > k_len) {
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = b * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                    s[b][r] = kt * KT + key >= k_len ? NEG : s[b][r];
                }
        }
        float mt = max3(s[0][0], s[0][1], s[0][2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) mt = max3(mt, s[0][r], s[0][r + 1]);
        mt = max3(mt, s[0][15], s[1][0]);
#pragma unroll
        for (int r = 1; r < 15; r += 2) mt = max3(mt, s[1][r], s[1][r + 1]);
        mt = __builtin_fmaxf(mt, s[1][15]);
        if (__any((mt - m_run) * c > RESCALE_LOG2)) {
            const float mrow = __builtin_fmaxf(mt, __shfl_xor(mt, 32, 64));
            const float m_new = __builtin_fmaxf(m_run, mrow);
            const float alpha = fast_exp2((m_run - m_new) * c);
            l_run *= alpha;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
            m_run = m_new;
        }
        __builtin_amdgcn_sched_barrier(0);

        // ---- one basic block: P(t) = exp2(S c - m c) -> bf16, S(t+1) = K(t+1) Q^T, O^T += V(t)^T P^T
        const char* kl = smem + nxt * 2 * TILE_BYTES;
        const char* vl = smem + cur * 2 * TILE_BYTES + TILE_BYTES;
        const float nm = -m_run * c;
        float ls0 = 0.f, ls1 = 0.f;
        bf16x8 pf[2][2];
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
                const float e0 = fast_exp2(__builtin_fmaf(s[b][r], c, nm));
                const float e1 = fast_exp2(__builtin_fmaf(s[b][r + 1], c, nm));
                ls0 += e0;
                ls1 += e1;
                pf[b][r >> 3][r & 7] = (__bf16)e0;
                pf[b][r >> 3][(r & 7) + 1] = (__bf16)e1;
            }
        l_run += ls0 + ls1;
        qk(kl, s);  // last iteration: harmless MFMAs on a stale stage, result unused
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            const int col = dt * 32 + 16 * (g & 1) + 4 * pp;
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int sp = 0; sp < 2; ++sp) {
                    const int row = b * 32 + 16 * sp + 4 * (g >> 1) + qq;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        LDS_PTR(s16x4, vl + swz_off(row, col >> 3) + (col & 7) * 2));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        LDS_PTR(s16x4, vl + swz_off(row + 8, col >> 3) + (col & 7) * 2));
                    const auto a16 = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                    o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a16), pf[b][sp],
                                                                    o[dt], 0, 0, 0);
                }
        }
        const int t0 = cur;
        cur = nxt;
        nxt = fre;
        fre = t0;
    }

    // ---- epilogue: lane owns query (lane & 31), d = dt*32 + 8 gq + 4 half + 0..3
    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
    const int qrow_o = q0 + qi;
    if (qrow_o >= q_len) return;
    const int orow = q_start + qrow_o;
    if (p.n_split > 1) {
        float* po = p.part_o + ((int64_t)split * p.part_rows + orow) * (p.n_heads * HD) + hoff;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int gq = 0; gq < 4; ++gq)
                *reinterpret_cast<float4*>(po + dt * 32 + 8 * gq + 4 * half) =
                    make_float4(o[dt][4 * gq], o[dt][4 * gq + 1], o[dt][4 * gq + 2], o[dt][4 * gq + 3]);
        if (half == 0) {
            float* pm = p.part_ml + (((int64_t)split * p.part_rows + orow) * p.n_heads + h) * 2;
            pm[0] = nt > 0 ? m_run * c : NEG;
            pm[1] = l_tot;
        }
        return;
    }
    const float inv = l_tot > 0.f ? 1.0f / l_tot : 0.f;
    bf16_t* dst = p.o + (int64_t)orow * p.ldo + hoff;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            uint2 pk;
            pk.x = p.o_f16 ? pack_f16x2(o[dt][4 * gq + 0] * inv, o[dt][4 * gq + 1] * inv)
                           : pack_bf16x2(o[dt][4 * gq + 0] * inv, o[dt][4 * gq + 1] * inv);
            pk.y = p.o_f16 ? pack_f16x2(o[dt][4 * gq + 2] * inv, o[dt][4 * gq + 3] * inv)
                           : pack_bf16x2(o[dt][4 * gq + 2] * inv, o[dt][4 * gq + 3] * inv);
            *reinterpret_cast<uint2*>(dst + dt * 32 + 8 * gq + 4 * half) = pk;
        }
}

#endif  // RF_STUDY

// ---------------------------------------------------------------------------------------------
// Stream-K varlen kernel (rf_attn_fwd with n_split == 0, the default).
//
// Work decomposition: the launch's (problem, head, 256-row q-block, 64-key tile) space is flattened
// and every workgroup of a one-per-CU grid takes an equal contiguous range of it, so the CUs finish
// together whatever the unit count (184 units of 89 tiles on 256 CUs at the bench shape).  A unit
// cut between workgroups is finished by the workgroup holding its first tile (the "owner", which
// reaches that tile at the END of its range): every later piece is published as an unnormalised
// partial (O, m, l in register order, sc1 stores + flag) and folded into the owner's registers
// before its epilogue.  Q-blocks split each problem's rows evenly (<= 256 rows each).
//
// Main loop, per 64-key tile t (8 waves x 32 query rows), two half-tile phases split by barriers:
//   A(t): softmax of S(t) (exp2 / bf16 pack / row sums: the VALU work) woven into
//         S(t+1) = K(t+1) Q^T (16 v_mfma_f32_32x32x16_bf16, query on the lane);
//   B(t): O^T += V(t)^T P(t)^T (16 MFMAs, P as the B operand with no lane movement).
//   Waves 4-7 run one phase behind waves 0-3, so each SIMD pairs A of one wave with B of its partner
//   (VALU beside MFMA instead of both waves fighting over the same pipe).
//   * K(t+2) / V(t+1) arrive by LDS-DMA at the top of A(t) / B(t) (inline asm, so hipcc does not
//     put a vmcnt(0) in front of the transposed V reads) into 2-deep K and V rings (64 KiB), and are
//     waited for at the end of that phase; the loop is unrolled by 2 so every LDS offset is an
//     immediate.
//   * q arrives pre-scaled by scale*log2(e) (rf_qk_norm_rope seg0_scale) and the QK^T chain starts
//     from C = -m (the running max), so P = exp2(S) needs no per-score FMA (UNIT) and no per-tile row
//     max: the running max (exact on a piece's first tile) is only re-based (deferred rescale, guide
//     T13) when a half-row sum of P(t) exceeds 2^12 (which bounds every P by 2^12), checked at the seam
//     after A(t); that tile's P is then recomputed on the new base.

constexpr int NW5 = 8;
constexpr int QB5 = NW5 * 32;
constexpr int K5 = 0;                  // K ring: 2 x 16 KiB
constexpr int V5 = 2 * TILE_BYTES;     // V ring: 2 x 16 KiB
constexpr int Q5 = 4 * TILE_BYTES;     // Q image of a piece: 8 waves x 8 KiB (attn_sk_kernel)
constexpr int QS5 = Q5 + 8 * 8192;     // the piece's q row sums (rf_attn_fwd_qn): 8 waves x 32 rows x 32 B
constexpr int SK5_MAX_GRID = 512;
static_assert(KT == rf::ATTN_KT && QB5 == rf::ATTN_QB && SK5_MAX_GRID == rf::ATTN_MAX_GRID,
              "attn_sched.cpp prices the kernel's geometry");
constexpr int PIECE_O = QB5 * HD;                // f32, register order
constexpr int PIECE_FLOATS = PIECE_O + QB5 * 2 * 2;  // + (m, l) per lane

RF_DEV float vmax3(float a, float b, float c) { return __builtin_fmaxf(__builtin_fmaxf(a, b), c); }  // v_max3_f32

// two f32 -> one packed bf16x2 (RNE, as the (__bf16) cast), pinned where it is written (volatile asm)
RF_DEV uint32_t cvt_pk_bf16(float lo, float hi) {
    uint32_t r;
    asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
    return r;
}
// two f32 -> one packed fp16x2 (RNE), pinned like cvt_pk_bf16
RF_DEV uint32_t cvt_pk_f16(float lo, float hi) {
    uint32_t r;
    asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
    return r;
}
// the P operand format of the stream-K kernel follows its q/k/v format (F16: fp16, else bf16).  Fragments are
// carried as bf16x8 bit containers either way and re-typed at the MFMA (mfma32).
template <bool F16>
RF_DEV uint32_t cvt_pk_p(float lo, float hi) { return F16 ? cvt_pk_f16(lo, hi) : cvt_pk_bf16(lo, hi); }
template <bool F16>
RF_DEV __bf16 to_p16(float e) {
    if constexpr (F16) return __builtin_bit_cast(__bf16, (_Float16)e);
    else return (__bf16)e;
}
// v_mfma_f32_32x32x16_bf16 / _f16 (same cycles) on 8 x 16-bit fragments
template <bool F16>
RF_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
    if constexpr (F16)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                      0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// DBG & 2048 (study build, timing only): every v_mfma_f32_32x32x16 of the tile loop replaced by two
// v_mfma_f32_16x16x32 on the same operand registers into two 4-register slices of its accumulator — the same FLOP
// and the same VALU / LDS work per tile, issued in the 16x16x32 shape: a probe of that shape's clock and issue cost
// in this loop (MI355X_MICROARCH "DVFS give-back" item 7) before building the full 16x16x32 kernel.  Garbage results.
template <bool F16>
RF_DEV f32x16 mfma16x2(const bf16x8& a, const bf16x8& b, const f32x16& c) {
    f32x4 lo = {c[0], c[1], c[2], c[3]}, hi = {c[4], c[5], c[6], c[7]};
    if constexpr (F16) {
        lo = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), lo, 0, 0,
                                                   0);
        hi = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), hi, 0, 0,
                                                   0);
    } else {
        lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, lo, 0, 0, 0);
        hi = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, hi, 0, 0, 0);
    }
    f32x16 r = c;
    r[0] = lo[0], r[1] = lo[1], r[2] = lo[2], r[3] = lo[3];
    r[4] = hi[0], r[5] = hi[1], r[6] = hi[2], r[7] = hi[3];
    return r;
}
// dword w (0..3) of an MFMA bf16x8 operand
RF_DEV void set_pk(bf16x8& f, int w, uint32_t v) {
    u32x4 u = __builtin_bit_cast(u32x4, f);
    u[w] = v;
    f = __builtin_bit_cast(bf16x8, u);
}

// x through an empty asm: computations from the result cannot be hoisted out of the enclosing loop (hoisted
// lane-constant offsets of the piece epilogue were spilled across the tile loop and reloaded behind vmcnt(0))
RF_DEV int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

// One 1-KiB LDS-DMA piece: lane l's 16 B land at LDS byte lds + 16 l.  Inline asm so hipcc neither
// counts it (the loop waits with its own vmcnt) nor guards later ds_read_b64_tr_b16 with vmcnt(0).
// M0 is declared clobbered (hipcc warns: reserved register); the kernel has no other M0 user (checked
// in the .s: every m0 access is one of these statements), so it is not saved/restored (guide §5.7).
RF_DEV void dma_piece(const bf16_t* g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds) : "memory", "m0");
}

// DBG (diagnostic builds only, RF_ATTN_DBG; results are garbage): 1 = no K/V DMA in the loop,
// 2 = no top-of-tile wait + barrier, 4 = no PV MFMAs, 8 = no exp2 (P = bf16(S)), 16 = no QK MFMAs,
// 32 = s_memtime stamps per segment (cycles summed over tiles) into the workspace's last piece slot,
// 64 = no static priority for waves 4-7, 1024 = keep the QK^T chains' C operand (-m) live across tiles and
// rewrite it only where m moves (rebase) — valid results, but it spills, see MINIT_EVERY
// IF16: q, k, v (and P) as fp16 on v_mfma_f32_32x32x16_f16 — the reference's default half precision hands
// flash_attn_varlen_* fp16 operands (rendering_pipeline.py:37, attention.py:166-172); else bf16.  P <= 2^thr
// (= 2^12 by default) stays inside fp16's range.
template <bool UNIT, int DBG = 0, bool OF16 = false, bool IF16 = false>
__global__ __launch_bounds__(NW5 * 64, 1) void attn_sk_kernel(AttnArgs p) {
    // SPLIT: half of each tile's softmax (keys 32-63) moves from phase A (QK^T, VALU-heavy) into the first
    // half of phase B (PV, VALU-light), balancing the two phases that share each SIMD; DBG & 128 = unsplit
    constexpr bool SPLIT = (DBG & 128) != 0;  // measured: no gain (the per-tile total stays ~3,200 cycles)
    // CVT_PIN: the bf16 packs of P are inline-asm v_cvt_pk_bf16_f32 in their MFMA gaps (hipcc otherwise
    // sinks all 16 of them into one VALU burst after the last QK^T MFMA); DBG & 256 = compiler casts
    constexpr bool CVT_PIN = !(DBG & 256);
    // MINIT_EVERY: the 16 C-operand registers (-m) are rebuilt by one v_mov per PV gap each tile.  DBG & 1024
    // keeps them live across tiles and rewrites them only on rebase: 16 more live VGPRs, which spill (17-23 VGPRs
    // to scratch at 2 waves/SIMD), so the per-tile form stays the default
    constexpr bool MINIT_EVERY = (DBG & 1024) == 0;
    constexpr auto x_blk = [](int x) { return x >> 4; };
    constexpr auto x_sp = [](int x) { return (x >> 3) & 1; };
    // K ring, V ring (2 x 16 KiB each), then the Q image of the next piece (8 waves x 8 KiB)
    __shared__ __attribute__((aligned(16))) char smem[QS5 + NW5 * 1024];  // 136 KiB

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR): row windows, flags
    const int half = lane >> 5;
    const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(char, smem);
    const bool late = __builtin_amdgcn_readfirstlane(tid) >= 256;  // waves 4-7 (SIMD partners of 0-3)
    // the second-dispatched half loses VALU arbitration to its older partner: static priority (guide T5)
    if constexpr (!(DBG & 64))
        if (late) __builtin_amdgcn_s_setprio(1);

    const int nwg = gridDim.x, hw = blockIdx.x;
    int gend = 0;
    const int wg = sk_attn_block(p, hw, nwg, gend);  // logical index: ranges, partial slots and flags
    if (wg < 0) {  // a range table that does not fit this launch: refuse it (never read past the problems)
        if (tid == 0) report_device_error(p.err, RF_DEVERR_SK_SCHED);
        return;
    }
    // The problem table and the range table are read-only for the launch: constant-address-space (scalar) loads
    // keep them off the vector memory counter.  (As vector loads, their results sat in VGPRs across pieces and the
    // compiler's wait for them at the next piece's top was a vmcnt(0) that also drained the previous piece's
    // partial stores before the next piece issued a single load.)
    const RF_CONST int32_t* probs = (const RF_CONST int32_t*)p.problems;
    const RF_CONST int64_t* bnds = (const RF_CONST int64_t*)p.bounds;
    int64_t it = bnds[wg];
    const int64_t it_end = bnds[wg + 1];

    const float c = UNIT ? 1.f : p.c;
    const float inv_c = UNIT ? 1.f : 1.f / p.c;
    const float sum_thr = exp2f(p.thr);  // half-row sum of one tile's P above which the running max moves
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;  // ds_read_b64_tr_b16 lane geometry
    // LDS image of a K/V tile (guide T10 image (a)): 8-row x 32-column subtiles of 512 B,
    // off(row, ch) = 2048 (row >> 3) + 512 (ch >> 2) + 64 (row & 7) + 16 ((ch & 3) ^ ((row >> 2) & 3)),
    // conflict-free for the K ds_read_b128 and the V ds_read_b64_tr_b16 of the 32x32x16 operands, and
    // every read is one of two lane bases per operand plus an immediate.
    // DMA: wave w fills row group w (pieces 2w, 2w+1 = column groups {0,1}, {2,3}); lane l writes
    // 16 B at piece + 16 l = row 8w + ((l >> 2) & 7), physical chunk l & 3 of column group (l >> 5) (+2).
    const int d_row = 8 * wave + ((lane >> 2) & 7);
    const int d_ch = 4 * (lane >> 5) + ((lane & 3) ^ ((d_row >> 2) & 3));
    const int kr = lane & 31;
    const int kb_even = 2048 * (kr >> 3) + 64 * (kr & 7) + 16 * (half ^ ((kr >> 2) & 3));
    const int kb_odd = 2048 * (kr >> 3) + 64 * (kr & 7) + 16 * ((2 + half) ^ ((kr >> 2) & 3));
    const int vb_lo = 64 * (4 * (g >> 1) + qq) + 16 * ((2 * (g & 1) + (pp >> 1)) ^ ((g >> 1) & 3)) + 8 * (pp & 1);
    const int vb_hi = 64 * (4 * (g >> 1) + qq) + 16 * ((2 * (g & 1) + (pp >> 1)) ^ ((2 + (g >> 1)) & 3)) + 8 * (pp & 1);

    int pi = -1;
    int64_t base = 0, usz = 0;
    int q_start = 0, q_len = 0, k_start = 0, k_len = 0, v_start = 0, nqb = 1, nt = 1;
    // the current piece: tiles [kt0, kt1) of its unit (n of them), query rows [q0, q1) of head column hoff
    int kt0 = 0, kt1 = 0, n = 0, q0 = 0, q1 = 0, hoff = 0;
    int64_t unit_end = 0;
    bool active = false;  // wave-uniform: this wave owns at least one row
    // DBG & 32: top wait, K DMA issue, mask+max+check, A, seam wait, V DMA issue, B, tiles
    uint64_t stamp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t t_prev = 0, clk0 = 0, ref0 = 0;
    if constexpr (DBG & 32) {
        clk0 = __builtin_amdgcn_s_memtime();
        ref0 = __builtin_amdgcn_s_memrealtime();
    }
    auto stamp_at = [&](int k) {
        if constexpr (DBG & 32) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            stamp[k] += now - t_prev;
            t_prev = now;
        }
    };
    auto next_piece = [&]() {  // the piece holding tile `it` (scalar: SGPRs only)
        while (it >= base + usz) {  // advance to the problem holding tile `it`
            base += usz;
            ++pi;
            const RF_CONST int32_t* d = probs + 5 * pi;
            q_start = d[0];
            q_len = d[1];
            k_start = d[2];
            k_len = d[3];
            v_start = d[4];
            nqb = (q_len + QB5 - 1) / QB5;
            nt = (k_len + KT - 1) / KT;
            usz = (int64_t)p.n_heads * nqb * nt;
        }
        const int64_t rel = it - base;
        const int unit = (int)(rel / nt);
        kt0 = (int)(rel - (int64_t)unit * nt);
        kt1 = (int)min((int64_t)nt, kt0 + (it_end - it));
        n = kt1 - kt0;
        unit_end = base + (int64_t)(unit + 1) * nt;
        it += n;
        const int h = unit / nqb, qb = unit - (unit / nqb) * nqb;
        q0 = (int)((int64_t)qb * q_len / nqb);
        q1 = (int)((int64_t)(qb + 1) * q_len / nqb);
        hoff = h * HD;
        active = q0 + wave * 32 < q1;
    };

    const bf16_t* kp = nullptr;
    const bf16_t* vp = nullptr;
    int64_t kstep = 0, vstep = 0;
    // tiles are issued in order; rows past k_len (tail tile) re-read row k_len - 1, masked later
    auto issue = [&](const bf16_t*& src, int64_t ld, int64_t step, int t, uint32_t dst) {
        const uint32_t d0 = __builtin_amdgcn_readfirstlane(dst + wave * 2048);
        if ((t + 1) * KT <= k_len) {
            dma_piece(src, d0);
            dma_piece(src + 64, d0 + 1024);
        } else {
            const int over = t * KT + opaque(d_row) - (k_len - 1);
            const bf16_t* a = src - (int64_t)(over > 0 ? over : 0) * ld;
            dma_piece(a, d0);
            dma_piece(a + 64, d0 + 1024);
        }
        src += step;
    };
    // A piece's first loads, in vector-memory-counter order: Q (8 LDS-DMA pieces per wave into the wave's 8 KiB
    // of the Q image: piece st holds lane l's 16 B of qf[st], so the ds_read_b128 back is lane-linear), K(t0),
    // K(t0+1) when n > 1 (the K ring is free once every wave is past the previous piece's last phase A), then,
    // after a barrier, V(t0) (its slot may still be read by the partner group's last phase B).  Issued at the end
    // of the previous piece's tile loop, AHEAD of its partial or O stores: vmcnt counts loads and stores together
    // in issue order, so the piece's counted waits below leave the younger stores in flight (nst of them).
    auto issue_qk = [&]() {
        {
            const int ql = wave * 32 + (opaque(lane) & 31);
            const int qrow = q_start + min(q0 + ql, q1 - 1);
            const bf16_t* src = p.q + (int64_t)qrow * p.ldq + hoff + 8 * half;
            const uint32_t d0 = __builtin_amdgcn_readfirstlane(lds0 + Q5 + wave * 8192);
#pragma unroll
            for (int st = 0; st < 8; ++st) dma_piece(src + 16 * st, d0 + 1024 * st);
            if (p.qk_ss) {  // lane l: 16 B (4 of the 8 slots) of row l >> 1 of the wave's 32 rows, lane-linear in LDS
                const int srow = q_start + min(q0 + wave * 32 + (opaque(lane) >> 1), q1 - 1);
                const float* ssrc = p.qk_ss + (int64_t)srow * p.qk_ld + 4 * (lane & 1);
                dma_piece(reinterpret_cast<const bf16_t*>(ssrc), __builtin_amdgcn_readfirstlane(lds0 + QS5 + wave * 1024));
            }
        }
        kp = p.k + (int64_t)(k_start + kt0 * KT + d_row) * p.ldk + hoff + 8 * d_ch;
        vp = p.v + (int64_t)(v_start + kt0 * KT + d_row) * p.ldv + hoff + 8 * d_ch;
        kstep = KT * p.ldk;
        vstep = KT * p.ldv;
        issue(kp, p.ldk, kstep, kt0, lds0 + K5);
        if (n > 1) issue(kp, p.ldk, kstep, kt0 + 1, lds0 + K5 + TILE_BYTES);
    };
    auto issue_v0 = [&]() { issue(vp, p.ldv, vstep, kt0, lds0 + V5); };

    // pend: the previous piece's partial is stored but its flag not raised; it goes up after this piece's first
    // barrier, which every wave passes after a vmcnt(0) that covers both the piece's loads and those stores
    bool pend = false;
    auto raise_pend = [&]() {
        if (pend) {
            if (tid == 0) __hip_atomic_store(p.flag + wg, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pend = false;
        }
    };
    const bool any = it < it_end;
    if (any) {
        next_piece();
        issue_qk();
        issue_v0();
    }
    while (any) {  // one pass per piece; ends after the range's last piece
        uint64_t t_piece = 0;  // DBG & 32: piece prologue cycles -> stamp[6]
        if constexpr (DBG & 32) t_piece = __builtin_amdgcn_s_memtime();
        // the piece's loads (Q, K(t0), K(t0+1), V(t0)) and the previous piece's stores, issued after them, completed
        // for this wave: the wait is the longer of the two flights, not their sum ...
        attn_wait_vm<0>();
        __builtin_amdgcn_s_barrier();  // ... and for every wave
        __builtin_amdgcn_sched_barrier(0);
        raise_pend();  // every storing wave drained its partial stores before this barrier
        bf16x8 qf[8];
#pragma unroll
        for (int st = 0; st < 8; ++st)
            qf[st] = *reinterpret_cast<const bf16x8*>(smem + Q5 + wave * 8192 + 1024 * st + 16 * lane);
        if (p.qk_ss) {  // the q norm's 1 / rms (and the softmax scale) of this lane's query row, folded into its Q
            const char* sp = smem + QS5 + wave * 1024 + 32 * (lane & 31);
            const f32x4 a0 = *reinterpret_cast<const f32x4*>(sp), a1 = *reinterpret_cast<const f32x4*>(sp + 16);
            const float sum = ((a0[0] + a0[1]) + (a0[2] + a0[3])) + ((a1[0] + a1[1]) + (a1[2] + a1[3]));
            const float f = p.qk_scale / sqrtf(sum / (float)p.qk_dim + p.qk_eps);
#pragma unroll
            for (int st = 0; st < 8; ++st) {
                u32x4 u = __builtin_bit_cast(u32x4, qf[st]);
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    u[e] = cvt_pk_bf16(__uint_as_float(u[e] << 16) * f, __uint_as_float(u[e] & 0xffff0000u) * f);
                qf[st] = __builtin_bit_cast(bf16x8, u);
            }
        }
        f32x16 o[4];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
        float m_run = 0.f, l_run = 0.f;  // m_run in exp2 units, identical in both lane halves
        // -m in score units: the C operand of the QK^T chains, rebuilt from m_run in every phase B (a
        // rescale at the seam also shifts the S(t+1) already issued on the old base).
        f32x16 minit;
#pragma unroll
        for (int r = 0; r < 16; ++r) minit[r] = 0.f;

        auto qk = [&](const int koff, f32x16* s) {
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int st = 0; st < 8; ++st) {
                    const bf16x8 a = *reinterpret_cast<const bf16x8*>(smem + koff + (st & 1 ? kb_odd : kb_even) +
                                                                      8192 * b + 512 * (st >> 1));
                    s[b] = mfma32<IF16>(a, qf[st], st == 0 ? minit : s[b]);
                }
        };
        auto mask_tail = [&](f32x16* sv, int t) {  // keys >= k_len of tile t -> -inf (tail tile only)
            if ((t + 1) * KT > k_len) {
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int key = b * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                        sv[b][r] = t * KT + key >= k_len ? NEG : sv[b][r];
                    }
            }
        };
        auto row_max = [&](const f32x16* sv) {
            float mt = vmax3(sv[0][0], sv[0][1], sv[0][2]);
#pragma unroll
            for (int r = 3; r < 15; r += 2) mt = vmax3(mt, sv[0][r], sv[0][r + 1]);
            mt = vmax3(mt, sv[0][15], sv[1][0]);
#pragma unroll
            for (int r = 1; r < 15; r += 2) mt = vmax3(mt, sv[1][r], sv[1][r + 1]);
            return vmax3(mt, sv[1][15], sv[1][15]);
        };
        // rare path: re-base the running max on S's row max (exactly on a piece's first tile).  Everything
        // accumulated so far (O, l) is at the old base and is scaled by alpha; S (and S2, the next tile's
        // scores, already issued on the old base) move with the base.
        auto rebase = [&](f32x16* sv, f32x16* sv2, bool fresh) {
            const float mt = row_max(sv);
            const float mrow = __builtin_fmaxf(mt, __shfl_xor(mt, 32, 64)) * c;
            const float delta = fresh ? mrow : __builtin_fmaxf(mrow, 0.f);
            const float alpha = fresh ? 1.f : fast_exp2(-delta);
            l_run *= alpha;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
            m_run += delta;
            if constexpr (!MINIT_EVERY) {
#pragma unroll
                for (int r = 0; r < 16; ++r) minit[r] = -m_run * inv_c;
            }
            const float ds = delta * inv_c;
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    sv[b][r] -= ds;
                    if (sv2) sv2[b][r] -= ds;
                }
        };


        f32x16 sA[2], sB[2];
        qk(K5, sA);  // raw scores of the piece's first tile (base 0)
        mask_tail(sA, kt0);
        rebase(sA, nullptr, true);
#pragma unroll
        for (int r = 0; r < 16; ++r) minit[r] = -m_run * inv_c;
        // stagger (guide MI355X_MICROARCH "Two waves per SIMD", item 9): waves 4-7 run half a tile behind,
        // so on every SIMD one wave's phase A (QK^T + softmax VALU) pairs with its partner's phase B (PV)
        if (late) __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (DBG & 32) stamp[6] += __builtin_amdgcn_s_memtime() - t_piece;

        // one tile: A(t) = softmax(S(t)) woven into S(t+1) = K(t+1) Q^T; seam; B(t) = PV(t) with the
        // minit rebuild and the row max of S(t+1) woven in; then the (rare) rescale of S(t+1)
        auto body = [&](const int i, auto par_c, f32x16(&s)[2], f32x16(&sn)[2]) {
            constexpr int PAR = decltype(par_c)::value;
            const int t = kt0 + i;
            const bool has_next = i + 1 < n;
            (void)has_next;
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (DBG & 32) t_prev = __builtin_amdgcn_s_memtime();
            if constexpr (!(DBG & 2)) {
                attn_wait_vm<0>();             // K(t+1) and V(t) landed for this wave ...
                __builtin_amdgcn_s_barrier();  // ... and for every wave; K(t) and V(t-1) are free
            }
            __builtin_amdgcn_sched_barrier(0);
            stamp_at(0);

            const int koff = K5 + (PAR ^ 1) * TILE_BYTES;
            const int voff = V5 + PAR * TILE_BYTES;
            auto kread = [&](int j) {  // QK step j: chain b = j & 1, k-slice st = j >> 1
                const int b = j & 1, st = j >> 1;
                return *reinterpret_cast<const bf16x8*>(smem + koff + (st & 1 ? kb_odd : kb_even) + 8192 * b +
                                                        512 * (st >> 1));
            };
            auto vread = [&](int j) {  // PV step j: chain dt = j & 3, key block (b, sp) = j >> 2
                const int dt = j & 3, b = (j >> 2) >> 1, sp = (j >> 2) & 1;
                const int imm = voff + 2048 * (4 * b + 2 * sp) + 512 * dt;
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, smem + imm + vb_lo));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, smem + imm + 2048 + vb_hi));
                return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            };
            bf16x8 kf[3], vf[3];
            bf16x8 pf[2][2];
            float ls[4];

            // ---- phase A: S(t+1) chains b = 0, 1 alternating; each gap: 2 exp2, 2 row-sum adds, 1 bf16 pack
            // of P(t) (SPLIT: the first 8 gaps, keys 0-31 of the tile; keys 32-63 go to phase B); K fragments
            // two MFMAs ahead; K(t+2)'s LDS-DMA rides in gap 1
            if (i > 0) mask_tail(s, t);  // (tile kt0 was masked in the prologue)
            kf[0] = kread(0);
            kf[1] = kread(1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (j + 2 < 16) kf[(j + 2) % 3] = kread(j + 2);
                const int b = j & 1, st = j >> 1;
                if constexpr (DBG & 16) {
                    if (st == 0) sn[b] = minit;
                    asm volatile("" : "+v"(kf[j % 3]));
                } else {
                    if constexpr (DBG & 2048)
                        sn[b] = mfma16x2<IF16>(kf[j % 3], qf[st], st == 0 ? minit : sn[b]);
                    else
                        sn[b] = mfma32<IF16>(kf[j % 3], qf[st], st == 0 ? minit : sn[b]);
                }
                if (!SPLIT || j < 8) {
                    float e[2];
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int x = 2 * j + u;
                        const float v = s[x >> 4][x & 15];
                        e[u] = (DBG & 8) ? v : fast_exp2(UNIT ? v : v * c);
                        ls[x & 3] = j < 2 ? e[u] : ls[x & 3] + e[u];
                        asm volatile("" : "+v"(ls[x & 3]));  // keep the add in this gap (IR passes sink it)
                    }
                    if constexpr (CVT_PIN) {
                        set_pk(pf[j >> 3][(j >> 2) & 1], j & 3, cvt_pk_p<IF16>(e[0], e[1]));
                    } else {
                        pf[j >> 3][(j >> 2) & 1][2 * (j & 3)] = to_p16<IF16>(e[0]);
                        pf[j >> 3][(j >> 2) & 1][2 * (j & 3) + 1] = to_p16<IF16>(e[1]);
                    }
                }
                if constexpr (!(DBG & 1)) {
                    if (j == 1 && i + 2 < n) issue(kp, p.ldk, kstep, t + 2, lds0 + K5 + PAR * TILE_BYTES);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            // ---- overflow check (deferred rescale, guide T13): a half-row sum <= 2^thr bounds every P(t) by
            // 2^thr, so the running max only moves (rare) when some sum exceeds it; the P(t) not yet in O is
            // then recomputed on the new base and S(t+1), issued on the old one, is shifted with it.  SPLIT:
            // checked per 32-key half (here for keys 0-31, in phase B for 32-63: O and l then already hold keys
            // 0-31 on the old base and are scaled with everything else).
            constexpr int XA = SPLIT ? 16 : 32;  // P values produced in phase A
            float l_tile = (ls[0] + ls[1]) + (ls[2] + ls[3]);
            if (__any(l_tile > sum_thr)) {
                rebase(s, sn, false);
                l_tile = 0.f;
#pragma unroll
                for (int x = 0; x < XA; ++x) {
                    const float v = s[x >> 4][x & 15];
                    const float e = fast_exp2(UNIT ? v : v * c);
                    l_tile += e;
                    pf[x >> 4][(x >> 3) & 1][x & 7] = to_p16<IF16>(e);
                }
            }
            l_run += l_tile;
            __builtin_amdgcn_sched_barrier(0);
            stamp_at(1);
            // ---- half-tile seam: K(t+2) landed for this wave; the partner group switches phase
            if constexpr (!(DBG & 2)) {
                attn_wait_vm<0>();
                __builtin_amdgcn_s_barrier();
            }
            __builtin_amdgcn_sched_barrier(0);
            stamp_at(2);

            // ---- phase B: four O chains alternating; V^T fragments two MFMAs ahead; V(t+1)'s LDS-DMA in gap
            // 1.  SPLIT: gaps 0-7 (PV of keys 0-31) produce P for keys 32-63, checked before gap 8; gaps 8-15
            // rebuild minit (the C operand of the next QK^T chains), two registers each.  Unsplit: one minit
            // register per gap.
            vf[0] = vread(0);
            vf[1] = vread(1);
            __builtin_amdgcn_sched_barrier(0);
            float l2 = 0.f;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (j + 2 < 16) vf[(j + 2) % 3] = vread(j + 2);
                const int dt = j & 3, b = (j >> 2) >> 1, sp = (j >> 2) & 1;
                if (SPLIT && j == 8) {
                    l2 = (ls[0] + ls[1]) + (ls[2] + ls[3]);
                    if (__any(l2 > sum_thr)) {
                        rebase(s, sn, false);
                        l2 = 0.f;
#pragma unroll
                        for (int x = 16; x < 32; ++x) {
                            const float v = s[x >> 4][x & 15];
                            const float e = fast_exp2(UNIT ? v : v * c);
                            l2 += e;
                            pf[x >> 4][(x >> 3) & 1][x & 7] = to_p16<IF16>(e);
                        }
                    }
                    l_run += l2;
                }
                if constexpr (DBG & 4) {
                    asm volatile("" : "+v"(vf[j % 3]), "+v"(pf[b][sp]));
                } else {
                    if constexpr (DBG & 2048)
                        o[dt] = mfma16x2<IF16>(vf[j % 3], pf[b][sp], o[dt]);
                    else
                        o[dt] = mfma32<IF16>(vf[j % 3], pf[b][sp], o[dt]);
                }
                if (SPLIT && j < 8) {
                    float e[2];
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int x = 16 + 2 * j + u;
                        const float v = s[x >> 4][x & 15];
                        e[u] = (DBG & 8) ? v : fast_exp2(UNIT ? v : v * c);
                        ls[x & 3] = j < 2 ? e[u] : ls[x & 3] + e[u];
                        asm volatile("" : "+v"(ls[x & 3]));
                    }
                    if constexpr (CVT_PIN) {
                        set_pk(pf[x_blk(16 + 2 * j)][x_sp(16 + 2 * j)], j & 3, cvt_pk_p<IF16>(e[0], e[1]));
                    } else {
                        pf[x_blk(16 + 2 * j)][x_sp(16 + 2 * j)][(2 * j) & 7] = to_p16<IF16>(e[0]);
                        pf[x_blk(16 + 2 * j)][x_sp(16 + 2 * j)][(2 * j + 1) & 7] = to_p16<IF16>(e[1]);
                    }
                } else if (SPLIT) {
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int r = 2 * (j - 8) + u;
                        minit[r] = -m_run * inv_c;
                        asm volatile("" : "+v"(minit[r]));  // keep the v_mov in this gap
                    }
                } else if constexpr (MINIT_EVERY) {
                    minit[j] = -m_run * inv_c;
                    asm volatile("" : "+v"(minit[j]));  // one v_mov per PV gap (otherwise hoisted into phase A)
                }
                if constexpr (!(DBG & 1)) {
                    if (j == 1 && has_next) issue(vp, p.ldv, vstep, t + 1, lds0 + V5 + (PAR ^ 1) * TILE_BYTES);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            stamp_at(3);
            if constexpr (DBG & 32) stamp[7] += 1;
        };
        int i = 0;
        for (; i + 1 < n; i += 2) {
            body(i, std::integral_constant<int, 0>{}, sA, sB);
            body(i + 1, std::integral_constant<int, 1>{}, sB, sA);
        }
        if (i < n) body(i, std::integral_constant<int, 0>{}, sA, sB);
        if (!late) __builtin_amdgcn_s_barrier();  // re-align the groups' barrier counts

        // ---- piece epilogue.  This piece's state first (the next piece's loads go out before its stores).
        // Register order: lane owns query (lane & 31), d = dt*32 + 8 gq + 4 half + 0..3
        const bool e_pub = kt0 > 0;     // not the unit's first tile: publish the partial for the owner
        const bool e_cut = kt1 < nt;    // the unit continues in later workgroups: merge their partials
        const int64_t e_unit_end = unit_end;
        const bool e_active = active;
        // O rows of this wave: a buffer window of its 32 rows (rows >= q1 land out of range and are dropped: no
        // per-lane branch around the stores)
        bf16_t* const e_orow = p.o + (int64_t)(q_start + q0 + wave * 32) * p.ldo + hoff;
        const int eln = opaque(lane);  // the epilogue's lane offsets are computed here, not hoisted
        const int e_ovalid = q0 + wave * 32 + (eln & 31) < q1;
        if (!e_pub && e_cut) {
            // owner of a cut unit: fold in the partials of the logically later workgroups that hold its other
            // tiles (lower blockIdx: SkLayout), the LAST one first: the middle piece of a unit cut three ways (a
            // workgroup whose whole range lies inside the unit) publishes at the end of its range, the tail piece
            // at the start of its range, so merging the tail first leaves the middle piece one more merge of slack
            // (rf_attn_schedule prices it so).  The batch (up to 32 later workgroups, normally 1-2) is found in
            // uniform (scalar) code; a unit running past the group's end is a bad table (device error).
            int cw0 = wg + 1;
            bool done = false;
            while (cw0 < gend) {
                uint32_t mask = 0;
                int cw = cw0;
                for (; cw < gend && cw - cw0 < 32; ++cw) {
                    const int64_t cs = bnds[cw], ce = bnds[cw + 1];
                    if (cs >= e_unit_end) {
                        done = true;
                        break;
                    }
                    if (ce > cs) mask |= 1u << (cw - cw0);
                }
                for (uint32_t m = mask; m;) {
                    const int bit = 31 - __builtin_clz(m);
                    m &= ~(1u << bit);
                    const int f = cw0 + bit;
                    if (tid == 0) {
                        int spins = 0;
                        while (__hip_atomic_load(p.flag + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != p.epoch &&
                               ++spins < p.spin)
                            __builtin_amdgcn_s_sleep(1);
                        if (spins >= p.spin) report_device_error(p.err, RF_DEVERR_SK_ATTN);  // never silent
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    __syncthreads();
                    if (e_active) {
                        // all the partial's loads in flight at once (one round trip), then the fold
                        const float* src = p.part_o + (int64_t)f * PIECE_FLOATS;
                        const f32x2 ml = *reinterpret_cast<const f32x2*>(src + PIECE_O + (wave * 64 + lane) * 2);
                        if constexpr (OF16) {
                            // fp16 partial, normalised by the publisher's row sum: O += 2^(m' - m) l' * O'/l'
                            u32x4 ph[8];
#pragma unroll
                            for (int k = 0; k < 8; ++k)
                                ph[k] = *reinterpret_cast<const u32x4*>(src + (((wave * 8 + k) * 64) + lane) * 4);
                            __builtin_amdgcn_sched_barrier(0);
                            const float mx = __builtin_fmaxf(m_run, ml[0]);
                            const float wa = fast_exp2(m_run - mx), wb = fast_exp2(ml[0] - mx);
                            const float lpub = ml[1] + __shfl_xor(ml[1], 32, 64);  // the publisher's whole-row sum
                            const float wbo = wb * lpub;
                            l_run = l_run * wa + ml[1] * wb;
                            m_run = mx;
#pragma unroll
                            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                                for (int gq = 0; gq < 4; ++gq)
#pragma unroll
                                    for (int e = 0; e < 4; ++e) {
                                        const uint32_t wrd = ph[dt * 2 + (gq >> 1)][(gq & 1) * 2 + (e >> 1)];
                                        const float v = f16_bits_to_f32((uint16_t)(e & 1 ? wrd >> 16 : wrd & 0xffffu));
                                        o[dt][4 * gq + e] = o[dt][4 * gq + e] * wa + v * wbo;
                                    }
                        } else {
                            f32x4 pv[16];
#pragma unroll
                            for (int k = 0; k < 16; ++k)
                                pv[k] = *reinterpret_cast<const f32x4*>(src + (((wave * 16 + k) * 64) + lane) * 4);
                            __builtin_amdgcn_sched_barrier(0);
                            const float mx = __builtin_fmaxf(m_run, ml[0]);
                            const float wa = fast_exp2(m_run - mx), wb = fast_exp2(ml[0] - mx);
                            l_run = l_run * wa + ml[1] * wb;
                            m_run = mx;
#pragma unroll
                            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                                for (int gq = 0; gq < 4; ++gq)
#pragma unroll
                                    for (int e = 0; e < 4; ++e)
                                        o[dt][4 * gq + e] = o[dt][4 * gq + e] * wa + pv[dt * 4 + gq][e] * wb;
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (done) break;
                cw0 = cw;
            }
            if (!done && bnds[gend] < e_unit_end && tid == 0) report_device_error(p.err, RF_DEVERR_SK_SCHED);
        }
        const bool more = it < it_end;
        // the next piece's first loads go out before this piece's stores (after the merge's loads: the owner's
        // merge is normally its range's last piece, and its partial reads want the registers)
        if (more) {
            next_piece();
            issue_qk();                    // the K ring is free: every wave is past this piece's last phase A
            __builtin_amdgcn_s_barrier();  // every wave is past its last phase B: V slot 0 is free
            issue_v0();
        }

        float* piece = p.part_o + (int64_t)wg * PIECE_FLOATS;
        if (e_pub) {
            // publish the unnormalised partial for the owner (sc1 stores; every storing wave drains and one lane
            // flags after the next piece's drain, or after the loop; guide Guideline 16 / MI355X_MICROARCH hand-offs)
            if (e_active) {
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(piece, 0, PIECE_FLOATS * 4, 0x00020000);
                if constexpr (OF16) {
                    // fp16 O / l (the frame's fp16-output launches): half the bytes of the fp32 partial; O / l is a
                    // convex combination of V rows like the output itself, so it fits fp16 where the output does
                    // (checked: a partial beyond fp16's range raises the range word as the output would)
                    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
                    const float inv = l_tot > 0.f ? 1.0f / l_tot : 0.f;
                    float amax = 0.f;
#pragma unroll
                    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                        for (int gq = 0; gq < 4; gq += 2) {
                            u32x4 w4;
#pragma unroll
                            for (int h2 = 0; h2 < 2; ++h2) {
                                const float a = o[dt][4 * (gq + h2)] * inv, b = o[dt][4 * (gq + h2) + 1] * inv;
                                const float c = o[dt][4 * (gq + h2) + 2] * inv, d = o[dt][4 * (gq + h2) + 3] * inv;
                                amax = amax3(amax3(amax, a, b), c, d);
                                w4[2 * h2] = pack_f16x2(a, b);
                                w4[2 * h2 + 1] = pack_f16x2(c, d);
                            }
                            __builtin_amdgcn_raw_buffer_store_b128(w4, rs, (((wave * 8 + dt * 2 + (gq >> 1)) * 64) + eln) * 16,
                                                                   0, 16);
                        }
                    if (e_ovalid && p.range && !f16_in_range(amax)) report_f16_range(p.range, RF_RANGE_ATTN);
                } else {
#pragma unroll
                    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                        for (int gq = 0; gq < 4; ++gq) {
                            const f32x4 v4 = {o[dt][4 * gq], o[dt][4 * gq + 1], o[dt][4 * gq + 2], o[dt][4 * gq + 3]};
                            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v4), rs,
                                                                   (((wave * 16 + dt * 4 + gq) * 64) + eln) * 16, 0, 16);
                        }
                }
                const f32x2 ml = {m_run, l_run};
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, ml), rs,
                                                      PIECE_O * 4 + (wave * 64 + eln) * 8, 0, 16);
            }
            pend = true;  // flag raised in the next piece's first tile, or after the loop
            if (!more) break;
            continue;
        }
        if (e_active) {
            const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
            const float inv = l_tot > 0.f ? 1.0f / l_tot : 0.f;
            // row-per-lane store widened to 16 B (guide T21): column group k = 4 dt + gq is split across the halves
            // (lane l: columns 8k..8k+3, lane l+32: 8k+4..8k+7); one v_permlane32_swap per dword of the pair (k, k+1)
            // gives the lower half columns 8k..8k+7 and the upper half 8k+8..8k+15.  (Staging the tile through LDS
            // for whole-line stores measured slower: 137 vs 129 us per stage-1 launch, the extra registers spill.)
            if constexpr (OF16) {  // fp16 O: |O| <= max |V| row-wise, but V (bf16) may exceed fp16's range
                float amax = 0.f;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                    for (int r = 0; r < 16; r += 2) amax = amax3(amax, o[dt][r] * inv, o[dt][r + 1] * inv);
                if (e_ovalid && p.range && !f16_in_range(amax)) report_f16_range(p.range, RF_RANGE_ATTN);
            }
            const __amdgpu_buffer_rsrc_t ro =
                __builtin_amdgcn_make_buffer_rsrc(e_orow, 0, (int)(32 * p.ldo * 2), 0x00020000);
            // (lanes l and l + 32 hold the same query row: both store or neither)
            const int obase = e_ovalid ? (int)(((eln & 31) * p.ldo + 8 * (eln >> 5)) * 2) : 0x40000000;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int gq = 0; gq < 4; gq += 2) {
                    uint32_t a0 = pack_o<OF16>(o[dt][4 * gq + 0] * inv, o[dt][4 * gq + 1] * inv);
                    uint32_t a1 = pack_o<OF16>(o[dt][4 * gq + 2] * inv, o[dt][4 * gq + 3] * inv);
                    uint32_t b0 = pack_o<OF16>(o[dt][4 * gq + 4] * inv, o[dt][4 * gq + 5] * inv);
                    uint32_t b1 = pack_o<OF16>(o[dt][4 * gq + 6] * inv, o[dt][4 * gq + 7] * inv);
                    const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
                    const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
                    const u32x4 w4 = {r0[0], r1[0], r0[1], r1[1]};
                    __builtin_amdgcn_raw_buffer_store_b128(w4, ro, obase + (dt * 32 + 8 * gq) * 2, 0, 0);
                }
        }
        if (!more) break;
    }
    if (pend) {  // the range ended with a published piece
        attn_wait_vm<0>();
        __syncthreads();
        if (tid == 0) __hip_atomic_store(p.flag + wg, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (DBG & 32) {  // diagnostic: [wg][wave][8] u64 in the last piece slot of the workspace;
        // slots 4 / 5 hold the wave's shader-clock and 100-MHz reference-clock spans (in-kernel clock)
        stamp[4] = __builtin_amdgcn_s_memtime() - clk0;
        stamp[5] = __builtin_amdgcn_s_memrealtime() - ref0;
        if (lane == 0) {
            uint64_t* dbg = reinterpret_cast<uint64_t*>(p.part_o + (int64_t)(SK5_MAX_GRID - 1) * PIECE_FLOATS);
#pragma unroll
            for (int k = 0; k < 8; ++k) dbg[(wg * NW5 + wave) * 8 + k] = stamp[k];
        }
    }
}

#ifdef RF_STUDY  // the one-wave-per-SIMD stream-K kernel (10 % slower than attn_sk_kernel): study build only
// ---------------------------------------------------------------------------------------------
// One-wave-per-SIMD stream-K kernel (attn_p4_kernel): the unit decomposition, partial format and owner merge
// of attn_sk_kernel, but 4 waves per workgroup, each owning 64 query rows (two 32-row sub-blocks qs = 0, 1)
// with the whole register file (O and Q in AGPRs, scores and P in VGPRs): every K / V fragment read from LDS
// feeds two MFMAs (half the LDS reads of the 8-wave kernel), and the softmax is spread at one exp per MFMA gap
// over both phases of a tile:
//   Q(t): S(t+1) = K(t+1) Q^T (32 MFMAs)  ||  exps of tile t, keys 32-63 (b = 1)
//   P(t): O^T += V(t)^T P(t)^T (32 MFMAs) ||  exps of tile t+1, keys 0-31 (b = 0)
// K(t+3) / V(t+1) arrive by LDS-DMA issued one piece every 8 MFMAs of P(t) / Q(t) into 2-deep rings (three
// phases of flight), waited for with counted vmcnt at the phase tops.  Every wave issues every piece (tiles past
// the piece's end re-read row k_len - 1 into a free slot), so the counts are fixed; the QK^T of the tile after
// the piece's last is computed and dropped (one half-tile per piece).
// Running max: exact on the piece's first tile and then FIXED — no O rescale in the loop.  Scores later in the
// piece may exceed it (P > 1): harmless up to the half-row sum threshold 2^60 (fp32 O / l and bf16 P keep
// their relative precision).  Past it (a key far above everything before it) the wave raises a workgroup flag
// with a higher floor for its rows' max, and the workgroup replays the piece from its first tile (rare; each
// replay raises the floor by >= 1 octave, so replays end).
constexpr int NW4 = 4;
constexpr float P4_SUM_THR_LOG2 = 60.0f;

// MFMAs with pinned register files: S chains in VGPRs (read by the softmax VALU), Q and O in AGPRs (only MFMAs
// touch them).  hipcc would otherwise put every accumulator of a 512-register kernel in AGPRs (each score then
// costs a v_accvgpr_read) and spill.  Hazards the compiler no longer sees: VALU reads of S / O after the chains
// are separated by s_nop pads (mfma_drain).
RF_DEV void mfma_qk0(f32x16& d, const bf16x8& k, const bf16x8& q, const f32x16& c) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %3" : "=&v"(d) : "v"(k), "a"(q), "v"(c));
}
RF_DEV void mfma_qk(f32x16& d, const bf16x8& k, const bf16x8& q) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(k), "a"(q));
}
RF_DEV void mfma_pv(f32x16& o, const bf16x8& v, const bf16x8& p) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(o) : "v"(v), "v"(p));
}
RF_DEV void mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }

template <bool UNIT>
__global__ __launch_bounds__(NW4 * 64, 1) void attn_p4_kernel(AttnArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];  // K ring 2 x 16 KiB, V ring 2 x 16 KiB
    __shared__ int s_bad;  // replay request of the current piece

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int half = lane >> 5;
    const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(char, smem);
    if (tid == 0) s_bad = 0;  // ordered before its first read by the first piece's barrier

    const int nwg = gridDim.x, hw = blockIdx.x;
    int gend = 0;
    const int wg = sk_attn_block(p, hw, nwg, gend);
    if (wg < 0) {
        if (tid == 0) report_device_error(p.err, RF_DEVERR_SK_SCHED);
        return;
    }
    int64_t it = p.bounds[wg];
    const int64_t it_end = p.bounds[wg + 1];

    const float c = UNIT ? 1.f : p.c;
    const float inv_c = UNIT ? 1.f : 1.f / p.c;
    const float sum_thr = exp2f(p.thr);
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    // K/V LDS image as attn_sk_kernel (8-row x 32-column subtiles); wave w DMA-fills row groups w and w + 4
    const int d_row = 8 * wave + ((lane >> 2) & 7);
    const int d_ch = 4 * (lane >> 5) + ((lane & 3) ^ ((d_row >> 2) & 3));
    const int kr = lane & 31;
    const int kb_even = 2048 * (kr >> 3) + 64 * (kr & 7) + 16 * (half ^ ((kr >> 2) & 3));
    const int kb_odd = 2048 * (kr >> 3) + 64 * (kr & 7) + 16 * ((2 + half) ^ ((kr >> 2) & 3));
    const int vb_lo = 64 * (4 * (g >> 1) + qq) + 16 * ((2 * (g & 1) + (pp >> 1)) ^ ((g >> 1) & 3)) + 8 * (pp & 1);
    const int vb_hi = 64 * (4 * (g >> 1) + qq) + 16 * ((2 * (g & 1) + (pp >> 1)) ^ ((2 + (g >> 1)) & 3)) + 8 * (pp & 1);

    int pi = -1;
    int64_t base = 0, usz = 0;
    int q_start = 0, q_len = 0, k_start = 0, k_len = 0, v_start = 0, nqb = 1, nt = 1;
    while (it < it_end) {
        while (it >= base + usz) {
            base += usz;
            ++pi;
            const int32_t* d = p.problems + 5 * pi;
            q_start = d[0];
            q_len = d[1];
            k_start = d[2];
            k_len = d[3];
            v_start = d[4];
            nqb = (q_len + QB5 - 1) / QB5;
            nt = (k_len + KT - 1) / KT;
            usz = (int64_t)p.n_heads * nqb * nt;
        }
        const int64_t rel = it - base;
        const int unit = (int)(rel / nt);
        const int kt0 = (int)(rel - (int64_t)unit * nt);
        const int kt1 = (int)min((int64_t)nt, kt0 + (it_end - it));
        const int n = kt1 - kt0;
        const int64_t unit_end = base + (int64_t)(unit + 1) * nt;
        it += n;
        const int h = unit / nqb, qb = unit - (unit / nqb) * nqb;
        const int q0 = (int)((int64_t)qb * q_len / nqb), q1 = (int)((int64_t)(qb + 1) * q_len / nqb);
        const int hoff = h * HD;
        const int r0 = q0 + wave * 64;  // first row of sub-block 0 of this wave
        const bool act0 = r0 < q1, act1 = r0 + 32 < q1;
        // rows past k_len (the tail tile, and tiles past the piece's end: loaded into a free slot, never read)
        // re-read row k_len - 1
        const bf16_t* kb0 = p.k + (int64_t)k_start * p.ldk + hoff + 8 * d_ch;
        const bf16_t* vb0 = p.v + (int64_t)v_start * p.ldv + hoff + 8 * d_ch;
        auto piece = [&](const bf16_t* src, int64_t ld, int t, uint32_t dst, int e) {
            const int rg = e >> 1;
            const uint32_t d0 = __builtin_amdgcn_readfirstlane(dst + (wave + 4 * rg) * 2048 + 1024 * (e & 1));
            const int row = min(t * KT + 32 * rg + d_row, k_len - 1);
            dma_piece(src + (int64_t)row * ld + 64 * (e & 1), d0);
        };
        // the 4 piece sources of tile t, computed at a phase top (off the MFMA gaps: 3 dependent VALU each)
        auto piece_src = [&](const bf16_t* src, int64_t ld, int t, const bf16_t* (&a)[4]) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                a[e] = src + (int64_t)min(t * KT + 32 * (e >> 1) + d_row, k_len - 1) * ld + 64 * (e & 1);
        };
        auto piece_go = [&](const bf16_t* a, uint32_t dst, int e) {
            dma_piece(a, __builtin_amdgcn_readfirstlane(dst + (wave + 4 * (e >> 1)) * 2048 + 1024 * (e & 1)));
        };
        auto issue_all = [&](const bf16_t* src, int64_t ld, int t, uint32_t dst) {
#pragma unroll
            for (int e = 0; e < 4; ++e) piece(src, ld, t, dst, e);
        };
        auto kread = [&](int koff, int j) {  // K fragment j: key block b = j & 1, k-slice st = j >> 1
            const int b = j & 1, st = j >> 1;
            return *reinterpret_cast<const bf16x8*>(smem + koff + (st & 1 ? kb_odd : kb_even) + 8192 * b +
                                                    512 * (st >> 1));
        };
        auto vread = [&](int voff, int j) {  // V^T fragment j: chain dt = j & 3, key block (b, sp) = j >> 2
            const int dt = j & 3, b = (j >> 2) >> 1, sp = (j >> 2) & 1;
            const int imm = voff + 2048 * (4 * b + 2 * sp) + 512 * dt;
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, smem + imm + vb_lo));
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, smem + imm + 2048 + vb_hi));
            return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        };
        auto mask_tail = [&](f32x16 (&sv)[2][2], int t) {  // keys >= k_len of tile t -> -inf
            if ((t + 1) * KT > k_len) {
#pragma unroll
                for (int qs = 0; qs < 2; ++qs)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int key = b * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                            sv[qs][b][r] = t * KT + key >= k_len ? NEG : sv[qs][b][r];
                        }
            }
        };
        auto row_max = [&](const f32x16& s0, const f32x16* s1) {  // max over both lane halves (the whole row)
            float mt = vmax3(s0[0], s0[1], s0[2]);
#pragma unroll
            for (int r = 3; r < 15; r += 2) mt = vmax3(mt, s0[r], s0[r + 1]);
            mt = __builtin_fmaxf(mt, s0[15]);
            if (s1) {
#pragma unroll
                for (int r = 0; r < 16; r += 2) mt = vmax3(mt, (*s1)[r], (*s1)[r + 1]);
            }
            return __builtin_fmaxf(mt, __shfl_xor(mt, 32, 64));
        };
        // exp2 of scores r, r+1 of one 16-score chain into the bf16 P fragment and the row sums
        // software-pipelined form for the MFMA gaps: value v = 0..31 of a half (sub-block v & 1, score v >> 1
        // of its 16-score chain); gap v takes exp(v), the row-sum add of v - 1 and the bf16 pack of the pair
        // (v - 3, v - 1) when v - 3 is the even score of a pair: every dependent VALU is >= 1 MFMA after its input
        auto gap_soft = [&](const f32x16 (&sv)[2][2], int b, bf16x8 (&pq)[2][2][2], float (&ls)[2][4], float (&e)[32],
                            int v) {
            e[v] = fast_exp2(UNIT ? sv[v & 1][b][v >> 1] : sv[v & 1][b][v >> 1] * c);
            if (v >= 1) {
                const int u = v - 1, qs = u & 1, r = u >> 1;
                ls[qs][r & 3] = r < 4 ? e[u] : ls[qs][r & 3] + e[u];
                asm volatile("" : "+v"(ls[qs][r & 3]));
            }
            if (v >= 3 && (((v - 3) >> 1) & 1) == 0) {
                const int u = v - 3, qs = u & 1, r = u >> 1;
                set_pk(pq[qs][b][r >> 3], (r & 7) >> 1, cvt_pk_bf16(e[u], e[u + 2]));
            }
        };
        auto gap_soft_tail = [&](int b, bf16x8 (&pq)[2][2][2], float (&ls)[2][4], float (&e)[32]) {  // after gap 31
            ls[1][3] += e[31];
            asm volatile("" : "+v"(ls[1][3]));
            set_pk(pq[1][b][1], 3, cvt_pk_bf16(e[29], e[31]));
        };
        auto soft = [&](const f32x16& sv, bf16x8 (&pq)[2], float (&ls)[4], int r, int first) {
            float e[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const float v = sv[r + u];
                e[u] = fast_exp2(UNIT ? v : v * c);
                ls[(r + u) & 3] = first ? e[u] : ls[(r + u) & 3] + e[u];
                asm volatile("" : "+v"(ls[(r + u) & 3]));
            }
            set_pk(pq[r >> 3], (r & 7) >> 1, cvt_pk_bf16(e[0], e[1]));
        };

        float m_floor[2] = {-3.0e38f, -3.0e38f};  // log2 units; raised by a replay request
        f32x16 o[2][4];
        float m_run[2], l_run[2];
        for (;;) {  // one attempt at the piece (a replay is rare)
            attn_wait_vm<0>();
            __syncthreads();  // the previous piece's / attempt's LDS readers and stores are done

            bf16x8 qf[2][8];
#pragma unroll
            for (int qs = 0; qs < 2; ++qs) {
                const int qrow = q_start + min(r0 + 32 * qs + kr, q1 - 1);
                const bf16_t* src = p.q + (int64_t)qrow * p.ldq + hoff + 8 * half;
#pragma unroll
                for (int st = 0; st < 8; ++st) qf[qs][st] = *reinterpret_cast<const bf16x8*>(src + 16 * st);
            }
#pragma unroll
            for (int qs = 0; qs < 2; ++qs)
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) o[qs][dt][r] = 0.f;
            f32x16 minit[2];
#pragma unroll
            for (int qs = 0; qs < 2; ++qs)
#pragma unroll
                for (int r = 0; r < 16; ++r) minit[qs][r] = 0.f;

            // ---- prologue: Q, K(t0), K(t0+1), V(t0) in flight; S(t0) raw; the running max; P(t0) keys 0-31
            issue_all(kb0, p.ldk, kt0, lds0 + K5);
            issue_all(kb0, p.ldk, kt0 + 1, lds0 + K5 + TILE_BYTES);
            issue_all(vb0, p.ldv, kt0, lds0 + V5);
            attn_wait_vm<8>();
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);

            f32x16 sA[2][2], sB[2][2];
            bf16x8 pA[2][2][2], pB[2][2][2];
            float lsA[2][4], lsB[2][4];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const bf16x8 kf = kread(K5, j);
                const int b = j & 1, st = j >> 1;
#pragma unroll
                for (int qs = 0; qs < 2; ++qs) {
                    if (st == 0)
                        mfma_qk0(sA[qs][b], kf, qf[qs][st], minit[qs]);
                    else
                        mfma_qk(sA[qs][b], kf, qf[qs][st]);
                }
            }
            mfma_drain();
            mask_tail(sA, kt0);
#pragma unroll
            for (int qs = 0; qs < 2; ++qs) {
                const float mrow = __builtin_fmaxf(row_max(sA[qs][0], &sA[qs][1]) * c, m_floor[qs]);
                m_run[qs] = mrow;
                const float ds = mrow * inv_c;
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int r = 0; r < 16; ++r) sA[qs][b][r] -= ds;
#pragma unroll
                for (int r = 0; r < 16; ++r) minit[qs][r] = -ds;
#pragma unroll
                for (int r = 0; r < 16; r += 2) soft(sA[qs][0], pA[qs][0], lsA[qs], r, r < 4);
                l_run[qs] = (lsA[qs][0] + lsA[qs][1]) + (lsA[qs][2] + lsA[qs][3]);
            }
            __builtin_amdgcn_s_barrier();  // every wave is done reading K(t0): its slot takes K(t0+2)
            issue_all(kb0, p.ldk, kt0 + 2, lds0 + K5);
            __builtin_amdgcn_sched_barrier(0);

            // a replay request: rows whose max grew get a new floor (rounded up to whole octaves, so replays end);
            // returns whether any row of the lane grew (a sum over the threshold with no growth needs no replay)
            auto request_replay = [&](int qs, float mt) {
                const float up = mt * c;
                if (up > 0.f) m_floor[qs] = __builtin_fmaxf(m_floor[qs], m_run[qs] + __builtin_ceilf(up));
                return up > 0.f;
            };
            auto raise_flag = [&]() {
                if (lane == 0) s_bad = 1;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // visible before this wave's next barrier
            };

            // ---- one tile: Q(t) then P(t).  s / pc / lsc: tile t (keys 0-31 already in pc[.][0]); sn / pn / lsn:
            // t+1.  Returns true when the workgroup must replay the piece (flag read one phase after it is set).
            int pend = 0;
            auto body = [&](const int i, auto par_c, f32x16 (&s)[2][2], f32x16 (&sn)[2][2], bf16x8 (&pc)[2][2][2],
                            bf16x8 (&pn)[2][2][2], float (&lsc)[2][4], float (&lsn)[2][4]) -> bool {
                constexpr int PAR = decltype(par_c)::value;
                const int t = kt0 + i;
                const bool has1 = t + 1 < kt1;
                const int koff = K5 + (PAR ^ 1) * TILE_BYTES;  // K(t+1)
                const int voff = V5 + PAR * TILE_BYTES;        // V(t)
                const uint32_t vdst = lds0 + V5 + (PAR ^ 1) * TILE_BYTES;
                const uint32_t kdst = lds0 + K5 + (PAR ^ 1) * TILE_BYTES;
                __builtin_amdgcn_sched_barrier(0);
                // ---- top of Q(t): K(t+1) landed (younger: V(t), K(t+2))
                attn_wait_vm<8>();
                __builtin_amdgcn_s_barrier();  // all waves done with P(t-1): V slot PAR^1 is free
                if (pend) return true;         // (uniform: every wave read the flag after the same barrier)
                __builtin_amdgcn_sched_barrier(0);
                {
                    bf16x8 kf[3];
                    const bf16_t* va[4];
                    piece_src(vb0, p.ldv, t + 1, va);
                    kf[0] = kread(koff, 0);
                    kf[1] = kread(koff, 1);
                    float e[32];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int m = 0; m < 32; ++m) {
                        const int j = m >> 1, qs = m & 1, b = j & 1, st = j >> 1;
                        if (st == 0)
                            mfma_qk0(sn[qs][b], kf[j % 3], qf[qs][st], minit[qs]);
                        else
                            mfma_qk(sn[qs][b], kf[j % 3], qf[qs][st]);
                        __builtin_amdgcn_sched_barrier(0);  // the gap's fillers stay behind its MFMA
                        if (qs == 0 && j + 2 < 16) kf[(j + 2) % 3] = kread(koff, j + 2);
                        gap_soft(s, 1, pc, lsc, e, m);  // exps of tile t, keys 32-63
                        if ((m & 7) == 5) piece_go(va[m >> 3], vdst, m >> 3);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    gap_soft_tail(1, pc, lsc, e);
                    mfma_drain();
                }
                // ---- keys 32-63 of tile t: within the threshold, or a replay request
                float lh[2];
#pragma unroll
                for (int qs = 0; qs < 2; ++qs) lh[qs] = (lsc[qs][0] + lsc[qs][1]) + (lsc[qs][2] + lsc[qs][3]);
                if (__any(lh[0] > sum_thr || lh[1] > sum_thr)) {
                    bool grew = false;
#pragma unroll
                    for (int qs = 0; qs < 2; ++qs) grew |= request_replay(qs, row_max(s[qs][1], nullptr));
                    if (__any(grew)) raise_flag();
                }
                l_run[0] += lh[0];
                l_run[1] += lh[1];
                __builtin_amdgcn_sched_barrier(0);

                // ---- top of P(t): V(t) landed (younger: K(t+2), V(t+1))
                attn_wait_vm<8>();
                __builtin_amdgcn_s_barrier();  // all waves done with Q(t): K slot PAR^1 is free
                pend = __builtin_amdgcn_readfirstlane(s_bad);  // consumed at the next phase top
                __builtin_amdgcn_sched_barrier(0);
                mask_tail(sn, t + 1);
                {
                    bf16x8 vf[3];
                    const bf16_t* ka[4];
                    piece_src(kb0, p.ldk, t + 3, ka);
                    vf[0] = vread(voff, 0);
                    vf[1] = vread(voff, 1);
                    float e[32];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int m = 0; m < 32; ++m) {
                        const int j = m >> 1, qs = m & 1, dt = j & 3, b = (j >> 2) >> 1, sp = (j >> 2) & 1;
                        mfma_pv(o[qs][dt], vf[j % 3], pc[qs][b][sp]);
                        __builtin_amdgcn_sched_barrier(0);
                        if (qs == 0 && j + 2 < 16) vf[(j + 2) % 3] = vread(voff, j + 2);
                        gap_soft(sn, 0, pn, lsn, e, m);  // exps of tile t+1, keys 0-31
                        if ((m & 7) == 5) piece_go(ka[m >> 3], kdst, m >> 3);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    gap_soft_tail(0, pn, lsn, e);
                    mfma_drain();
                }
                if (has1) {
                    // ---- keys 0-31 of tile t+1
#pragma unroll
                    for (int qs = 0; qs < 2; ++qs) lh[qs] = (lsn[qs][0] + lsn[qs][1]) + (lsn[qs][2] + lsn[qs][3]);
                    if (__any(lh[0] > sum_thr || lh[1] > sum_thr)) {
                        bool grew = false;
#pragma unroll
                        for (int qs = 0; qs < 2; ++qs) grew |= request_replay(qs, row_max(sn[qs][0], &sn[qs][1]));
                        if (__any(grew)) raise_flag();
                    }
                    l_run[0] += lh[0];
                    l_run[1] += lh[1];
                }
                __builtin_amdgcn_sched_barrier(0);
                return false;
            };
            bool replay = false;
            int i = 0;
            for (; i + 1 < n; i += 2) {
                if (body(i, std::integral_constant<int, 0>{}, sA, sB, pA, pB, lsA, lsB) ||
                    body(i + 1, std::integral_constant<int, 1>{}, sB, sA, pB, pA, lsB, lsA)) {
                    replay = true;
                    break;
                }
            }
            if (!replay && i < n) replay = body(i, std::integral_constant<int, 0>{}, sA, sB, pA, pB, lsA, lsB);
            if (!replay) {  // a flag raised in the last tile's checks
                __syncthreads();
                replay = pend || __builtin_amdgcn_readfirstlane(s_bad);
            }
            if (!replay) break;
            attn_wait_vm<0>();
            __syncthreads();  // every wave has read the flag
            if (tid == 0) s_bad = 0;  // (ordered before the next reads by the attempt's first barrier)
        }

        // ---- piece epilogue.  Register order: lane owns query (lane & 31) of sub-block qs, d = dt*32 + 8 gq + 4 half
        float* pc_ = p.part_o + (int64_t)wg * PIECE_FLOATS;
        if (kt0 > 0) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(pc_, 0, PIECE_FLOATS * 4, 0x00020000);
#pragma unroll
            for (int qs = 0; qs < 2; ++qs) {
                if (!(qs ? act1 : act0)) continue;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        const f32x4 v4 = {o[qs][dt][4 * gq], o[qs][dt][4 * gq + 1], o[qs][dt][4 * gq + 2], o[qs][dt][4 * gq + 3]};
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v4), rs,
                                                               ((((wave * 2 + qs) * 16 + dt * 4 + gq) * 64) + lane) * 16, 0, 16);
                    }
                const f32x2 ml = {m_run[qs], l_run[qs]};
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, ml), rs,
                                                      PIECE_O * 4 + ((wave * 2 + qs) * 64 + lane) * 8, 0, 16);
            }
            attn_wait_vm<0>();
            __syncthreads();
            if (tid == 0) __hip_atomic_store(p.flag + wg, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            continue;
        }
        if (kt1 < nt) {
            int cw = wg + 1;
            for (; cw < gend; ++cw) {  // later pieces: lower blockIdx (SkLayout)
                const int64_t cs = p.bounds[cw], ce = p.bounds[cw + 1];
                if (cs >= unit_end) break;
                if (ce == cs) continue;
                if (tid == 0) {
                    int spins = 0;
                    while (__hip_atomic_load(p.flag + cw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != p.epoch &&
                           ++spins < p.spin)
                        __builtin_amdgcn_s_sleep(1);
                    if (spins >= p.spin) report_device_error(p.err, RF_DEVERR_SK_ATTN);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __syncthreads();
                const float* src = p.part_o + (int64_t)cw * PIECE_FLOATS;
#pragma unroll
                for (int qs = 0; qs < 2; ++qs) {
                    if (!(qs ? act1 : act0)) continue;
                    const f32x2 ml = *reinterpret_cast<const f32x2*>(src + PIECE_O + ((wave * 2 + qs) * 64 + lane) * 2);
                    const float mx = __builtin_fmaxf(m_run[qs], ml[0]);
                    const float wa = fast_exp2(m_run[qs] - mx), wb = fast_exp2(ml[0] - mx);
                    l_run[qs] = l_run[qs] * wa + ml[1] * wb;
                    m_run[qs] = mx;
#pragma unroll
                    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                        for (int gq = 0; gq < 4; ++gq) {
                            const f32x4 v4 = *reinterpret_cast<const f32x4*>(
                                src + ((((wave * 2 + qs) * 16 + dt * 4 + gq) * 64) + lane) * 4);
#pragma unroll
                            for (int e = 0; e < 4; ++e) o[qs][dt][4 * gq + e] = o[qs][dt][4 * gq + e] * wa + v4[e] * wb;
                        }
                }
            }
            if (cw == gend && p.bounds[gend] < unit_end && tid == 0) report_device_error(p.err, RF_DEVERR_SK_SCHED);
        }
#pragma unroll
        for (int qs = 0; qs < 2; ++qs) {
            if (!(qs ? act1 : act0)) continue;
            const float l_tot = l_run[qs] + __shfl_xor(l_run[qs], 32, 64);
            const int qrow_o = r0 + 32 * qs + kr;
            if (qrow_o < q1) {
                const float inv = l_tot > 0.f ? 1.0f / l_tot : 0.f;
                bf16_t* dst = p.o + (int64_t)(q_start + qrow_o) * p.ldo + hoff;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                    for (int gq = 0; gq < 4; gq += 2) {
                        auto pk = [&](float lo, float hi) { return p.o_f16 ? pack_f16x2(lo, hi) : pack_bf16x2(lo, hi); };
                        uint32_t a0 = pk(o[qs][dt][4 * gq + 0] * inv, o[qs][dt][4 * gq + 1] * inv);
                        uint32_t a1 = pk(o[qs][dt][4 * gq + 2] * inv, o[qs][dt][4 * gq + 3] * inv);
                        uint32_t b0 = pk(o[qs][dt][4 * gq + 4] * inv, o[qs][dt][4 * gq + 5] * inv);
                        uint32_t b1 = pk(o[qs][dt][4 * gq + 6] * inv, o[qs][dt][4 * gq + 7] * inv);
                        const auto w0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
                        const auto w1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
                        *reinterpret_cast<uint4*>(dst + dt * 32 + 8 * gq + 8 * half) = make_uint4(w0[0], w1[0], w0[1], w1[1]);
                    }
            }
        }
    }
}
#endif  // RF_STUDY

#ifdef RF_STUDY
// merge split partials: out = sum_s 2^(m_s - M) O_s / sum_s 2^(m_s - M) l_s   (one wave per (row, head))
__global__ __launch_bounds__(256) void attn_combine_kernel(const float* __restrict__ part_o,
                                                           const float* __restrict__ part_ml, int64_t part_rows,
                                                           int n_split, int n_heads, const int32_t* __restrict__ rows,
                                                           int n_rows, bf16_t* __restrict__ o, int64_t ldo) {
    const int lane = threadIdx.x & 63;
    const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (item >= (int64_t)n_rows * n_heads) return;
    const int h = (int)(item % n_heads);
    const int row = rows ? rows[item / n_heads] : (int)(item / n_heads);
    float mx = NEG;
    for (int s = 0; s < n_split; ++s) mx = fmaxf(mx, part_ml[(((int64_t)s * part_rows + row) * n_heads + h) * 2]);
    float l = 0.f, a0 = 0.f, a1 = 0.f;
    for (int s = 0; s < n_split; ++s) {
        const float* ml = part_ml + (((int64_t)s * part_rows + row) * n_heads + h) * 2;
        const float w = exp2f(ml[0] - mx);
        l += w * ml[1];
        const float* po = part_o + ((int64_t)s * part_rows + row) * (n_heads * HD) + h * HD;
        a0 += w * po[lane];
        a1 += w * po[lane + 64];
    }
    const float inv = l > 0.f ? 1.0f / l : 0.f;
    bf16_t* dst = o + (int64_t)row * ldo + h * HD;
    dst[lane] = f32_to_bf16(a0 * inv);
    dst[lane + 64] = f32_to_bf16(a1 * inv);
}
#endif  // RF_STUDY

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2F = 0.69314718055994530942f;

int cu_count() {  // per-device, queried once
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cache[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cache[dev] = n;
    }
    return cache[dev];
}

struct QNorm {  // rf_attn_fwd_qn's q row scale (AttnArgs::qk_ss ...)
    const float* ss = nullptr;
    int64_t ld = 0;
    int dim = 0;
    float eps = 0.f, scale = 1.f;
};

int attn_sk_launch(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv, void* o,
                   int64_t ldo, const int32_t* problems, int n_problems, int n_heads, float scale, void* workspace,
                   void* stream, const int64_t* bounds = nullptr, int grid = 0, bool o_f16 = false,
                   bool i_f16 = false, const QNorm* qn = nullptr) {
    RF_REQUIRE(workspace, "rf_attn_fwd: stream-K mode needs the workspace (rf_attn_workspace_bytes(0, H, 0))");
    if (!bounds) {
        grid = cu_count();
        if (const char* env = getenv("RF_ATTN_GRID")) grid = atoi(env);  // tests: force many cut units
    }
    RF_REQUIRE(grid >= 1 && grid <= SK5_MAX_GRID, "rf_attn_fwd: grid %d out of range", grid);
    hipStream_t st0 = (hipStream_t)stream;
    AttnArgs a{};
    a.q = (const bf16_t*)q;
    a.k = (const bf16_t*)k;
    a.v = (const bf16_t*)v;
    a.o = (bf16_t*)o;
    a.ldq = ldq;
    a.ldk = ldk;
    a.ldv = ldv;
    a.ldo = ldo;
    a.problems = problems;
    a.n_problems = n_problems;
    a.n_heads = n_heads;
    a.c = scale * LOG2E;
    a.part_o = (float*)workspace;
    a.flag = (int*)(a.part_o + (int64_t)SK5_MAX_GRID * PIECE_FLOATS);
    a.o_f16 = o_f16;
    a.range = o_f16 ? rf::range_word() : nullptr;
    a.ascend = getenv("RF_SK_ASCEND") && atoi(getenv("RF_SK_ASCEND")) == 1;
    a.bounds = bounds;
    if (qn && qn->ss) {
        a.qk_ss = qn->ss;
        a.qk_ld = qn->ld;
        a.qk_dim = qn->dim;
        a.qk_eps = qn->eps;
        a.qk_scale = qn->scale;
    }
    if (!bounds) {  // equal split per XCD group, written on the device ahead of the launch (stream-ordered)
        int64_t* eq = (int64_t*)(a.flag + SK5_MAX_GRID);
        RF_LAUNCH(attn_equal_bounds_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a, grid, eq);
        a.bounds = eq;
    }
    a.thr = getenv("RF_ATTN_THR") ? (float)atof(getenv("RF_ATTN_THR")) : SUM_THR_LOG2;
    a.err = rf::device_error_word();
    a.spin = rf::spin_limit();
    // a fresh flag value per launch: a publisher's flag from an earlier launch (even one that timed out and left
    // a late flag behind) never equals this launch's, so flags need no re-arm and no memset
    a.epoch = rf::next_epoch(a.flag, SK5_MAX_GRID * sizeof(int), st0);
    if (a.epoch == 0) return RF_ERR_LAUNCH;  // the flag area could not be re-zeroed at an epoch wrap
    // (the grid may exceed the CUs: the SkLayout waits only go to earlier-dispatched blocks)
    // q pre-scaled by scale*log2(e) upstream (scale = ln 2): scores are already exp2 exponents
    const bool unit = fabsf(a.c - 1.0f) < 1e-6f;
    const int dbg = getenv("RF_ATTN_DBG") ? atoi(getenv("RF_ATTN_DBG")) : 0;
    const dim3 g(grid), b(NW5 * 64);
    hipStream_t st = (hipStream_t)stream;
    if (i_f16) {  // fp16 q/k/v (rf_attn_fwd_dt): the production kernel only, no diagnostic variants
        if (unit && o_f16)
            RF_LAUNCH((attn_sk_kernel<true, 0, true, true>), g, b, 0, st, a);
        else if (unit)
            RF_LAUNCH((attn_sk_kernel<true, 0, false, true>), g, b, 0, st, a);
        else if (o_f16)
            RF_LAUNCH((attn_sk_kernel<false, 0, true, true>), g, b, 0, st, a);
        else
            RF_LAUNCH((attn_sk_kernel<false, 0, false, true>), g, b, 0, st, a);
        return rf::check_launch("rf_attn_fwd_dt");
    }
    if (getenv("RF_ATTN_P4") && atoi(getenv("RF_ATTN_P4")) == 1) {  // one-wave-per-SIMD kernel
#ifdef RF_STUDY
        a.thr = getenv("RF_ATTN_THR") ? (float)atof(getenv("RF_ATTN_THR")) : P4_SUM_THR_LOG2;
        if (unit)
            RF_LAUNCH((attn_p4_kernel<true>), g, dim3(NW4 * 64), 0, st, a);
        else
            RF_LAUNCH((attn_p4_kernel<false>), g, dim3(NW4 * 64), 0, st, a);
        return rf::check_launch("rf_attn_fwd");
#else
        return rf::study_only("rf_attn_fwd: RF_ATTN_P4=1 (the one-wave-per-SIMD kernel)");
#endif
    }
#ifndef RF_STUDY
    if (unit && dbg) return rf::study_only("rf_attn_fwd: RF_ATTN_DBG (ablation builds)");
#endif
    switch (unit ? dbg : 0) {  // diagnostic variants (garbage results): ablation timing only
#ifdef RF_STUDY
        case 1: RF_LAUNCH((attn_sk_kernel<true, 1>), g, b, 0, st, a); break;
        case 2: RF_LAUNCH((attn_sk_kernel<true, 2>), g, b, 0, st, a); break;
        case 3: RF_LAUNCH((attn_sk_kernel<true, 3>), g, b, 0, st, a); break;
        case 4: RF_LAUNCH((attn_sk_kernel<true, 4>), g, b, 0, st, a); break;
        case 8: RF_LAUNCH((attn_sk_kernel<true, 8>), g, b, 0, st, a); break;
        case 16: RF_LAUNCH((attn_sk_kernel<true, 16>), g, b, 0, st, a); break;
        case 20: RF_LAUNCH((attn_sk_kernel<true, 20>), g, b, 0, st, a); break;
        case 11: RF_LAUNCH((attn_sk_kernel<true, 11>), g, b, 0, st, a); break;
        case 32:  // stamps on the output format asked for (fp16 O: the frame's instantiation)
            if (o_f16) RF_LAUNCH((attn_sk_kernel<true, 32, true>), g, b, 0, st, a);
            else RF_LAUNCH((attn_sk_kernel<true, 32>), g, b, 0, st, a);
            break;
        case 64: RF_LAUNCH((attn_sk_kernel<true, 64>), g, b, 0, st, a); break;
        case 96: RF_LAUNCH((attn_sk_kernel<true, 96>), g, b, 0, st, a); break;
        case 128: RF_LAUNCH((attn_sk_kernel<true, 128>), g, b, 0, st, a); break;
        case 160: RF_LAUNCH((attn_sk_kernel<true, 160>), g, b, 0, st, a); break;
        case 256: RF_LAUNCH((attn_sk_kernel<true, 256>), g, b, 0, st, a); break;
        case 288: RF_LAUNCH((attn_sk_kernel<true, 288>), g, b, 0, st, a); break;
        case 384: RF_LAUNCH((attn_sk_kernel<true, 384>), g, b, 0, st, a); break;
        case 512: RF_LAUNCH((attn_sk_kernel<true, 512>), g, b, 0, st, a); break;
        case 2048:  // the 16x16x32 shape probe (o_f16 as the frame's instantiation)
            if (o_f16) RF_LAUNCH((attn_sk_kernel<true, 2048, true>), g, b, 0, st, a);
            else RF_LAUNCH((attn_sk_kernel<true, 2048>), g, b, 0, st, a);
            break;
        case 2080:  // the probe with the per-segment stamps and the in-kernel clock (DBG & 32)
            if (o_f16) RF_LAUNCH((attn_sk_kernel<true, 2080, true>), g, b, 0, st, a);
            else RF_LAUNCH((attn_sk_kernel<true, 2080>), g, b, 0, st, a);
            break;
        case 1024:  // (correct results: the per-tile C-operand rebuild, A/B against the default)
            if (o_f16) RF_LAUNCH((attn_sk_kernel<true, 1024, true>), g, b, 0, st, a);
            else RF_LAUNCH((attn_sk_kernel<true, 1024>), g, b, 0, st, a);
            break;
#endif
        default:
            if (unit && o_f16)
                RF_LAUNCH((attn_sk_kernel<true, 0, true>), g, b, 0, st, a);
            else if (unit)
                RF_LAUNCH((attn_sk_kernel<true, 0>), g, b, 0, st, a);
            else if (o_f16)
                RF_LAUNCH((attn_sk_kernel<false, 0, true>), g, b, 0, st, a);
            else
                RF_LAUNCH((attn_sk_kernel<false, 0>), g, b, 0, st, a);
    }
    return rf::check_launch("rf_attn_fwd");
}

}  // namespace

extern "C" int rf_attn_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                           void* o, int64_t ldo, const int32_t* problems, int n_problems, int max_q_len, int n_heads,
                           int head_dim, float scale, int n_split, void* workspace, int64_t ws_rows, void* stream) {
    RF_REQUIRE(q && k && v && o && problems, "rf_attn_fwd: null pointer");
    RF_REQUIRE(head_dim == HD, "rf_attn_fwd: head_dim must be 128 (got %d)", head_dim);
    RF_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0, "rf_attn_fwd: strides must be 16-B aligned");
    RF_REQUIRE(n_split >= 0 && n_split <= 16, "rf_attn_fwd: n_split must be 0..16");
    // (n_split == 0: the stream-K workspace only, ws_rows ignored as rf.h says; n_split > 1: the split partials)
    RF_REQUIRE(n_split <= 1 || (workspace && ws_rows > 0), "rf_attn_fwd: split needs a workspace");
    if (n_problems <= 0 || max_q_len <= 0) return RF_OK;
    if (n_split == 0) return attn_sk_launch(q, ldq, k, ldk, v, ldv, o, ldo, problems, n_problems, n_heads, scale,
                                            workspace, stream);
#ifndef RF_STUDY
    return rf::study_only("rf_attn_fwd: n_split >= 1 (the legacy split-KV kernels)");
#else
    const int kv = getenv("RF_ATTN_KERNEL") ? atoi(getenv("RF_ATTN_KERNEL")) : 3;
    const int qrows = kv == 2 ? 128 : 256;  // v2: 128 rows per workgroup; v3 (8 x 32): 256
    const int n_qblk = (max_q_len + qrows - 1) / qrows;
    const int64_t total = (int64_t)n_qblk * n_heads * n_split * n_problems;
    RF_REQUIRE(total < (1ll << 31), "rf_attn_fwd: grid too large");
    AttnArgs a{};
    a.q = (const bf16_t*)q;
    a.k = (const bf16_t*)k;
    a.v = (const bf16_t*)v;
    a.o = (bf16_t*)o;
    a.ldq = ldq;
    a.ldk = ldk;
    a.ldv = ldv;
    a.ldo = ldo;
    a.problems = problems;
    a.c = scale * LOG2E;
    a.window = 8;
    a.n_qblk = n_qblk;
    a.n_heads = n_heads;
    a.n_split = n_split;
    a.n_total = (int)total;
    a.part_rows = ws_rows;
    if (n_split > 1) {
        a.part_o = (float*)workspace;
        a.part_ml = a.part_o + (int64_t)n_split * ws_rows * n_heads * HD;
    }
    if (kv == 3)
        RF_LAUNCH(attn_v3_kernel, dim3((unsigned)total), dim3(NW3 * 64), 0, (hipStream_t)stream, a);
    else if (kv == 28)
        RF_LAUNCH((attn_fwd_kernel<false, 8>), dim3((unsigned)total), dim3(512), 0, (hipStream_t)stream, a);
    else
        RF_LAUNCH((attn_fwd_kernel<false, 4>), dim3((unsigned)total), dim3(256), 0, (hipStream_t)stream, a);
    return rf::check_launch("rf_attn_fwd");
#endif
}

extern "C" int rf_attn_grid(void) { return cu_count(); }

extern "C" int rf_attn_fwd_sched(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                                 void* o, int64_t ldo, const int32_t* problems, int n_problems, int n_heads,
                                 int head_dim, float scale, void* workspace, const int64_t* bounds, int grid,
                                 void* stream) {
    RF_REQUIRE(q && k && v && o && problems && bounds, "rf_attn_fwd_sched: null pointer");
    RF_REQUIRE(head_dim == HD, "rf_attn_fwd_sched: head_dim must be 128 (got %d)", head_dim);
    RF_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0,
               "rf_attn_fwd_sched: strides must be 16-B aligned");
    if (n_problems <= 0) return RF_OK;
    return attn_sk_launch(q, ldq, k, ldk, v, ldv, o, ldo, problems, n_problems, n_heads, scale, workspace, stream,
                          bounds, grid);
}

extern "C" int rf_attn_fwd_sk(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                              void* o, int64_t ldo, int o_dtype, const int32_t* problems, int n_problems, int n_heads,
                              int head_dim, float scale, void* workspace, const int64_t* bounds, int grid,
                              void* stream) {
    RF_REQUIRE(q && k && v && o && problems && workspace, "rf_attn_fwd_sk: null pointer");
    RF_REQUIRE(head_dim == HD, "rf_attn_fwd_sk: head_dim must be 128 (got %d)", head_dim);
    RF_REQUIRE(o_dtype == RF_DT_BF16 || o_dtype == RF_DT_F16, "rf_attn_fwd_sk: o_dtype must be RF_DT_BF16/F16");
    RF_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0, "rf_attn_fwd_sk: strides must be 16-B aligned");
    if (n_problems <= 0) return RF_OK;
    return attn_sk_launch(q, ldq, k, ldk, v, ldv, o, ldo, problems, n_problems, n_heads, scale, workspace, stream,
                          bounds, bounds ? grid : 0, o_dtype == RF_DT_F16);
}

extern "C" int rf_attn_fwd_dt(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                              void* o, int64_t ldo, int qkv_dtype, int o_dtype, const int32_t* problems,
                              int n_problems, int n_heads, int head_dim, float scale, void* workspace,
                              const int64_t* bounds, int grid, void* stream) {
    RF_REQUIRE(q && k && v && o && problems && workspace, "rf_attn_fwd_dt: null pointer");
    RF_REQUIRE(head_dim == HD, "rf_attn_fwd_dt: head_dim must be 128 (got %d)", head_dim);
    RF_REQUIRE(qkv_dtype == RF_DT_BF16 || qkv_dtype == RF_DT_F16, "rf_attn_fwd_dt: qkv_dtype must be RF_DT_BF16/F16");
    RF_REQUIRE(o_dtype == RF_DT_BF16 || o_dtype == RF_DT_F16, "rf_attn_fwd_dt: o_dtype must be RF_DT_BF16/F16");
    RF_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0, "rf_attn_fwd_dt: strides must be 16-B aligned");
    RF_REQUIRE(n_heads >= 1, "rf_attn_fwd_dt: n_heads must be >= 1");
    if (n_problems <= 0) return RF_OK;
    return attn_sk_launch(q, ldq, k, ldk, v, ldv, o, ldo, problems, n_problems, n_heads, scale, workspace, stream,
                          bounds, bounds ? grid : 0, o_dtype == RF_DT_F16, qkv_dtype == RF_DT_F16);
}

extern "C" int rf_attn_fwd_qn(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                              void* o, int64_t ldo, int o_dtype, const float* q_ss, int64_t ld_ss, int q_dim, float eps,
                              float q_scale, const int32_t* problems, int n_problems, int n_heads, int head_dim,
                              void* workspace, const int64_t* bounds, int grid, void* stream) {
    RF_REQUIRE(q && k && v && o && problems && workspace && q_ss, "rf_attn_fwd_qn: null pointer");
    RF_REQUIRE(head_dim == HD, "rf_attn_fwd_qn: head_dim must be 128 (got %d)", head_dim);
    RF_REQUIRE(o_dtype == RF_DT_BF16 || o_dtype == RF_DT_F16, "rf_attn_fwd_qn: o_dtype must be RF_DT_BF16/F16");
    RF_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0, "rf_attn_fwd_qn: strides must be 16-B aligned");
    RF_REQUIRE(((uintptr_t)q_ss & 15) == 0 && ld_ss >= 8 && ld_ss % 4 == 0 && q_dim > 0,
               "rf_attn_fwd_qn: q_ss rows of >= 8 partial sums, 16-B aligned");
    RF_REQUIRE(n_heads >= 1, "rf_attn_fwd_qn: n_heads must be >= 1");
    if (n_problems <= 0) return RF_OK;
    QNorm qn;
    qn.ss = q_ss;
    qn.ld = ld_ss;
    qn.dim = q_dim;
    qn.eps = eps;
    qn.scale = q_scale;
    // q_scale carries softmax_scale * log2(e): the kernel runs on exp2 exponents (scale = ln 2)
    return attn_sk_launch(q, ldq, k, ldk, v, ldv, o, ldo, problems, n_problems, n_heads, LN2F, workspace, stream,
                          bounds, bounds ? grid : 0, o_dtype == RF_DT_F16, false, &qn);
}

extern "C" int64_t rf_attn_workspace_bytes(int64_t rows, int n_heads, int n_split) {
    if (n_split == 0)  // partial slots, flags, the device-built equal range table
        return (int64_t)SK5_MAX_GRID * PIECE_FLOATS * 4 + SK5_MAX_GRID * 4 + (SK5_MAX_GRID + 1) * 8;
    return n_split <= 1 ? 0 : (int64_t)n_split * rows * n_heads * (HD + 2) * (int64_t)sizeof(float);
}

extern "C" int rf_attn_combine(const void* workspace, int64_t ws_rows, int n_split, int n_heads, const int32_t* rows,
                               int n_rows, void* o, int64_t ldo, void* stream) {
    RF_REQUIRE(workspace && o, "rf_attn_combine: null pointer");
    if (n_rows <= 0) return RF_OK;
#ifndef RF_STUDY
    (void)ws_rows, (void)n_split, (void)n_heads, (void)rows, (void)ldo, (void)stream;
    return rf::study_only("rf_attn_combine (the legacy split-KV merge)");
#else
    const float* po = (const float*)workspace;
    const float* pml = po + (int64_t)n_split * ws_rows * n_heads * HD;
    const int64_t items = (int64_t)n_rows * n_heads;
    RF_LAUNCH(attn_combine_kernel, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, (hipStream_t)stream, po,
                       pml, ws_rows, n_split, n_heads, rows, n_rows, (bf16_t*)o, ldo);
    return rf::check_launch("rf_attn_combine");
#endif
}

static int swin_launch(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv, void* o,
                       int64_t ldo, int o_dtype, int n_images, int grid_h, int grid_w, int window, int shift,
                       int n_heads, int head_dim, float scale, bool qkn, const float* qk_ss, const float* qk_w,
                       float eps, float q_scale, void* stream) {
    RF_REQUIRE(q && k && v && o, "rf_swin_attn_fwd: null pointer");
    RF_REQUIRE(head_dim == HD, "rf_swin_attn_fwd: head_dim must be 128");
    RF_REQUIRE(window == 8, "rf_swin_attn_fwd: window must be 8 (64-token tiles)");
    RF_REQUIRE(grid_h % window == 0 && grid_w % window == 0, "rf_swin_attn_fwd: grid %dx%d not divisible by window",
               grid_h, grid_w);
    RF_REQUIRE(shift >= 0 && shift < window, "rf_swin_attn_fwd: bad shift");
    RF_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0, "rf_swin_attn_fwd: strides must be 16-B aligned");
    RF_REQUIRE(!qkn || (qk_w && qk_ss && ((uintptr_t)qk_ss & 15) == 0),
               "rf_swin_attn_fwd_qkn: qk_norm_w and qk_ss (16-B aligned) are required");
    if (n_images <= 0) return RF_OK;
    AttnArgs a{};
    a.q = (const bf16_t*)q;
    a.k = (const bf16_t*)k;
    a.v = (const bf16_t*)v;
    a.o = (bf16_t*)o;
    a.ldq = ldq;
    a.ldk = ldk;
    a.ldv = ldv;
    a.ldo = ldo;
    a.c = scale * LOG2E;
    a.gh = grid_h;
    a.gw = grid_w;
    a.shift = shift;
    a.window = window;
    a.n_split = 1;
    a.qk_ss = qk_ss;
    a.qk_w = qk_w;
    a.qk_eps = eps;
    a.qk_scale = q_scale;
    a.qk_dim = n_heads * HD;
    dim3 grid((grid_h / window) * (grid_w / window), n_heads, n_images);
    RF_REQUIRE(o_dtype == RF_DT_BF16 || o_dtype == RF_DT_F16, "rf_swin_attn_fwd: o_dtype must be RF_DT_BF16/F16");
    a.range = o_dtype == RF_DT_F16 ? rf::range_word() : nullptr;
    if (qkn) {
        if (o_dtype == RF_DT_F16)
            RF_LAUNCH((attn_fwd_kernel<true, 2, true, true>), grid, dim3(128), 0, (hipStream_t)stream, a);
        else
            RF_LAUNCH((attn_fwd_kernel<true, 2, false, true>), grid, dim3(128), 0, (hipStream_t)stream, a);
    } else {
        if (o_dtype == RF_DT_F16)
            RF_LAUNCH((attn_fwd_kernel<true, 2, true>), grid, dim3(128), 0, (hipStream_t)stream, a);
        else
            RF_LAUNCH((attn_fwd_kernel<true, 2>), grid, dim3(128), 0, (hipStream_t)stream, a);
    }
    return rf::check_launch("rf_swin_attn_fwd");
}

extern "C" int rf_swin_attn_fwd_dt(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                                   void* o, int64_t ldo, int o_dtype, int n_images, int grid_h, int grid_w, int window,
                                   int shift, int n_heads, int head_dim, float scale, void* stream) {
    return swin_launch(q, ldq, k, ldk, v, ldv, o, ldo, o_dtype, n_images, grid_h, grid_w, window, shift, n_heads,
                       head_dim, scale, false, nullptr, nullptr, 0.f, 1.f, stream);
}

extern "C" int rf_swin_attn_fwd_qkn(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                                    void* o, int64_t ldo, int o_dtype, int n_images, int grid_h, int grid_w, int window,
                                    int shift, int n_heads, int head_dim, float scale, const float* qk_ss,
                                    const float* qk_norm_w, float eps, float q_scale, void* stream) {
    return swin_launch(q, ldq, k, ldk, v, ldv, o, ldo, o_dtype, n_images, grid_h, grid_w, window, shift, n_heads,
                       head_dim, scale, true, qk_ss, qk_norm_w, eps, q_scale, stream);
}

extern "C" int rf_swin_attn_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                                void* o, int64_t ldo, int n_images, int grid_h, int grid_w, int window, int shift,
                                int n_heads, int head_dim, float scale, void* stream) {
    return rf_swin_attn_fwd_dt(q, ldq, k, ldk, v, ldv, o, ldo, RF_DT_BF16, n_images, grid_h, grid_w, window, shift,
                               n_heads, head_dim, scale, stream);
}
