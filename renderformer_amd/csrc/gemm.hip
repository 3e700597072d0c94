// MFMA GEMM engine for gfx950: every projection of both transformer stages and
// every DPT convolution runs through this one kernel template.
//
//   C[M,N] (epilogue) A[M,K] * W[N,K]^T
//
// * Operands are K-contiguous bf16 (nn.Linear weight layout [out, in]); the A
//   rows are either dense (a + m*lda) or gathered (DPT convolutions: im2col of an
//   NHWC activation plane, one 32-wide K step = one filter tap, out-of-image rows
//   point at a zero row) — no im2col buffer is ever materialised.
// * Operand precision NTERM: 1 = bf16; 3 = fp32-accurate products from bf16 hi/lo splits of
//   both operands, a.b ~= ah.bh + ah.bl + al.bh; 2 = fp16 operands (one MFMA, 11-bit
//   mantissa: the DPT head's default, see dpt.py).
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
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "common.h"

namespace {

constexpr int BK = 32;
constexpr int P_F16 = 2;  // NTERM value of the fp16-operand mode

// E_ROPE (rf_gemm_qk_rope): E_BF16 whose q/k column segments get the attention's q/k norm weight and rotary position
// encoding applied in the epilogue (and per-row partial sums of squares for the norm's 1 / rms, applied downstream)
enum Epi { E_BF16 = RF_EPI_BF16, E_F32 = RF_EPI_F32, E_ADD = RF_EPI_ADD_F32, E_SWIGLU = RF_EPI_SWIGLU, E_CONV = 16,
           E_ROPE = 17 };

// Tile configuration: BM x BN block tile, WGM x WGN waves (each (BM/WGM) x (BN/WGN)), S-deep LDS ring of
// K-steps of KH x 32 (KH = 2: a 64-deep step staged as two 32-deep planes, half the barriers per K).
template <int BM_, int BN_, int WGM_, int WGN_, int STAGES_, int KH_ = 1>
struct Tile {
    static constexpr int BM = BM_, BN = BN_, WGM = WGM_, WGN = WGN_, STAGES = STAGES_, KH = KH_;
    static constexpr int NWAVE = WGM * WGN, THREADS = NWAVE * 64;
    static constexpr int MW = BM / WGM, NWD = BN / WGN, TI = MW / 16, TJ = NWD / 16;
    // 1-KiB LDS-DMA pieces per wave per plane; with fewer A pieces than waves (BM < 16 x waves: the short
    // tiles of the N = 1,024 projections) waves 0..BM/16-1 stage one A piece each and the rest none
    static constexpr int APIECES = BM / 16;
    static constexpr bool ASHARE = APIECES < NWAVE;
    static constexpr int PA = ASHARE ? 1 : BM / 16 / NWAVE, PB = BN / 16 / NWAVE;
    static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
    static_assert(PA >= 1 && PB >= 1 && (ASHARE || PA * NWAVE * 16 == BM) && PB * NWAVE * 16 == BN,
                  "tile/wave mismatch");
    static_assert(TI >= 1 && TJ >= 2 && TJ % 2 == 0, "wave tile too small");
};

struct EngineArgs {
    const bf16_t* a;
    const bf16_t* a_lo;
    int64_t lda;
    const bf16_t* w;
    const bf16_t* w_lo;
    int64_t ldw;
    int m, n, k;
    // gathered A (convolution): NHWC plane [img][hi][wi][cin_pad]
    int hi, wi, cin_pad, ho, wo, kw, stride, pad;
    uint64_t cin_m, kw_m;  // magic multipliers: x / cin_pad == (x * cin_m) >> 32 (x < 2^16), same for kw
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
    int plane_f16;  // output plane is one fp16 plane (p_hi) instead of bf16 hi/lo
    const float* w_fin;
    const float* b_fin;
    float elu_alpha;
    // stream-K: per-CTA partial tiles [grid][BM*BN] f32, then one int flag per CTA
    float* sk_part;
    int* sk_flag;
    int sk_epoch;
    int group_m;  // tile raster: groups of group_m m-tiles, n fastest within a group (host-chosen)
    const int* gate;  // optional device flag: the launch is a no-op unless *gate != 0 (rf_gemm_bf16_if)
    int halo_lg;      // halo-tiled 3x3 convolution: log2 of the tile width in pixels (halo_kernel)
    int* err;         // device error word (rf::device_error_word): stream-K hand-off timeouts
    int spin;         // stream-K hand-off spin bound (polls)
    uint64_t* stamps; // diagnostics (RF_GEMM_STAMPS=1): per-block s_memtime stamps, [grid][16]; normally null
    // MX fp8 operands (rf_gemm_mx8): per-row E8M0 scales of every 32-element K block, [rows][ld_s] bytes
    const uint8_t* sa;
    const uint8_t* sw;
    int ld_sa, ld_sw;
    int persist;  // phased_sk_kernel: whole tiles strided over the grid, next tile's first K-tiles prefetched
    int l2pf;     // phased3 loop: L2 run-ahead distance in K-tiles (0: off; RF_GEMM_L2PF)
    int out_f16;  // E_BF16 / E_SWIGLU: 16-bit output as fp16 instead of bf16 (rf_gemm_f16's RF_EPI_*_F16)
    int* range;   // fp16 outputs (out_f16, fp16 conv planes): the mapped range flag, raised on |x| > 65504
    // Deferred RMSNorm (rf_gemm_add_prenorm / rf_gemm_rownorm, rf.h).  Producer (E_ADD, xg set): besides the
    // fp32 residual, xg = 16-bit(x * g) and, per row, one partial sum of x^2 per BN-column tile into slot n0 / BN
    // of that row's RF_PRENORM_SLOTS floats in ss_out (tile 0 zeroes the unused slots).  Consumer (E_BF16 /
    // E_SWIGLU, rs_part set): every output row scaled by 1 / sqrt(sum of its slots / rs_n + rs_eps) before the
    // bias / SwiGLU, i.e. rmsnorm(x) W^T = (x * g) W^T / rms(x) with the row scale after the dot products.
    bf16_t* xg;
    int64_t ldxg;
    const float* norm_g;
    float* ss_out;
    int xg_f16;
    const float* rs_part;
    float rs_n, rs_eps;
    // E_BF16 with seg_ss (rf_gemm_rownorm's q/k sums for a following full-width q/k RMSNorm): per row and per
    // segment s < seg_n of seg_w output columns, PN_SLOTS partial sums of the squares of the written (rounded)
    // values, seg_ss[row][s][slot], slot = (n0 % seg_w) / BN (the segment's first tile zeroes the unused slots)
    float* seg_ss;
    int seg_w, seg_n;
    // E_ROPE (rf_gemm_qk_rope): the q/k segments' rotary encoding, in the pair-interleaved column order of the
    // permuted projection rows (per head, column 2 m + t holds dimension m + 64 t): angle of pair m of row r =
    // rope_pos[r * rope_ld + m / rope_nf] * rope_freqs[m % rope_nf] for m < 9 rope_nf (else 0); rope_g: the
    // segments' norm weights in the same order (null: no norm, and no sums); segment 0 also times rope_qscale
    const float* rope_pos;
    int64_t rope_ld;
    int rope_div;  // position row of output row r: r / rope_div (the ray tokens of one view share the view's position)
    const float* rope_freqs;
    int rope_nf;
    const float* rope_g;
    float rope_qscale;
};

constexpr int PN_SLOTS = RF_PRENORM_SLOTS;  // partial sums per row (N <= PN_SLOTS x the narrowest BN, 128)

// Deferred-RMSNorm operands of a tile live in an LDS area after the main loop's buffers (PN_AREA bytes), filled by
// LDS-DMA (pn_issue) before the tile's main loop, so the epilogue reads them from LDS: a global load there would
// wait (vmcnt counts in issue order) behind the epilogue's own stores or the next tile's prefetched operands.
//   consumer (E_BF16 / E_SWIGLU, rs_part): the tile's BM rows x PN_SLOTS partial sums (32 B a row);
//   producer (E_ADD, xg): g of the tile's BN columns, then BM x WGN floats of row-sum scratch.
// Every issuing wave has passed its main loop's last operand wait (newer than these loads) before the epilogue,
// whose first barrier then makes the area visible to all waves.

// two f32 -> the kernel's 16-bit output pair (RNE): fp16 when the launch asks for it, else bf16
RF_DEV uint32_t pack16(const EngineArgs& p, float lo, float hi) {
    return p.out_f16 ? pack_f16x2(lo, hi) : pack_bf16x2(lo, hi);
}

// the value of one 16-bit output as written (fp16 when the launch writes fp16, else bf16)
RF_DEV float unpack16(const EngineArgs& p, uint32_t h) {
    return p.out_f16 ? f16_bits_to_f32((uint16_t)h) : __uint_as_float(h << 16);
}

// uniform early exit of a gated launch (every block reads the same flag, so a stream-K grid exits whole)
RF_DEV bool gated_off(const EngineArgs& p) { return p.gate && *p.gate == 0; }

// x / d for 0 <= x < 2^16 and 1 <= d < 2^16 as one 64-bit multiply: m = 2^32 / d + 1 (the error of
// x * m / 2^32 is below x / 2^32 < 1 / d, so the floor is exact); replaces runtime integer divisions
// (~30 scalar instructions each) in the gathered-convolution staging
RF_DEV int udiv_m(int x, uint64_t m) { return (int)(((uint64_t)(uint32_t)x * m) >> 32); }
inline uint64_t udiv_magic(int d) { return (1ull << 32) / (uint64_t)d + 1; }


// Tile raster.  Each XCD runs a contiguous range of tile ids (see the remap in engine_kernel); with
// groups of group_m m-tiles walked n-fastest, that range is a ~group_m x (range/group_m) rectangle of
// the output, so an XCD's L2 serves both the A rows and the W columns it reuses.  The host picks
// group_m ~ sqrt(range * BN / BM) (square in elements: least L2-miss traffic per XCD).
RF_DEV void tile_coords(int tile, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
    const int per_group = group_m * tiles_n;
    const int g = tile / per_group, r = tile - g * per_group;
    const int first = g * group_m;
    const int gm = min(tiles_m - first, group_m);
    tm = first + r % gm;
    tn = r / gm;
}

RF_DEV int lds_off(int row, int ch) { return row * 64 + ((ch ^ ((row >> 1) & 3)) << 4); }


template <int N>
RF_DEV void wait_vm() {
    static_assert(N >= 0 && N <= 24, "unsupported vmcnt");
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if constexpr (N == 11) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
    else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if constexpr (N == 13) asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
    else if constexpr (N == 14) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
    else if constexpr (N == 15) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
    else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if constexpr (N == 17) asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
    else if constexpr (N == 18) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
    else if constexpr (N == 19) asm volatile("s_waitcnt vmcnt(19)" ::: "memory");
    else if constexpr (N == 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if constexpr (N == 21) asm volatile("s_waitcnt vmcnt(21)" ::: "memory");
    else if constexpr (N == 22) asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
    else if constexpr (N == 23) asm volatile("s_waitcnt vmcnt(23)" ::: "memory");
    else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
}

template <class C, int NTERM>
constexpr int stage_bytes() {
    return C::KH * (NTERM == 3 ? 2 : 1) * (C::A_BYTES + C::B_BYTES);
}

// Residual epilogue (x += A W^T): the accumulators START from the fp32 C tile instead of zero, loaded before
// the main loop's first staging so their latency hides under it; the epilogue is then a plain store (no
// read-modify-write round trip per output row at the end: that serialised 8-16 dependent HBM round trips
// per tile, ~10 us of a 256x256 tile's epilogue).  Layout as engine_epilogue: acc[i][j][e] =
// C[rbase + i*16 + (lane & 15)][cbase + j*16 + 4*(lane >> 4) + e]; rows >= M start at zero.
template <int TI, int TJ>
RF_DEV void load_c_acc(const EngineArgs& p, int rbase, int cbase, f32x4 (&acc)[TI][TJ]) {
    const int lane = threadIdx.x & 63;
    const float* c = reinterpret_cast<const float*>(p.c);
#pragma unroll
    for (int i = 0; i < TI; ++i) {
        const int row = rbase + i * 16 + (lane & 15);
        const bool ok = row < p.m;
        const float* src = c + (int64_t)(ok ? row : 0) * p.ldc + cbase + 4 * (lane >> 4);
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            const bool okc = cbase + 4 * (lane >> 4) + j * 16 < p.n;
            const float4 v = okc ? *reinterpret_cast<const float4*>(src + j * 16) : float4{0.f, 0.f, 0.f, 0.f};
            acc[i][j] = ok ? f32x4{v.x, v.y, v.z, v.w} : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
}

// acc = A[m0:m0+BM, kbeg*BK:kend*BK] * W[n0:n0+BN, same]^T for this wave's sub-tile
// (+ the C tile when INITC and this is the tile's first K range: see load_c_acc)
template <class C, int NTERM, bool GATHER, bool INITC = false>
RF_DEV void engine_mainloop(const EngineArgs& p, char* smem, int m0, int n0, int kbeg, int kend,
                            f32x4 (&acc)[C::TI][C::TJ]) {
    constexpr int S = C::STAGES, TI = C::TI, TJ = C::TJ, PA = C::PA, PB = C::PB, KH = C::KH;
    constexpr int PLANE_A = C::A_BYTES, PLANE_B = C::B_BYTES;
    constexpr int STAGE_BYTES = stage_bytes<C, NTERM>();
    constexpr int HALF_BYTES = STAGE_BYTES / KH;                // one 32-deep plane pair of a stage
    constexpr int GPS = KH * (NTERM == 3 ? 2 : 1) * (PA + PB);  // LDS-DMA instructions per thread per stage
    constexpr int GPS_B = KH * (NTERM == 3 ? 2 : 1) * PB;       // ... for a wave that stages no A piece (ASHARE)
    static_assert(KH == 1 || (!GATHER && NTERM != 3), "64-deep steps: plain single-plane operands only");

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave / C::WGN, wn = wave % C::WGN;
    const bool stage_a = !C::ASHARE || __builtin_amdgcn_readfirstlane(wave) < C::APIECES;  // wave-uniform

    // ---- staging geometry: piece pc of this wave covers 16 rows x 64 B; lane -> (row, 16-B chunk)
    int arow[PA], alc[PA], brow[PB], blc[PB];
#pragma unroll
    for (int pc = 0; pc < PA; ++pc) {
        arow[pc] = (wave * PA + pc) * 16 + (lane >> 2);
        alc[pc] = (lane & 3) ^ ((arow[pc] >> 1) & 3);
    }
#pragma unroll
    for (int pc = 0; pc < PB; ++pc) {
        brow[pc] = (wave * PB + pc) * 16 + (lane >> 2);
        blc[pc] = (lane & 3) ^ ((brow[pc] >> 1) & 3);
    }
    int g_img[PA], g_iy[PA], g_ix[PA];
    const bf16_t* a_row[PA];
    const bf16_t* a_row_lo[PA];
#pragma unroll
    for (int pc = 0; pc < PA; ++pc) {
        int m = m0 + arow[pc];
        const bool ok = m < p.m;
        m = ok ? m : p.m - 1;
        g_img[pc] = g_iy[pc] = g_ix[pc] = 0;
        if constexpr (GATHER) {
            const int ox = m % p.wo, t = m / p.wo;
            g_img[pc] = ok ? t / p.ho : -1;
            g_iy[pc] = (t % p.ho) * p.stride - p.pad;
            g_ix[pc] = ox * p.stride - p.pad;
        }
        a_row[pc] = p.a + (int64_t)m * p.lda;
        a_row_lo[pc] = NTERM == 3 ? p.a_lo + (int64_t)m * p.lda : nullptr;
    }

    auto issue = [&](int kt, int buf) {
#pragma unroll
      for (int h = 0; h < KH; ++h) {
        char* st = smem + buf * STAGE_BYTES + h * HALF_BYTES;
        const int k0 = (kt * KH + h) * BK;
        int cb = k0, ky = 0, kx = 0;
        if constexpr (GATHER) {
            const int tap = udiv_m(k0, p.cin_m);
            cb = k0 - tap * p.cin_pad;
            ky = udiv_m(tap, p.kw_m);
            kx = tap - ky * p.kw;
        }
#pragma unroll
        for (int pc = 0; pc < PA; ++pc) {
            if (!stage_a) break;
            const int piece = wave * PA + pc;
            const int kofs = alc[pc] * 8;
            const bf16_t* sa;
            const bf16_t* sa_lo = nullptr;
            if constexpr (GATHER) {
                const int iy = g_iy[pc] + ky, ix = g_ix[pc] + kx;
                const bool ok = g_img[pc] >= 0 && iy >= 0 && iy < p.hi && ix >= 0 && ix < p.wi;
                const int64_t off = (((int64_t)g_img[pc] * p.hi + iy) * p.wi + ix) * p.cin_pad + cb + kofs;
                sa = ok ? p.a + off : p.zero;
                if constexpr (NTERM == 3) sa_lo = ok ? p.a_lo + off : p.zero;
            } else {
                sa = a_row[pc] + k0 + kofs;
                if constexpr (NTERM == 3) sa_lo = a_row_lo[pc] + k0 + kofs;
            }
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, sa), LDS_PTR(void, st + piece * 1024), 16, 0, 0);
            if constexpr (NTERM == 3)
                __builtin_amdgcn_global_load_lds(GLB_PTR(void, sa_lo),
                                                 LDS_PTR(void, st + PLANE_A + PLANE_B + piece * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int pc = 0; pc < PB; ++pc) {
            const int piece = wave * PB + pc;
            const int64_t woff = (int64_t)(n0 + brow[pc]) * p.ldw + k0 + blc[pc] * 8;
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, p.w + woff), LDS_PTR(void, st + PLANE_A + piece * 1024), 16,
                                             0, 0);
            if constexpr (NTERM == 3)
                __builtin_amdgcn_global_load_lds(GLB_PTR(void, p.w_lo + woff),
                                                 LDS_PTR(void, st + 2 * PLANE_A + PLANE_B + piece * 1024), 16, 0, 0);
        }
      }
    };

    if (INITC && kbeg == 0) {
        load_c_acc<TI, TJ>(p, m0 + wm * C::MW, n0 + wn * C::NWD, acc);
    } else {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    const int nk = kend - kbeg;
    const int frag_row = lane & 15, frag_ch = lane >> 4;
    constexpr int TL = NTERM == 3 ? 1 : 0;  // lo-plane fragments present
    struct Frags {
        bf16x8 a[KH][TI], w[KH][TJ], al[TL ? TI : 1], wl[TL ? TJ : 1];
    };
    auto load_frags = [&](int kt, Frags& f) {
#pragma unroll
      for (int h = 0; h < KH; ++h) {
        const char* st = smem + (kt % S) * STAGE_BYTES + h * HALF_BYTES;
#pragma unroll
        for (int i = 0; i < TI; ++i)
            f.a[h][i] = *reinterpret_cast<const bf16x8*>(st + lds_off(wm * C::MW + i * 16 + frag_row, frag_ch));
#pragma unroll
        for (int j = 0; j < TJ; ++j)
            f.w[h][j] = *reinterpret_cast<const bf16x8*>(st + PLANE_A + lds_off(wn * C::NWD + j * 16 + frag_row, frag_ch));
      }
        if constexpr (TL) {
        const char* st = smem + (kt % S) * STAGE_BYTES;
#pragma unroll
            for (int i = 0; i < TI; ++i)
                f.al[i] = *reinterpret_cast<const bf16x8*>(st + PLANE_A + PLANE_B +
                                                           lds_off(wm * C::MW + i * 16 + frag_row, frag_ch));
#pragma unroll
            for (int j = 0; j < TJ; ++j)
                f.wl[j] = *reinterpret_cast<const bf16x8*>(st + 2 * PLANE_A + PLANE_B +
                                                           lds_off(wn * C::NWD + j * 16 + frag_row, frag_ch));
        }
    };
    auto mma = [&](const Frags& f) {
#pragma unroll
      for (int h = 0; h < KH; ++h)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                if constexpr (TL) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.wl[j], f.a[0][i], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.w[0][j], f.al[i], acc[i][j], 0, 0, 0);
                }
                if constexpr (NTERM == P_F16)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, f.w[h][j]),
                                                                       __builtin_bit_cast(f16x8, f.a[h][i]), acc[i][j], 0, 0, 0);
                else
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.w[h][j], f.a[h][i], acc[i][j], 0, 0, 0);
            }
    };
    // wait until this wave's DMA of step t landed, with `younger` later steps issued (and left in flight)
    auto wait_tile = [&](int younger) {
        constexpr int G = GPS;
        constexpr int GB = GPS_B;
        if (stage_a) {
            if (younger >= 4 && 4 * G <= 24) wait_vm<(4 * G <= 24 ? 4 * G : 0)>();
            else if (younger >= 3 && 3 * G <= 24) wait_vm<(3 * G <= 24 ? 3 * G : 0)>();
            else if (younger >= 2 && 2 * G <= 24) wait_vm<(2 * G <= 24 ? 2 * G : 0)>();
            else if (younger >= 1) wait_vm<G>();
            else wait_vm<0>();
        } else {
            if (younger >= 4 && 4 * GB <= 24) wait_vm<(4 * GB <= 24 ? 4 * GB : 0)>();
            else if (younger >= 3 && 3 * GB <= 24) wait_vm<(3 * GB <= 24 ? 3 * GB : 0)>();
            else if (younger >= 2 && 2 * GB <= 24) wait_vm<(2 * GB <= 24 ? 2 * GB : 0)>();
            else if (younger >= 1) wait_vm<GB>();
            else wait_vm<0>();
        }
    };

    // Ring of S stages.  Fragments are register double-buffered: step kt runs the MFMAs of tile kt
    // (fragments read during step kt-1) while the ds_reads of tile kt+1 and the DMA of tile kt+S
    // are in flight.  One barrier per step; before it, every wave's reads of tile kt have completed,
    // so tile kt's stage is free for tile kt+S right after it.
#pragma unroll
    for (int s = 0; s < S; ++s)
        if (s < nk) issue(kbeg + s, s);
    wait_tile(std::min(S, nk) - 1);  // (with 3+ younger tiles this waits for tile 1 as well)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    Frags f0, f1;
    load_frags(0, f0);
    auto step = [&](int kt, Frags& cur, Frags& nxt) {
        // lgkmcnt(0) as the builtin (not inline asm): hipcc's waitcnt pass sees it, knows `cur` is
        // complete and does not put a wait for the `nxt` reads in front of the MFMAs below
        __builtin_amdgcn_s_waitcnt(0xC07F);
        if (kt + 1 < nk) {
            const int y = std::min(S - 2, nk - 2 - kt);
            wait_tile(y < 0 ? 0 : y);
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt + S < nk) issue(kbeg + kt + S, kt % S);
        if (kt + 1 < nk) load_frags(kt + 1, nxt);
        mma(cur);
    };
    for (int kt = 0; kt < nk; kt += 2) {
        step(kt, f0, f1);
        if (kt + 1 < nk) step(kt + 1, f1, f0);
    }
}

// TW2D = 0: the tile's rows are BM consecutive output rows from m0.  TW2D > 0 (convolutions, halo2_kernel):
// the tile is a block TW2D pixels wide of one image (m0 = its top-left pixel, p.wo the image width), each
// wave's MW pixels are MW / TW2D whole rows of it and fragment i covers 16 consecutive pixels of one row.
// FINAL = false compiles out the fused-head path (RF_CONV_FINAL) for blocks that never take it: its silu
// values are loop-invariant across the head's outputs, get hoisted, and double the accumulators' registers.
// LDS accesses of the deferred-RMSNorm area as inline asm, and a barrier that waits for LDS only: hipcc guards a
// ds_read it can see with vmcnt(0) while a builtin LDS-DMA may be in flight (the persistent loop's next-tile
// prefetch), and __syncthreads() waits vmcnt(0) too; either would drain that prefetch and this tile's stores
RF_DEV uint32_t lds_addr(const char* p) { return (uint32_t)(uintptr_t)LDS_PTR(const char, p); }
RF_DEV float lds_ld_f32(const char* p) {
    float v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
    return v;
}
RF_DEV f32x4 lds_ld_f4(const char* p) {
    f32x4 v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
    return v;
}
RF_DEV void lds_st_f32(char* p, float v) { asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory"); }
RF_DEV void lds_sync() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

// E_ROPE's staged positions: [BM][9] floats by 256-B LDS-DMA pieces (one dword a lane), so the area is whole pieces
template <class C>
constexpr int ROPE_POS_BYTES = (C::BM * 9 + 63) / 64 * 256;
template <class C, int EPI>
constexpr int PN_AREA = EPI == E_ADD      ? C::BN * 4 + C::BM * C::WGN * 4
                        : EPI == E_BF16   ? C::BM * PN_SLOTS * 4 + C::BM * C::WGN * 4
                        // E_ROPE: + the q/k norm weights of the tile's columns, the tile rows' positions, the frequencies
                        : EPI == E_ROPE   ? C::BM * PN_SLOTS * 4 + C::BM * C::WGN * 4 + C::BN * 4 + ROPE_POS_BYTES<C> + 64 * 4
                        : EPI == E_SWIGLU ? C::BM * PN_SLOTS * 4
                                          : 0;

// LDS-DMA of tile (m0, n0)'s deferred-RMSNorm operands into `area` (a no-op unless the launch has them)
template <class C, int EPI>
RF_DEV void pn_issue(const EngineArgs& p, char* area, int m0, int n0) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if constexpr (EPI == E_ADD) {
        if (p.xg && wave == 0 && n0 + 4 * lane < p.n && 4 * lane < C::BN)  // 16 B (4 columns of g) a lane
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, p.norm_g + n0 + 4 * lane), LDS_PTR(void, area), 16, 0, 0);
    } else if constexpr (EPI == E_BF16 || EPI == E_SWIGLU || EPI == E_ROPE) {
        if (p.rs_part) {
            static_assert(C::BM % 32 == 0, "1-KiB pieces of 32 rows");
            for (int c = wave; c < C::BM / 32; c += C::NWAVE) {  // piece c: rows 32 c .. 32 c + 31, 2 lanes a row
                const int row = min(m0 + 32 * c + (lane >> 1), p.m - 1);
                __builtin_amdgcn_global_load_lds(GLB_PTR(void, p.rs_part + (int64_t)row * PN_SLOTS + 4 * (lane & 1)),
                                                 LDS_PTR(void, area + c * 1024), 16, 0, 0);
            }
        }
        if constexpr (EPI == E_ROPE) {
            if (n0 / p.seg_w < p.seg_n) {  // a q/k tile: its norm weights, the rows' positions, the frequencies
                char* const gl = area + C::BM * PN_SLOTS * 4 + C::BM * C::WGN * 4;
                char* const pl = gl + C::BN * 4;
                char* const fl = pl + ROPE_POS_BYTES<C>;  // (the last pos piece runs past BM * 9 floats)
                if (wave == 0 && p.rope_g && 4 * lane < C::BN)  // 16 B (4 columns) a lane
                    __builtin_amdgcn_global_load_lds(GLB_PTR(void, p.rope_g + n0 + 4 * lane), LDS_PTR(void, gl), 16, 0, 0);
                if (p.rope_pos) {
                    if (wave == C::NWAVE - 1)
                        __builtin_amdgcn_global_load_lds(GLB_PTR(void, p.rope_freqs + min(lane, p.rope_nf - 1)),
                                                         LDS_PTR(void, fl), 4, 0, 0);
                    // pos[m0 .. m0 + BM)[0..8] as [BM][9] floats, one dword a lane (rows of 9 floats are not 16-B aligned)
                    for (int c = wave; c * 64 < C::BM * 9; c += C::NWAVE) {
                        const int e = c * 64 + lane;
                        const int r = e / 9, col = e - r * 9;
                        const int row = min(m0 + min(r, C::BM - 1), p.m - 1) / p.rope_div;
                        __builtin_amdgcn_global_load_lds(GLB_PTR(void, p.rope_pos + (int64_t)row * p.rope_ld + col),
                                                         LDS_PTR(void, pl + c * 256), 4, 0, 0);
                    }
                }
            }
        }
    }
}

// area: the tile's deferred-RMSNorm LDS area (PN_AREA<C, EPI> bytes, staged by pn_issue; null for kernels without)
template <class C, int EPI, int TW2D = 0, bool FINAL = true>
RF_DEV void engine_epilogue(const EngineArgs& p, int m0, int n0, const f32x4 (&acc)[C::TI][C::TJ],
                            char* area = nullptr) {
    constexpr int TI = C::TI, TJ = C::TJ;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave / C::WGN, wn = wave % C::WGN;
    static_assert(TW2D == 0 || (EPI == E_CONV && TW2D % 16 == 0 && C::MW % TW2D == 0), "2-D conv tile");
    // ------------------------------------------------------------------ epilogue
    // acc[i][j][e] = C[row][col + e], row = m0 + wm*MW + i*16 + (lane & 15),
    //                                  col = n0 + wn*NWD + j*16 + 4*(lane >> 4)
    const int rl = lane & 15, cq = 4 * (lane >> 4);
    const int rbase = m0 + wm * C::MW, cbase = n0 + wn * C::NWD;
    // output row (pixel) of fragment i for this lane
    auto frow = [&](int i) -> int {
        if constexpr (TW2D == 0) return rbase + i * 16 + rl;
        else return m0 + (wm * (C::MW / TW2D) + (i * 16) / TW2D) * p.wo + (i * 16) % TW2D + rl;
    };
    float amax = 0.f;  // fp16 outputs: running max |value| (NaN-propagating) for the range flag
    // deferred RMSNorm consumer: 1 / rms of each row, one thread per row from its slot sums in slot order (unused
    // slots hold +0, so any producer tiling gives its partials' exact sum), kept in slot 0 of the row's LDS entry;
    // the stores below read it per row (no per-lane array across the epilogue: the 256-row tiles are at 256 VGPRs)
    const bool rsc = (EPI == E_SWIGLU || EPI == E_BF16 || EPI == E_ROPE) && p.rs_part && area;
    if constexpr (EPI == E_SWIGLU || EPI == E_BF16 || EPI == E_ROPE) {
        if (rsc) {
            lds_sync();  // the staged rows are visible (their DMA was waited for inside the main loop)
            for (int t = threadIdx.x; t < C::BM; t += C::THREADS) {
                char* q = area + t * (PN_SLOTS * 4);
                const f32x4 a = lds_ld_f4(q), b = lds_ld_f4(q + 16);
                const float sum = ((a[0] + a[1]) + (a[2] + a[3])) + ((b[0] + b[1]) + (b[2] + b[3]));
                lds_st_f32(q, 1.0f / sqrtf(sum / p.rs_n + p.rs_eps));
            }
            lds_sync();
        }
    }
    auto row_scale = [&](int i) -> float {
        return rsc ? lds_ld_f32(area + (wm * C::MW + i * 16 + rl) * (PN_SLOTS * 4)) : 1.f;
    };
    if constexpr (EPI == E_SWIGLU) {
        bf16_t* c = reinterpret_cast<bf16_t*>(p.c);
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const float rsi = row_scale(i);
#pragma unroll
            for (int pair = 0; pair < TJ / 2; ++pair) {
                const int gcol = cbase + pair * 32;  // 32-row interleave group: [w1 x16 | w3 x16]
                const int ocol = (gcol >> 5) * 16 + cq;
                const int row = rbase + i * 16 + rl;
                if (row < p.m) {
                    float o[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float g = acc[i][2 * pair][e] * rsi, u = acc[i][2 * pair + 1][e] * rsi;
                        if (p.bias) {
                            g += p.bias[gcol + cq + e];
                            u += p.bias[gcol + 16 + cq + e];
                        }
                        o[e] = silu(g) * u;
                    }
                    amax = amax3(amax3(amax, o[0], o[1]), o[2], o[3]);
                    *reinterpret_cast<uint2*>(c + (int64_t)row * p.ldc + ocol) =
                        make_uint2(pack16(p, o[0], o[1]), pack16(p, o[2], o[3]));
                }
            }
        }
        if (p.range && !f16_in_range(amax)) report_f16_range(p.range, RF_RANGE_GEMM);
        return;
    } else if constexpr (EPI == E_CONV) {
        if (FINAL && (p.flags & RF_CONV_FINAL)) {
            // SiLU -> 1x1 (cout <= NWD channels, all in the wn == 0 waves) -> ELU -> [10^x - 1].  silu(conv +
            // bias) is recomputed per output feature (n_fin = 3) rather than held in a TI x TJ array: that
            // array doubled the accumulators' registers and made every conv tile with this epilogue spill
            float bsum[TJ][4];  // bias, 0 in padded channels
#pragma unroll
            for (int j = 0; j < TJ; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int col = cbase + j * 16 + cq + e;
                    bsum[j][e] = (p.bias && col < p.cout) ? p.bias[col] : 0.f;
                }
            for (int f = 0; f < p.n_fin; ++f) {
                const float bfin = p.b_fin[f];  // (read before this output's stores, not behind them)
                float wf[TJ][4];
#pragma unroll
                for (int j = 0; j < TJ; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int col = cbase + j * 16 + cq + e;
                        wf[j][e] = col < p.cout ? p.w_fin[f * p.cout + col] : 0.f;
                    }
#pragma unroll
                for (int i = 0; i < TI; ++i) {
                    float s = 0.f;
#pragma unroll
                    for (int j = 0; j < TJ; ++j)
#pragma unroll
                        for (int e = 0; e < 4; ++e) s += silu(acc[i][j][e] + bsum[j][e]) * wf[j][e];
                    s += __shfl_xor(s, 16, 64);
                    s += __shfl_xor(s, 32, 64);
                    const int m = frow(i);
                    if (lane < 16 && wn == 0 && m < p.m) {
                        float y = elu_fast(s + bfin, p.elu_alpha);
                        if (p.flags & RF_CONV_LOG_DECODE) y = pow10m1_fast(y);
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
        const bool border = (p.flags & RF_CONV_BORDER_BIAS) && !kk;
        // Every load of this epilogue is issued before the stores it could wait behind: vmcnt counts loads and
        // stores together in issue order, so a load issued after a fragment's stores (the bias re-read per
        // fragment, since hipcc could not prove it does not alias the output) made each fragment wait for the
        // previous fragment's stores to be acknowledged — 34 of a 256^2 conv's 92 us.  The bias of
        // the plain case is loop-invariant and read once; the per-pixel operands of fragment i + 1 (residuals,
        // border-class bias row) are read before fragment i is stored.
        float* __restrict__ outp = reinterpret_cast<float*>(p.c);
        const float* __restrict__ res1 = p.res1;
        const float* __restrict__ res2 = p.res2;
        const float* __restrict__ bias = p.bias;
        struct PixOp {
            float4 r1[TJ], r2[TJ], b[TJ];
            int64_t pix[TJ];
            int co[TJ];
        };
        float4 bconst[TJ];
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            const int col = cbase + j * 16 + cq;
            bconst[j] = float4{0.f, 0.f, 0.f, 0.f};
            if (bias && !border && !kk && col < nreal) bconst[j] = *reinterpret_cast<const float4*>(bias + col);
        }
        auto fetch = [&](int i, PixOp& o) {
            const int m = frow(i);
            int img = 0, y = 0, x = 0;
            if (kk || border) {
                x = m % p.wo;
                const int t = m / p.wo;
                y = t % p.ho;
                img = t / p.ho;
            }
            // RF_CONV_BORDER_BIAS: bias row 3 ry + rx of the pixel's border class (rf.h)
            const float* brow = bias;
            if (border && brow)
                brow += (3 * (y == 0 ? 0 : y == p.ho - 1 ? 2 : 1) + (x == 0 ? 0 : x == p.wo - 1 ? 2 : 1)) * p.cout;
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int col = cbase + j * 16 + cq;
                int64_t pix = m;
                int co = col;
                if (kk) {
                    const int tap = col / p.cout, dy = tap / kk, dx = tap % kk;
                    co = col - tap * p.cout;
                    pix = ((int64_t)img * p.ho * kk + y * kk + dy) * (p.wo * kk) + x * kk + dx;
                }
                o.pix[j] = pix;
                o.co[j] = co;
                o.r1[j] = float4{0.f, 0.f, 0.f, 0.f};
                o.r2[j] = float4{0.f, 0.f, 0.f, 0.f};
                o.b[j] = bconst[j];
                if (m < p.m && col < nreal) {
                    if (res1) o.r1[j] = *reinterpret_cast<const float4*>(res1 + pix * p.cout + co);
                    if (res2) o.r2[j] = *reinterpret_cast<const float4*>(res2 + pix * p.cout + co);
                    if (brow && (border || kk)) o.b[j] = *reinterpret_cast<const float4*>(brow + co);
                }
            }
        };
        // (4-fragment-wide tiles (TJ = 4) fetch a fragment's operands at its own turn: double-buffered they spill)
        constexpr bool PF = TJ <= 2;
        PixOp ops[PF ? 2 : 1];
        if constexpr (PF) fetch(0, ops[0]);
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            if constexpr (PF) {
                if (i + 1 < TI) fetch(i + 1, ops[(i + 1) & 1]);
            } else {
                fetch(i, ops[0]);
            }
            const PixOp& o = ops[PF ? (i & 1) : 0];
            if (frow(i) >= p.m) continue;
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int col = cbase + j * 16 + cq;
                if (col >= nreal) continue;
                const int64_t pix = o.pix[j];
                const int co = o.co[j];
                const float bb[4] = {o.b[j].x, o.b[j].y, o.b[j].z, o.b[j].w};
                const float rr1[4] = {o.r1[j].x, o.r1[j].y, o.r1[j].z, o.r1[j].w};
                const float rr2[4] = {o.r2[j].x, o.r2[j].y, o.r2[j].z, o.r2[j].w};
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[e] = ((v[e] + bb[e]) + rr1[e]) + rr2[e];
                    if (p.flags & RF_CONV_SILU_OUT) v[e] = silu(v[e]);
                }
                if (outp)
                    *reinterpret_cast<float4*>(outp + pix * p.cout + co) = make_float4(v[0], v[1], v[2], v[3]);
                if (p.p_hi && p.plane_f16) {
                    float a[4] = {v[0], v[1], v[2], v[3]};
                    if (p.flags & RF_CONV_PLANE_SILU) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) a[e] = silu(a[e]);
                    }
                    amax = amax3(amax3(amax, a[0], a[1]), a[2], a[3]);
                    *reinterpret_cast<uint2*>(p.p_hi + pix * p.p_ld + co) = make_uint2(pack_f16x2(a[0], a[1]),
                                                                                       pack_f16x2(a[2], a[3]));
                } else if (p.p_hi) {
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
        if (p.range && !f16_in_range(amax)) report_f16_range(p.range, RF_RANGE_CONV);
        return;
    } else {
        // deferred-RMSNorm producer (E_ADD with p.xg): per-lane partial sums of x^2 of the lane's rows
        const bool pre = EPI == E_ADD && p.xg && area;
        // q/k segment sums of the written values (E_BF16 with seg_ss): this tile's segment, if it is one of them
        // (E_ROPE: of the projection's values before the norm weight and the rotation, in f32)
        const bool qkseg = EPI == E_ROPE && n0 / p.seg_w < p.seg_n;  // tile-uniform (seg_w is a multiple of BN)
        const bool segq = (EPI == E_BF16 || (EPI == E_ROPE && qkseg)) && p.seg_ss && area && n0 / p.seg_w < p.seg_n;
        // row-sum scratch: after g of the tile's columns (producer) / after the staged ss rows (consumer)
        char* const red = area + (EPI == E_ADD ? C::BN * 4 : C::BM * PN_SLOTS * 4);
        if (pre) lds_sync();  // g staged (pn_issue) and visible
        float ssr[TI];
#pragma unroll
        for (int i = 0; i < TI; ++i) ssr[i] = 0.f;
        // E_ROPE: the rotation's operands were staged in LDS before the main loop (pn_issue: a global load here would
        // wait behind the stores of earlier fragments, vmcnt counting both in issue order).  Per lane and column
        // fragment j the 4 columns cq..cq + 3 are rotation pairs m0 = (col % 128) / 2 and m0 + 1: angle = pos[row][pc]
        // * freq (pc, freq per (j, t) here; the position per row in the loop).
        const char* const gl = area + C::BM * PN_SLOTS * 4 + C::BM * C::WGN * 4;
        const float* const pl = reinterpret_cast<const float*>(gl + C::BN * 4);
        float frq[EPI == E_ROPE ? TJ : 1][2];
        int pcol[EPI == E_ROPE ? TJ : 1][2];
        float sscale = 1.f;
        if constexpr (EPI == E_ROPE) {
            if (qkseg) {
                if (!rsc) lds_sync();  // (the staged area is visible: rsc already synchronised)
                sscale = n0 / p.seg_w == 0 ? p.rope_qscale : 1.f;
                const int lim = 9 * p.rope_nf;
                const float* fl = pl + ROPE_POS_BYTES<C> / 4;
#pragma unroll
                for (int j = 0; j < TJ; ++j) {
                    const int col = cbase + j * 16 + cq;
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const int m = ((col & 127) >> 1) + t;
                        const bool on = p.rope_pos && m < lim;
                        const int pc = on ? m / p.rope_nf : 0;
                        frq[j][t] = on ? fl[m - pc * p.rope_nf] : 0.f;
                        pcol[j][t] = pc;
                    }
                }
            }
        }
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const int row = rbase + i * 16 + rl;
            if (row >= p.m) continue;
            const float rsi = row_scale(i);
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int col = cbase + j * 16 + cq;
                if (col >= p.n) continue;  // (a ragged last column tile of the 4-wave engine)
                float v[4] = {acc[i][j][0] * rsi, acc[i][j][1] * rsi, acc[i][j][2] * rsi, acc[i][j][3] * rsi};
                if (p.bias) {
                    const float4 b = *reinterpret_cast<const float4*>(p.bias + col);
                    v[0] += b.x;
                    v[1] += b.y;
                    v[2] += b.z;
                    v[3] += b.w;
                }
                const int64_t o = (int64_t)row * p.ldc + col;
                if constexpr (EPI == E_ROPE) {
                    if (qkseg) {
                        if (segq) ssr[i] += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
                        const f32x4 g = p.rope_g ? *reinterpret_cast<const f32x4*>(gl + (col - n0) * 4)
                                                 : f32x4{1.f, 1.f, 1.f, 1.f};
                        const float z0 = v[0] * g[0], z1 = v[1] * g[1], z2 = v[2] * g[2], z3 = v[3] * g[3];
                        const float* prow = pl + (wm * C::MW + i * 16 + rl) * 9;
                        float s0, c0, s1, c1;
                        __sincosf(prow[pcol[j][0]] * frq[j][0], &s0, &c0);
                        __sincosf(prow[pcol[j][1]] * frq[j][1], &s1, &c1);
                        // rotate_half on the (m, m + 64) pair, stored interleaved (rope.py:106-149)
                        v[0] = (z0 * c0 - z1 * s0) * sscale;
                        v[1] = (z1 * c0 + z0 * s0) * sscale;
                        v[2] = (z2 * c1 - z3 * s1) * sscale;
                        v[3] = (z3 * c1 + z2 * s1) * sscale;
                    }
                    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.c) + o) =
                        make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
                } else if constexpr (EPI == E_BF16) {
                    amax = amax3(amax3(amax, v[0], v[1]), v[2], v[3]);
                    const uint32_t lo = pack16(p, v[0], v[1]), hi = pack16(p, v[2], v[3]);
                    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.c) + o) = make_uint2(lo, hi);
                    if (segq) {  // squares of the rounded values, as a row kernel reading them back would sum
                        const float r0 = unpack16(p, lo & 0xffffu), r1 = unpack16(p, lo >> 16);
                        const float r2 = unpack16(p, hi & 0xffffu), r3 = unpack16(p, hi >> 16);
                        ssr[i] += r0 * r0 + r1 * r1 + r2 * r2 + r3 * r3;
                    }
                } else {  // E_F32, or E_ADD whose accumulators started from the C tile (load_c_acc)
                    *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.c) + o) = make_float4(v[0], v[1], v[2], v[3]);
                    if (pre) {
                        const f32x4 g = lds_ld_f4(area + (col - n0) * 4);
                        const float y0 = v[0] * g[0], y1 = v[1] * g[1], y2 = v[2] * g[2], y3 = v[3] * g[3];
                        amax = amax3(amax3(amax, y0, y1), y2, y3);
                        const uint32_t lo = p.xg_f16 ? pack_f16x2(y0, y1) : pack_bf16x2(y0, y1);
                        const uint32_t hi = p.xg_f16 ? pack_f16x2(y2, y3) : pack_bf16x2(y2, y3);
                        *reinterpret_cast<uint2*>(p.xg + (int64_t)row * p.ldxg + col) = make_uint2(lo, hi);
                        ssr[i] += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
                    }
                }
            }
        }
        if constexpr (EPI == E_BF16)
            if (p.range && !f16_in_range(amax)) report_f16_range(p.range, RF_RANGE_GEMM);
        if constexpr (EPI == E_ADD || EPI == E_BF16 || EPI == E_ROPE) {
            if (pre && p.xg_f16 && p.range && !f16_in_range(amax)) report_f16_range(p.range, RF_RANGE_RMSNORM);
            if (pre || segq) {
                // row sums: the 4 lane groups of a row (lanes l, l ^ 16, l ^ 32, l ^ 48), then the WGN waves of
                // its row band through LDS, in a fixed order (bit-reproducible)
#pragma unroll
                for (int i = 0; i < TI; ++i) {
                    ssr[i] += __shfl_xor(ssr[i], 16, 64);
                    ssr[i] += __shfl_xor(ssr[i], 32, 64);
                }
                if (lane < 16) {
#pragma unroll
                    for (int i = 0; i < TI; ++i) lds_st_f32(red + (wn * C::BM + wm * C::MW + i * 16 + rl) * 4, ssr[i]);
                }
                lds_sync();
                // destination row block and slot: the producer's [row][PN_SLOTS] (slot = column tile), or the
                // segment's [row][seg_n][PN_SLOTS] (slot = column tile inside the segment)
                int slot, nslots, ld;
                float* base;
                if (pre) {
                    slot = n0 / C::BN;
                    nslots = (p.n + C::BN - 1) / C::BN;
                    ld = PN_SLOTS;
                    base = p.ss_out;
                } else {
                    slot = (n0 % p.seg_w) / C::BN;
                    nslots = p.seg_w / C::BN;
                    ld = p.seg_n * PN_SLOTS;
                    base = p.seg_ss + (n0 / p.seg_w) * PN_SLOTS;
                }
                for (int t = threadIdx.x; t < C::BM; t += C::THREADS) {
                    const int row = m0 + t;
                    if (row < p.m) {
                        float s = 0.f;
#pragma unroll
                        for (int w = 0; w < C::WGN; ++w) s += lds_ld_f32(red + (w * C::BM + t) * 4);
                        float* dst = base + (int64_t)row * ld;
                        dst[slot] = s;
                        if (slot == 0)
                            for (int z = nslots; z < PN_SLOTS; ++z) dst[z] = 0.f;
                    }
                }
            }
        }
    }
}



// ---------------------------------------------------------------------------------------------
// 256x256 tile, BK = 64, 8 waves (2 x 4, each 128 x 64): the phased main loop.
//
// One K-tile = 4 phases; a phase = a load section {ds_read this phase's fragments, issue LDS-DMA
// of the next tiles' freed regions, [counted vmcnt], lgkmcnt(0)}, barrier, an MFMA section {16
// MFMAs at raised priority}, barrier.  Waves 4-7 run one barrier behind waves 0-3 (one extra
// barrier before the loop, matched by one after it for waves 0-3), so on every SIMD one wave's
// MFMA section overlaps its partner's load section (ping-pong); every LDS hazard below is closed
// by a wait placed before a barrier that both groups pass before the dependent access.  The wave's 128x64 output is walked in quadrants q0 = (m0, n0), q1 = (m0, n1),
// q2 = (m1, n1), q3 = (m1, n0) (m = 64 rows, n = 32 columns), so the A/B fragments a phase
// needs are read once: q0 reads A(m0) + B(n0), q1 B(n1), q2 A(m1), q3 nothing (B(n0) kept).
// LDS holds two K-tiles, each as four 16-KiB regions: RA0 = A rows {0-63, 128-191} (every wave's
// m0 rows), RA1 = the m1 rows, RB0 = B rows {64 wc + 0..31}, RB1 = {64 wc + 32..63}.  A region
// is re-filled with tile t+2 one phase after its last read of tile t (RA0/RB0 in phase 1, RB1
// in phase 2, RA1 in phase 3), so every DMA has a whole K-tile of MFMA work to land under, and
// one counted vmcnt per K-tile (end of phase 3: all of tile t+1 landed, tile t+2's 8 in flight)
// publishes the next tile.  Image: [k-half][row][64 B], 16-B chunk ^ ((row >> 1) & 3) as in the
// engine above; one 1-KiB LDS-DMA piece = 16 rows x 32 k.
namespace ph {
constexpr int BN = 256, BK2 = 64;
constexpr int REGION = 16384;  // 128 rows x 64 k x 2 B
// BM = 256: regions RA0, RA1, RB0, RB1; BM = 128 (wave tile 64 x 64): RA, RB0, RB1.  BM = 96 / 64 (wave tile
// 48 / 32 x 64; the short tiles of the N = 1,024 projections): the same three regions with a BM-row RA that
// only waves 0..BM/16-1 stage (the others skip it and count fewer LDS-DMA in their waits)
template <int BM>
struct Cfg {
    static constexpr int NREG = BM == 256 ? 4 : 3;
    static constexpr int NA = BM == 256 ? 2 : 1;  // A regions come first
    static constexpr int A_IMG = BM * 128;        // [2 k-halves][BM rows][64 B]
    static constexpr int TILE = A_IMG + 256 * 128;
    static constexpr int LDS = 2 * TILE;
    static constexpr int MI = BM / 32;  // 16-row M fragments per wave
    static constexpr int GLDS = 2 * NREG;  // LDS-DMA per lane per K-tile
    static constexpr int FA = BM == 256 ? 4 : BM / 32;  // A fragments per wave per phase (rows / 16)
    static_assert(BM == 256 || BM == 128 || BM == 96 || BM == 64, "phased tile height");
};
// tile row of region row j (0..127); runs of 16 consecutive j map to 16 consecutive rows
template <int BM>
RF_DEV int region_row(int r, int j) {
    if constexpr (BM == 256) {
        switch (r) {
            case 0: return j < 64 ? j : j + 64;
            case 1: return j < 64 ? j + 64 : j + 128;
            case 2: return (j >> 5) * 64 + (j & 31);
            default: return (j >> 5) * 64 + 32 + (j & 31);
        }
    } else {
        switch (r) {
            case 0: return j;
            case 1: return (j >> 5) * 64 + (j & 31);
            default: return (j >> 5) * 64 + 32 + (j & 31);
        }
    }
}
// LDS byte offset of (row, k-half, 16-B chunk) in an operand image [2][rows][64 B]
template <int ROWS>
RF_DEV int img(int row, int kh, int ch) { return kh * (ROWS * 64) + row * 64 + ((ch ^ ((row >> 1) & 3)) << 4); }
}  // namespace ph

template <int BM, int NTERM, bool GATHER, bool INITC = false>
RF_DEV void phased_mainloop(const EngineArgs& p, char* smem, int m0, int n0, int kbeg, int kend,
                            f32x4 (&acc)[BM / 32][4], bool pre = false) {
    using namespace ph;
    using G = Cfg<BM>;
    constexpr int NREG = G::NREG, NA = G::NA, MI = G::MI;
    static_assert(NTERM == 1 || NTERM == P_F16, "phased loop: single-term operands");
    constexpr int FA = G::FA;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int nk = kend - kbeg;  // K-tiles of this call; local tile t is global K-tile kbeg + t
    // BM < 128: only waves 0..BM/16-1 stage the A region (wave-uniform)
    const bool has_a = BM >= 128 || __builtin_amdgcn_readfirstlane(wave) < BM / 16;

    // ---- DMA geometry: wave w fills region rows 16 w .. 16 w + 15 (both k-halves) of each region
    const int jrow = 16 * wave + (lane >> 2);
    int trow[NREG], grow[NREG];  // this lane's tile row; first tile row of the wave's 16-row piece (wave-uniform)
    const bf16_t* src[NREG];
#pragma unroll
    for (int r = 0; r < NREG; ++r) {
        trow[r] = region_row<BM>(r, jrow);
        grow[r] = region_row<BM>(r, 16 * wave);
    }
    int am[NA], gi[NA], gy[NA], gx[NA];  // A rows (gathered for convolutions)
#pragma unroll
    for (int r = 0; r < NA; ++r) {
        const int m = m0 + trow[r];
        am[r] = m < p.m ? m : p.m - 1;
        src[r] = p.a + (int64_t)am[r] * p.lda;
        gi[r] = gy[r] = gx[r] = 0;
        if constexpr (GATHER) {
            const int ox = am[r] % p.wo, t = am[r] / p.wo;
            gi[r] = m < p.m ? t / p.ho : -1;
            gy[r] = (t % p.ho) * p.stride - p.pad;
            gx[r] = ox * p.stride - p.pad;
        }
    }
#pragma unroll
    for (int r = NA; r < NREG; ++r) src[r] = p.w + (int64_t)(n0 + trow[r]) * p.ldw;
    const int lch = lane & 3;

    // issue region r of K-tile kt into buffer kt & 1 (2 LDS-DMA per lane: the two 32-deep k-halves)
    auto issue = [&](int kt, int r) {
        const bool is_a = r < NA;
        if (is_a && !has_a) return;
        char* base = smem + (kt & 1) * G::TILE + (is_a ? 0 : G::A_IMG);
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
            const int row = trow[r];
            const int ch = lch ^ ((row >> 1) & 3);  // logical chunk that lands at physical chunk lch
            const int k0 = (kbeg + kt) * BK2 + kh * 32;
            const bf16_t* g = src[r] + k0 + ch * 8;
            if constexpr (GATHER) {
                if (is_a) {
                    const int tap = udiv_m(k0, p.cin_m), cb = k0 - tap * p.cin_pad;
                    const int ky = udiv_m(tap, p.kw_m), kx = tap - ky * p.kw;
                    const int iy = gy[r] + ky, ix = gx[r] + kx;
                    const bool ok = gi[r] >= 0 && iy >= 0 && iy < p.hi && ix >= 0 && ix < p.wi;
                    g = ok ? p.a + (((int64_t)gi[r] * p.hi + iy) * p.wi + ix) * p.cin_pad + cb + ch * 8 : p.zero;
                }
            }
            char* dst = base + kh * (is_a ? BM * 64 : 256 * 64) + grow[r] * 64;
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, g), LDS_PTR(void, dst), 16, 0, 0);
        }
    };

    if (INITC && kbeg == 0) {  // residual epilogue: start from the C tile (load_c_acc), issued before any DMA
        load_c_acc<MI, 4>(p, m0 + wr * (BM / 2), n0 + wc * 64, acc);
    } else {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    const int frow = lane & 15, fch = lane >> 4;  // fragment lane geometry (16x16x32: 16 rows x 4 chunks)
    bf16x8 fa[FA][2], fb0[2][2], fb1[2][2];       // A: FA frags (16 FA rows) x 2 k-slices; B(n0), B(n1): 2 x 2
    auto read_a = [&](const char* buf, int mi) {
#pragma unroll
        for (int i = 0; i < FA; ++i)
#pragma unroll
            for (int s = 0; s < 2; ++s)
                fa[i][s] = *reinterpret_cast<const bf16x8*>(buf + img<BM>(wr * (BM / 2) + mi * 64 + i * 16 + frow, s, fch));
    };
    auto read_b = [&](const char* buf, int ni, bf16x8 (&fb)[2][2]) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s)
                fb[j][s] = *reinterpret_cast<const bf16x8*>(buf + G::A_IMG + img<256>(wc * 64 + ni * 32 + j * 16 + frow, s, fch));
    };
    auto mma = [&](int mi, int ni, const bf16x8 (&fb)[2][2]) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < FA; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    f32x4& c = acc[mi * FA + i][ni * 2 + j];
                    if constexpr (NTERM == P_F16)
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fb[j][s]),
                                                                   __builtin_bit_cast(f16x8, fa[i][s]), c, 0, 0, 0);
                    else
                        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][s], fa[i][s], c, 0, 0, 0);
                }
        __builtin_amdgcn_s_setprio(0);
    };
    auto sync_in = [&]() {
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this phase's fragments are in registers (and its
        __builtin_amdgcn_sched_barrier(0);   // LDS reads retired before the barrier: the WAR side of the DMA)
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    auto sync_out = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    // prologue: tile 0 and (BM = 256) all of tile 1 / (BM = 128) tile 1 minus RB1 in flight; wait for tile 0
    constexpr int AHEAD = BM == 256 ? 8 : 4;  // LDS-DMA of tile 1 issued here (and of tile t+2 at a tile's wait)
    // (pre: the caller already issued K-tiles 0 and 1 of this call, in this order - phased_issue01)
    if (!pre) {
#pragma unroll
        for (int r = 0; r < NREG; ++r) issue(0, r);
    }
    if (nk > 1) {
        if (!pre) {
#pragma unroll
            for (int r = 0; r < (BM == 256 ? NREG : 2); ++r) issue(1, r);
        }
        if (has_a) wait_vm<AHEAD>();
        else wait_vm<AHEAD - 2>();  // (BM < 128, no RA: RB0 of tile 1 only)
    } else {
        wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const bool late = __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256;  // waves 4-7: the lagging group
    if (late) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);

    for (int t = 0; t < nk; ++t) {
        const char* buf = smem + (t & 1) * G::TILE;
        const bool pf = t + 2 < nk;
        if constexpr (BM == 256) {
            // phase 0: q0 = (m0, n0)
            read_b(buf, 0, fb0);
            read_a(buf, 0);
            sync_in();
            mma(0, 0, fb0);
            sync_out();
            // phase 1: q1 = (m0, n1); RA0 / RB0 of tile t were last read in phase 0
            read_b(buf, 1, fb1);
            if (pf) {
                issue(t + 2, 0);
                issue(t + 2, 2);
            }
            sync_in();
            mma(0, 1, fb1);
            sync_out();
            // phase 2: q2 = (m1, n1); RB1 free
            read_a(buf, 1);
            if (pf) issue(t + 2, 3);
            sync_in();
            mma(1, 1, fb1);
            sync_out();
            // phase 3: q3 = (m1, n0), no reads; RA1 free; publish tile t+1
            if (pf) {
                issue(t + 2, 1);
                wait_vm<8>();
            } else {
                wait_vm<0>();
            }
            sync_in();
            mma(1, 0, fb0);
            sync_out();
        } else {
            // phase 0: A (all 64 rows) + B(n0); RB1 of tile t-1 (buffer t+1) is free: tile t+1's RB1
            read_b(buf, 0, fb0);
            read_a(buf, 0);
            if (t + 1 < nk) issue(t + 1, 2);
            sync_in();
            mma(0, 0, fb0);
            sync_out();
            // phase 1: B(n1); RA / RB0 free: tile t+2's; publish tile t+1
            read_b(buf, 1, fb1);
            if (pf) {
                issue(t + 2, 0);
                issue(t + 2, 1);
                if (has_a) wait_vm<4>();
                else wait_vm<2>();
            } else {
                wait_vm<0>();
            }
            sync_in();
            mma(0, 1, fb1);
            sync_out();
        }
    }
    if (!late) __builtin_amdgcn_s_barrier();  // re-align the groups' barrier counts
}

// ---------------------------------------------------------------------------------------------
// Three-buffer phased loop for the short tiles (BM = 64 / 96 / 128, BN = 256; regions RA, RB0, RB1 as in
// the two-buffer loop).  Measured on the N = 1,024 projections with cold operands (the frame's case: each
// layer's weights are read once per frame), the two-buffer loop stalls on its DMA: RB1 of tile t+1 is
// issued only half a K-tile before it is read.  Here all of tile t+2 goes into the third buffer in phase 0
// of tile t (that buffer held tile t-1, whose last reads - the lagging waves' phase 1 - are done by then)
// and is waited for in phase 1 of tile t+1: every DMA has 1.5 K-tiles of MFMA work to land under.
// Same stagger (waves 4-7 one section behind), same one counted vmcnt per K-tile.
template <int BM, int NTERM, bool INITC>
RF_DEV void phased3_mainloop(const EngineArgs& p, char* smem, int m0, int n0, int kbeg, int kend,
                             f32x4 (&acc)[BM / 32][4], char* touch_lds = nullptr) {
    using namespace ph;
    using G = Cfg<BM>;
    static_assert(BM <= 128, "three-buffer loop: short tiles");
    constexpr int NREG = 3, FA = G::FA;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int nk = kend - kbeg;
    const bool has_a = BM >= 128 || __builtin_amdgcn_readfirstlane(wave) < BM / 16;
    const int jrow = 16 * wave + (lane >> 2);
    int trow[NREG], grow[NREG];
    const bf16_t* src[NREG];
#pragma unroll
    for (int r = 0; r < NREG; ++r) {
        trow[r] = region_row<BM>(r, jrow);
        grow[r] = region_row<BM>(r, 16 * wave);
    }
    {
        const int m = m0 + trow[0];
        src[0] = p.a + (int64_t)(m < p.m ? m : p.m - 1) * p.lda;
    }
#pragma unroll
    for (int r = 1; r < NREG; ++r) src[r] = p.w + (int64_t)(n0 + trow[r]) * p.ldw;
    const int lch = lane & 3;
    auto issue_tile = [&](int kt) {  // all three regions of K-tile kt into buffer kt % 3
        char* buf = smem + (kt % 3) * G::TILE;
#pragma unroll
        for (int r = 0; r < NREG; ++r) {
            const bool is_a = r == 0;
            if (is_a && !has_a) continue;
            char* base = buf + (is_a ? 0 : G::A_IMG);
#pragma unroll
            for (int kh = 0; kh < 2; ++kh) {
                const int row = trow[r];
                const int ch = lch ^ ((row >> 1) & 3);
                const int k0 = (kbeg + kt) * BK2 + kh * 32;
                char* dst = base + kh * (is_a ? BM * 64 : 256 * 64) + grow[r] * 64;
                __builtin_amdgcn_global_load_lds(GLB_PTR(void, src[r] + k0 + ch * 8), LDS_PTR(void, dst), 16, 0, 0);
            }
        }
    };
    // L2 run-ahead (study build, p.l2pf = P > 0, RF_GEMM_L2PF): after K-tile kt's LDS-DMA every lane issues one 4-B
    // LDS-DMA "touch" of one 128-B line of K-tile kt + P (thread t: A row t, then the 256 W rows; the rest repeat W
    // rows) into a dummy LDS word, so the tile's lines are in L2 when its real DMA issues P K-tiles later.  One more
    // vector-memory op per K-tile per wave: the counted waits below include it.  Measured 29-32 % SLOWER at every
    // P = 1..4 (profiles/r6_gemm_l2_runahead.txt): a 64-row touch costs the CU's address path about what two
    // operand pieces do, and the pieces' intake did not rise; production passes no touch area (l2pf = 0).
    const int l2pf = touch_lds ? p.l2pf : 0;
    const bf16_t* tsrc;
    {
        const int t = threadIdx.x;
        tsrc = t < BM ? p.a + (int64_t)min(m0 + t, p.m - 1) * p.lda
                      : p.w + (int64_t)(n0 + (t - BM) % 256) * p.ldw;
    }
    auto touch = [&](int kt) {
        const int kk = min(kt + l2pf, nk - 1);
        __builtin_amdgcn_global_load_lds(GLB_PTR(void, tsrc + (kbeg + kk) * BK2), LDS_PTR(void, touch_lds), 4, 0, 0);
    };
    if (INITC && kbeg == 0) {
        load_c_acc<BM / 32, 4>(p, m0 + wr * (BM / 2), n0 + wc * 64, acc);
    } else {
#pragma unroll
        for (int i = 0; i < BM / 32; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int frow = lane & 15, fch = lane >> 4;
    bf16x8 fa[FA][2], fb0[2][2], fb1[2][2];
    auto read_a = [&](const char* buf) {
#pragma unroll
        for (int i = 0; i < FA; ++i)
#pragma unroll
            for (int s = 0; s < 2; ++s)
                fa[i][s] = *reinterpret_cast<const bf16x8*>(buf + img<BM>(wr * (BM / 2) + i * 16 + frow, s, fch));
    };
    auto read_b = [&](const char* buf, int ni, bf16x8 (&fb)[2][2]) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s)
                fb[j][s] = *reinterpret_cast<const bf16x8*>(buf + G::A_IMG + img<256>(wc * 64 + ni * 32 + j * 16 + frow, s, fch));
    };
    auto mma = [&](int ni, const bf16x8 (&fb)[2][2]) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < FA; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    f32x4& c = acc[i][ni * 2 + j];
                    if constexpr (NTERM == P_F16)
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fb[j][s]),
                                                                   __builtin_bit_cast(f16x8, fa[i][s]), c, 0, 0, 0);
                    else
                        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][s], fa[i][s], c, 0, 0, 0);
                }
        __builtin_amdgcn_s_setprio(0);
    };
    auto sync_in = [&]() {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    auto sync_out = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // prologue: tiles 0 and 1 in flight, wait for tile 0 (this wave's 6 LDS-DMA per tile, 4 without RA)
    issue_tile(0);
    if (l2pf) touch(0);
    if (nk > 1) {
        issue_tile(1);
        if (l2pf) {
            touch(1);
            if (has_a) wait_vm<8>();
            else wait_vm<6>();
        } else {
            if (has_a) wait_vm<6>();
            else wait_vm<4>();
        }
    } else {
        wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const bool late = __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256;
    if (late) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    for (int t = 0; t < nk; ++t) {
        const char* buf = smem + (t % 3) * G::TILE;
        // phase 0: A + B(n0); tile t+2 into the buffer tile t-1 used
        read_b(buf, 0, fb0);
        read_a(buf);
        if (t + 2 < nk) {
            issue_tile(t + 2);
            if (l2pf) touch(t + 2);
        }
        sync_in();
        mma(0, fb0);
        sync_out();
        // phase 1: B(n1); publish tile t+1 (tile t+2 stays in flight)
        read_b(buf, 1, fb1);
        if (t + 2 < nk) {
            if (l2pf) {
                if (has_a) wait_vm<8>();
                else wait_vm<6>();
            } else {
                if (has_a) wait_vm<6>();
                else wait_vm<4>();
            }
        } else {
            wait_vm<0>();
        }
        sync_in();
        mma(1, fb1);
        sync_out();
    }
    if (!late) __builtin_amdgcn_s_barrier();
}

template <int BM, int EPI, int NTERM = 1>
__global__ __launch_bounds__(512, 1) void phased3_kernel(EngineArgs p) {
    using TE = Tile<BM, 256, 2, 4, 4>;  // the epilogue's view of the block
#ifdef RF_STUDY
    __shared__ __attribute__((aligned(16))) char smem[3 * ph::Cfg<BM>::TILE + PN_AREA<TE, EPI> + 256];
#else
    __shared__ __attribute__((aligned(16))) char smem[3 * ph::Cfg<BM>::TILE + PN_AREA<TE, EPI>];
#endif
    if (gated_off(p)) return;
    const int tiles_m = (p.m + BM - 1) / BM;
    const int nwg = gridDim.x;
    const int hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    int tm, tn;
    tile_coords(wg, tiles_m, p.n / ph::BN, p.group_m, tm, tn);
    f32x4 acc[BM / 32][4];
    char* const area = smem + 3 * ph::Cfg<BM>::TILE;
    pn_issue<TE, EPI>(p, area, tm * BM, tn * ph::BN);
#ifdef RF_STUDY  // the L2 run-ahead study (RF_GEMM_L2PF; profiles/r6_gemm_l2_runahead.txt): study build only
    char* const touch = area + PN_AREA<TE, EPI>;
#else
    char* const touch = nullptr;
#endif
    phased3_mainloop<BM, NTERM, EPI == E_ADD>(p, smem, tm * BM, tn * ph::BN, 0, p.k / ph::BK2, acc, touch);
    engine_epilogue<TE, EPI>(p, tm * BM, tn * ph::BN, acc, area);
}

template <int BM, int EPI, int NTERM, bool GATHER>
__global__ __launch_bounds__(512, 1) void phased_kernel(EngineArgs p) {
    using TE = Tile<BM, 256, 2, 4, 4>;
    __shared__ __attribute__((aligned(16))) char smem[ph::Cfg<BM>::LDS + PN_AREA<TE, EPI>];
    if (gated_off(p)) return;
    const int tiles_m = (p.m + BM - 1) / BM;
    const int nwg = gridDim.x;
    const int hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    int tm, tn;
    tile_coords(wg, tiles_m, p.n / ph::BN, p.group_m, tm, tn);
    f32x4 acc[BM / 32][4];
    char* const area = smem + ph::Cfg<BM>::LDS;
    pn_issue<TE, EPI>(p, area, tm * BM, tn * ph::BN);
    phased_mainloop<BM, NTERM, GATHER, EPI == E_ADD>(p, smem, tm * BM, tn * ph::BN, 0, p.k / ph::BK2, acc);
    engine_epilogue<TE, EPI>(p, tm * BM, tn * ph::BN, acc, area);
}

// K-tiles 0 and 1 of a 256x256 phased tile, issued exactly as phased_mainloop's prologue issues them (same
// regions, rows, swizzle and order), so that a persistent block can start the next tile's operand stream
// before it runs the current tile's epilogue; the next phased_mainloop call then runs with pre = true.
RF_DEV void phased_issue01(const EngineArgs& p, char* smem, int m0, int n0, int nk) {
    using namespace ph;
    using G = Cfg<256>;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int jrow = 16 * wave + (lane >> 2), lch = lane & 3;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
        if (kt == 1 && nk < 2) break;
#pragma unroll
        for (int r = 0; r < G::NREG; ++r) {
            const bool is_a = r < G::NA;
            const int trow = region_row<256>(r, jrow), grow = region_row<256>(r, 16 * wave);
            const bf16_t* src;
            if (is_a) {
                const int m = m0 + trow;
                src = p.a + (int64_t)(m < p.m ? m : p.m - 1) * p.lda;
            } else {
                src = p.w + (int64_t)(n0 + trow) * p.ldw;
            }
            char* base = smem + (kt & 1) * G::TILE + (is_a ? 0 : G::A_IMG);
#pragma unroll
            for (int kh = 0; kh < 2; ++kh) {
                const int ch = lch ^ ((trow >> 1) & 3);
                const bf16_t* g = src + kt * BK2 + kh * 32 + ch * 8;
                char* dst = base + kh * (256 * 64) + grow * 64;
                __builtin_amdgcn_global_load_lds(GLB_PTR(void, g), LDS_PTR(void, dst), 16, 0, 0);
            }
        }
    }
}

// Stream-K over the phased loop: the grid's blocks (<= one per CU, all co-resident) split the
// tiles x K-tiles iteration space evenly; partial tiles go to the workspace in accumulator order
// (sc1 stores), the block holding a tile's first K-tile folds them in and runs the epilogue.
template <int EPI, int NTERM>
__global__ __launch_bounds__(512, 1) void phased_sk_kernel(EngineArgs p) {
    constexpr int TI = 8, TJ = 4, BM = 256, TS = BM * ph::BN;
    using TE = Tile<256, 256, 2, 4, 4>;  // the epilogue's view of the block
    __shared__ __attribute__((aligned(16))) char smem[ph::Cfg<BM>::LDS + PN_AREA<TE, EPI>];
    char* const area = smem + ph::Cfg<BM>::LDS;
    const bool pn = p.xg || p.rs_part;  // deferred-RMSNorm operands staged per tile (pn_issue)
    if (gated_off(p)) return;
    const int tiles_m = (p.m + BM - 1) / BM, tiles_n = p.n / ph::BN;
    const int nwg = gridDim.x;
    const int hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    const int iters = p.k / ph::BK2;
    const int64_t ntiles64 = (int64_t)tiles_m * tiles_n;
    // partial-tile stream-K: ranges in the forward-progress layout (common.h SkLayout): a tile's owner only
    // waits on lower-numbered blocks
    const SkLayout lay(nwg, ntiles64);
    int grp = 0;
    const int L = lay.logical(hw, &grp);
    const int gend = lay.base(grp) + lay.size(grp);
    int64_t it, it_end;
    lay.equal_range(L, grp, ntiles64, iters, it, it_end);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    f32x4 acc[TI][TJ];
    if (p.persist) {
        // whole tiles wg, wg + nwg, ...: before each epilogue the next tile's first two K-tiles go into the
        // (now free) LDS buffers, so its operand stream lands while this tile's results are stored
        const int ntiles = tiles_m * tiles_n;
        bool pre = false;
        for (int tile = wg; tile < ntiles; tile += nwg) {
            int tm, tn;
            tile_coords(tile, tiles_m, tiles_n, p.group_m, tm, tn);
            if (pn) {
                if (tile != wg) lds_sync();  // the previous tile's epilogue is done with the area
                pn_issue<TE, EPI>(p, area, tm * BM, tn * ph::BN);
            }
            phased_mainloop<BM, NTERM, false, EPI == E_ADD>(p, smem, tm * BM, tn * ph::BN, 0, iters, acc, pre);
            pre = tile + nwg < ntiles;
            if (pre) {
                int tm2, tn2;
                tile_coords(tile + nwg, tiles_m, tiles_n, p.group_m, tm2, tn2);
                __syncthreads();  // every wave's last LDS reads of this tile are done (lgkmcnt drained per phase)
                phased_issue01(p, smem, tm2 * BM, tn2 * ph::BN, iters);
            }
            engine_epilogue<TE, EPI>(p, tm * BM, tn * ph::BN, acc, area);
        }
        return;
    }
    uint64_t st[16];
    int ns = 0;
    const bool stamp = p.stamps != nullptr;
    if (stamp) st[ns++] = __builtin_amdgcn_s_memtime();
    while (it < it_end) {
        const int tile = (int)(it / iters), kf = (int)(it % iters);
        const int kl = (int)min((int64_t)iters, kf + (it_end - it));
        int tm, tn;
        tile_coords(tile, tiles_m, tiles_n, p.group_m, tm, tn);
        const int m0 = tm * BM, n0 = tn * ph::BN;
        wait_vm<0>();
        __syncthreads();  // the previous segment's LDS readers are done
        if (pn && kf == 0) pn_issue<TE, EPI>(p, area, m0, n0);  // (only the tile's owner runs its epilogue)
        phased_mainloop<BM, NTERM, false, EPI == E_ADD>(p, smem, m0, n0, kf, kl, acc);
        if (stamp && ns < 14) st[ns++] = __builtin_amdgcn_s_memtime();
        if (kf != 0) {
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(p.sk_part + (int64_t)L * TS, 0, TS * 4, 0x00020000);
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j) {
                    const int off = (((wave * TI + i) * TJ + j) * 64 + lane) * 16;
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, off, 0, 16);
                }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_store(p.sk_flag + L, p.sk_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (kl < iters) {
                const int64_t tile_end = (int64_t)(tile + 1) * iters;
                for (int c = L + 1; c < gend; ++c) {  // the tile's later pieces: lower blockIdx (SkLayout)
                    int64_t cb, ce;
                    lay.equal_range(c, grp, ntiles64, iters, cb, ce);
                    if (cb >= tile_end) break;
                    if (ce == cb) continue;  // empty range: no partial
                    if (threadIdx.x == 0) {
                        int spins = 0;
                        while (__hip_atomic_load(p.sk_flag + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != p.sk_epoch &&
                               ++spins < p.spin)
                            __builtin_amdgcn_s_sleep(1);
                        if (spins >= p.spin) report_device_error(p.err, RF_DEVERR_SK_GEMM);  // never silent
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    __syncthreads();
                    const float4* src = reinterpret_cast<const float4*>(p.sk_part + (int64_t)c * TS) + wave * TI * TJ * 64 + lane;
#pragma unroll
                    for (int i = 0; i < TI; ++i)
#pragma unroll
                        for (int j = 0; j < TJ; ++j) {
                            const float4 v = src[(i * TJ + j) * 64];
                            acc[i][j][0] += v.x;
                            acc[i][j][1] += v.y;
                            acc[i][j][2] += v.z;
                            acc[i][j][3] += v.w;
                        }
                }
            }
            if (stamp && ns < 14) st[ns++] = __builtin_amdgcn_s_memtime();
            engine_epilogue<TE, EPI>(p, m0, n0, acc, area);
        }
        if (stamp && ns < 14) st[ns++] = __builtin_amdgcn_s_memtime();
        it += kl - kf;
    }
    if (stamp && threadIdx.x == 0) {
        for (int i = 0; i < 16; ++i) p.stamps[L * 16 + i] = i < ns ? st[i] : 0;
    }
}

// ---------------------------------------------------------------------------------------------
// The 4-wave engine ("quad"): one wave per SIMD with the whole register file, waves 2 x 2 over a BM x BN =
// 2 WM x 2 WN tile (256 x 256: 128 x 128 outputs, 256 accumulator registers per wave).  This is the shape of the
// vendor library's kernels on the frame's projection shapes (tools/kbench.py vendor, profiles/r4_vendor_study.txt:
// 4-wave MT256x256x64 / MT160x256x64 / MT128x192x64 on 16x16x32 MFMAs, 15-26 % faster than the 8-wave phased
// loop on W13, K/V-all and 8192^3).  A fragment read from LDS feeds WN/16 (A) or WM/16 (B) MFMAs — half the LDS
// bytes per MFMA of the 8-wave 128 x 64 wave tile — and with no partner wave on the SIMD the wave pipelines
// itself: one 64-deep K-tile = two phases, one per 32-deep k-half,
//   A(t): MFMAs of k-half 0 (set 0)  ||  ds_reads of tile t's k-half 1 -> set 1
//   lgkmcnt(0); vmcnt(0) (tile t+1 landed); barrier (every wave is done with buffer t & 1)
//   B(t): MFMAs of k-half 1 (set 1)  ||  ds_reads of tile t+1's k-half 0 -> set 0  ||  LDS-DMA of tile t+2
// with the LDS reads and DMA pieces spread between the MFMAs (sched_group_barrier).  One barrier per K-tile; a
// DMA lands under one K-tile of MFMAs.  The DMA is buffer_load ... lds: one per-lane VGPR offset per operand and
// each piece's row offset in an SGPR (no 64-bit address VALU per piece); rows past M read as zeros.
namespace qd {
template <int WM, int WN>
struct Cfg {
    static constexpr int BM = 2 * WM, BN = 2 * WN, TI = WM / 16, TJ = WN / 16;
    static constexpr int A_IMG = BM * 128, B_IMG = BN * 128, STAGE = A_IMG + B_IMG, LDS = 2 * STAGE;
    static constexpr int NPA = BM / 8, NPB = BN / 8, PPW = (NPA + NPB) / 4;  // 1-KiB DMA pieces per K-tile
    static constexpr int WGM = 2, WGN = 2, MW = WM, NWD = WN;               // engine_epilogue's view
    static constexpr int NWAVE = 4, THREADS = 256;
    static_assert(WM % 16 == 0 && WN % 16 == 0 && BM % 32 == 0 && BN % 32 == 0, "quad tile");
    static_assert(LDS <= 160 * 1024, "quad LDS");
};
constexpr uint32_t RSRC_CFG = 0x00020000;  // buffer descriptor word 3 (raw, as the stream-K partial stores)
}  // namespace qd

// MFMA with the accumulator pinned to AGPRs ("+a"): with 256 accumulator registers per wave hipcc otherwise keeps
// them in VGPRs and uses the AGPRs as spill space (a v_accvgpr copy pair around every MFMA).  Only MFMAs touch
// the accumulators until the epilogue, whose reads follow quad_drain().
template <int NTERM>
RF_DEV void mfma_agpr(f32x4& c, const bf16x8& b, const bf16x8& a) {
    if constexpr (NTERM == P_F16)
        asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
    else
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
}
RF_DEV void quad_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }

template <int WM, int WN, int NTERM, bool INITC>
RF_DEV void quad_mainloop(const EngineArgs& p, char* smem, int m0, int n0, int kbeg, int kend,
                          f32x4 (&acc)[WM / 16][WN / 16], bool pre = false) {
    using G = qd::Cfg<WM, WN>;
    constexpr int TI = G::TI, TJ = G::TJ, PPW = G::PPW, BM = G::BM, BN = G::BN, NPA = G::NPA;
    static_assert(NTERM == 1 || NTERM == P_F16, "quad loop: single-term operands");
    constexpr int NR = TI + TJ, NM = TI * TJ;  // reads and MFMAs per phase: group g = read g + MFMAs
    static_assert(PPW <= NR && NM >= NR, "quad interleave: a read and a DMA piece per MFMA group");  // [NM g / NR, NM (g+1) / NR)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    const int nk = kend - kbeg;
    const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(char, smem);

    if (INITC && kbeg == 0) {  // residual epilogue: start from the C tile
        load_c_acc<TI, TJ>(p, m0 + wr * WM, n0 + wc * WN, acc);
    } else {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // ---- LDS-DMA: piece q = wave + 4 u; q < NPA: A rows 16 (q >> 1) .. + 15, k-half q & 1 (u < NPA / 4 for
    // every wave); else B likewise.  Lane l: row l >> 2 of the piece, logical 16-B chunk (l & 3) ^ key(row).
    const int prow = lane >> 2;
    const int pch = (lane & 3) ^ ((prow >> 1) & 3);
    const int64_t a_bytes = (int64_t)(p.m - m0) * p.lda * 2;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.a + (int64_t)m0 * p.lda), 0, (int)(a_bytes < 0x7fffffff ? a_bytes : 0x7fffffff), qd::RSRC_CFG);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.w + (int64_t)n0 * p.ldw), 0, (int)((int64_t)min(BN, p.n - n0) * p.ldw * 2), qd::RSRC_CFG);
    const int va = (prow * (int)p.lda + pch * 8) * 2, vb = (prow * (int)p.ldw + pch * 8) * 2;
    const int kh_w = wave & 1;  // every piece of this wave is k-half (wave & 1)
    auto piece = [&](int kt, uint32_t stage, int u) {
        const int kb = (kbeg + kt) * 128 + kh_w * 64;  // bytes along K
        if (u < NPA / 4) {
            const int rg = (wave >> 1) + 2 * u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, LDS_PTR(void, (uintptr_t)(stage + kh_w * BM * 64 + rg * 1024)),
                                                     16, va, rg * 16 * (int)p.lda * 2 + kb, 0, 0);
        } else {
            const int rg = (wave >> 1) + 2 * u - NPA / 2;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rw, LDS_PTR(void, (uintptr_t)(stage + G::A_IMG + kh_w * BN * 64 + rg * 1024)), 16, vb,
                rg * 16 * (int)p.ldw * 2 + kb, 0, 0);
        }
    };
    auto issue = [&](int kt, uint32_t stage) {
#pragma unroll
        for (int u = 0; u < PPW; ++u) piece(kt, stage, u);
    };

    // ---- fragments: lane row frow, 16-B chunk fch of a 64-B k-half row (image of ph::img).  Read r of a set:
    // r < TJ: B fragment r, else A fragment r - TJ
    const int frow = lane & 15, fch = lane >> 4;
    const uint32_t sw = (uint32_t)((fch ^ ((frow >> 1) & 3)) << 4);
    const uint32_t a_rd = (uint32_t)((wr * WM + frow) * 64) + sw;
    const uint32_t b_rd = (uint32_t)(G::A_IMG + (wc * WN + frow) * 64) + sw;
    bf16x8 fa[2][TI], fb[2][TJ];
    auto read1 = [&](uint32_t stage, int kh, int s, int r) {
        if (r < TJ)
            fb[s][r] = *LDS_PTR(const bf16x8, (uintptr_t)(stage + b_rd + kh * BN * 64 + r * 1024));
        else
            fa[s][r - TJ] = *LDS_PTR(const bf16x8, (uintptr_t)(stage + a_rd + kh * BM * 64 + (r - TJ) * 1024));
    };
    // one phase: the TI x TJ MFMAs of set s (i-major) in NR groups of MPG; before group g, read g of set s ^ 1
    // (k-half rkh of `rstage`, when rd) and DMA piece g of K-tile dkt into `dstage` (when dma and g < PPW)
    auto phase = [&](int s, bool rd, uint32_t rstage, int rkh, bool dma, int dkt, uint32_t dstage) {
#pragma unroll
        for (int g = 0; g < NR; ++g) {
            if (rd) read1(rstage, rkh, s ^ 1, g);
            if (dma && g < PPW) piece(dkt, dstage, g);
#pragma unroll
            for (int m = NM * g / NR; m < NM * (g + 1) / NR; ++m) mfma_agpr<NTERM>(acc[m / TJ][m % TJ], fb[s][m % TJ], fa[s][m / TJ]);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // the body is branch-free (one register assignment for the whole loop): nk is even (the host guarantees
    // K % 128 == 0 and even stream-K ranges), the last tile's phase B still reads "tile nk" fragments (unused)
    // and its DMA pieces are skipped by a uniform branch around SALU / VMEM work only
    if (!pre) {
        issue(0, lds0);
        issue(1, lds0 + G::STAGE);
    }
    wait_vm<PPW>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < NR; ++r) read1(lds0, 0, 0, r);
    auto body = [&](const int t, auto par_c) {
        constexpr int PAR = decltype(par_c)::value;
        const uint32_t stage = lds0 + PAR * G::STAGE, nstage = lds0 + (PAR ^ 1) * G::STAGE;
        __builtin_amdgcn_sched_barrier(0);
        // phase A: k-half 0 of tile t (set 0) || reads of k-half 1 -> set 1
        __builtin_amdgcn_s_setprio(1);
        phase(0, true, stage, 1, false, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of buffer PAR are done
        wait_vm<0>();                          // this wave's pieces of tile t+1 landed
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        // phase B: k-half 1 of tile t (set 1) || reads of tile t+1's k-half 0 -> set 0 || DMA of tile t+2
        __builtin_amdgcn_s_setprio(1);
        phase(1, true, nstage, 0, t + 2 < nk, t + 2, stage);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    for (int t = 0; t < nk; t += 2) {
        body(t, std::integral_constant<int, 0>{});
        body(t + 1, std::integral_constant<int, 1>{});
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // (the unused reads of the last phase B)
    quad_drain();  // the last MFMAs' results are readable by VALU (epilogue, partial stores)
}

// quad_mainloop with the operands staged through registers instead of LDS-DMA (the library's form, PGR): a
// wave's 1-KiB pieces of K-tile t+3 are buffer_load_dwordx4 into 16 VGPR quads while K-tile t+2's quads are
// ds_write_b128 into the free LDS buffer — ~13 issue cycles per piece against 60-180 for an LDS-DMA piece, which
// one wave per SIMD cannot hide.  Per K-tile:
//   A(t): MFMAs of k-half 0 (set 0) || reads of tile t's k-half 1 -> set 1;  lgkmcnt(0); barrier
//   B(t): MFMAs of k-half 1 (set 1) || reads of tile t+1's k-half 0 -> set 0 || ds_write of tile t+2 into the
//         buffer tile t used || buffer loads of tile t+3
// (tile t+2's ds_writes are ordered before their readers in B(t+1) by A(t+1)'s lgkmcnt(0) + barrier).
template <int WM, int WN, int NTERM, bool INITC>
RF_DEV void quad_mainloop_reg(const EngineArgs& p, char* smem, int m0, int n0, int kbeg, int kend,
                              f32x4 (&acc)[WM / 16][WN / 16]) {
    using G = qd::Cfg<WM, WN>;
    constexpr int TI = G::TI, TJ = G::TJ, PPW = G::PPW, BM = G::BM, BN = G::BN, NPA = G::NPA;
    static_assert(NTERM == 1 || NTERM == P_F16, "quad loop: single-term operands");
    constexpr int NR = TI + TJ, NM = TI * TJ;
    static_assert(PPW <= NR && NM >= NR, "quad interleave: a read and a piece per MFMA group");
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    const int nk = kend - kbeg;
    const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(char, smem);

    if (INITC && kbeg == 0) {
        load_c_acc<TI, TJ>(p, m0 + wr * WM, n0 + wc * WN, acc);
    } else {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // pieces as quad_mainloop's (same LDS image); lane l holds row l >> 2, logical chunk (l & 3) ^ key(row), and
    // writes it at the piece base + 16 l
    const int prow = lane >> 2;
    const int pch = (lane & 3) ^ ((prow >> 1) & 3);
    const int64_t a_bytes = (int64_t)(p.m - m0) * p.lda * 2;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.a + (int64_t)m0 * p.lda), 0, (int)(a_bytes < 0x7fffffff ? a_bytes : 0x7fffffff), qd::RSRC_CFG);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.w + (int64_t)n0 * p.ldw), 0, (int)((int64_t)min(BN, p.n - n0) * p.ldw * 2), qd::RSRC_CFG);
    const int va = (prow * (int)p.lda + pch * 8) * 2, vb = (prow * (int)p.ldw + pch * 8) * 2;
    const int kh_w = wave & 1;
    u32x4 gq[PPW];
    auto gload = [&](int kt, int u) {
        const int kb = (kbeg + kt) * 128 + kh_w * 64;
        if (u < NPA / 4) {
            const int rg = (wave >> 1) + 2 * u;
            gq[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, va, rg * 16 * (int)p.lda * 2 + kb, 0);
        } else {
            const int rg = (wave >> 1) + 2 * u - NPA / 2;
            gq[u] = __builtin_amdgcn_raw_buffer_load_b128(rw, vb, rg * 16 * (int)p.ldw * 2 + kb, 0);
        }
    };
    auto swrite = [&](uint32_t stage, int u) {
        const uint32_t base = u < NPA / 4 ? kh_w * BM * 64 + ((wave >> 1) + 2 * u) * 1024
                                          : G::A_IMG + kh_w * BN * 64 + ((wave >> 1) + 2 * u - NPA / 2) * 1024;
        *LDS_PTR(u32x4, (uintptr_t)(stage + base + lane * 16)) = gq[u];
    };
    const int frow = lane & 15, fch = lane >> 4;
    const uint32_t sw = (uint32_t)((fch ^ ((frow >> 1) & 3)) << 4);
    const uint32_t a_rd = (uint32_t)((wr * WM + frow) * 64) + sw;
    const uint32_t b_rd = (uint32_t)(G::A_IMG + (wc * WN + frow) * 64) + sw;
    bf16x8 fa[2][TI], fb[2][TJ];
    auto read1 = [&](uint32_t stage, int kh, int s, int r) {
        if (r < TJ)
            fb[s][r] = *LDS_PTR(const bf16x8, (uintptr_t)(stage + b_rd + kh * BN * 64 + r * 1024));
        else
            fa[s][r - TJ] = *LDS_PTR(const bf16x8, (uintptr_t)(stage + a_rd + kh * BM * 64 + (r - TJ) * 1024));
    };
    // one phase: MFMA groups of set s; before group g: read g of the other set (rd), and (st) ds_write of piece g
    // into wstage then the buffer load of K-tile lkt's piece g (ld)
    auto phase = [&](int s, uint32_t rstage, int rkh, bool st, uint32_t wstage, bool ld, int lkt) {
#pragma unroll
        for (int g = 0; g < NR; ++g) {
            read1(rstage, rkh, s ^ 1, g);
            if (g < PPW) {
                if (st) swrite(wstage, g);
                if (ld) gload(lkt, g);
            }
#pragma unroll
            for (int m = NM * g / NR; m < NM * (g + 1) / NR; ++m) mfma_agpr<NTERM>(acc[m / TJ][m % TJ], fb[s][m % TJ], fa[s][m / TJ]);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // prologue: K-tiles 0 and 1 into the two buffers, K-tile 2 in registers
#pragma unroll
    for (int u = 0; u < PPW; ++u) gload(0, u);
#pragma unroll
    for (int u = 0; u < PPW; ++u) swrite(lds0, u);
#pragma unroll
    for (int u = 0; u < PPW; ++u) gload(1, u);
#pragma unroll
    for (int u = 0; u < PPW; ++u) swrite(lds0 + G::STAGE, u);
    if (nk > 2) {
#pragma unroll
        for (int u = 0; u < PPW; ++u) gload(2, u);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's ds_writes are done
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < NR; ++r) read1(lds0, 0, 0, r);
    auto body = [&](const int t, auto par_c) {
        constexpr int PAR = decltype(par_c)::value;
        const uint32_t stage = lds0 + PAR * G::STAGE, nstage = lds0 + (PAR ^ 1) * G::STAGE;
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        phase(0, stage, 1, false, 0, false, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's reads of buffer PAR (and B(t-1)'s ds_writes) are done
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        phase(1, nstage, 0, t + 2 < nk, stage, t + 3 < nk, t + 3);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    for (int t = 0; t < nk; t += 2) {
        body(t, std::integral_constant<int, 0>{});
        body(t + 1, std::integral_constant<int, 1>{});
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    quad_drain();
}

// K-tiles 0 and 1 of a quad tile, issued as quad_mainloop's prologue issues them (a persistent block starts the
// next tile's operand stream before the current tile's epilogue; the next mainloop call then runs with pre = true)
template <int WM, int WN>
RF_DEV void quad_issue01(const EngineArgs& p, char* smem, int m0, int n0, int nk) {
    using G = qd::Cfg<WM, WN>;
    constexpr int PPW = G::PPW, BM = G::BM, BN = G::BN, NPA = G::NPA;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(char, smem);
    const int prow = lane >> 2, pch = (lane & 3) ^ ((prow >> 1) & 3);
    const int64_t a_bytes = (int64_t)(p.m - m0) * p.lda * 2;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.a + (int64_t)m0 * p.lda), 0, (int)(a_bytes < 0x7fffffff ? a_bytes : 0x7fffffff), qd::RSRC_CFG);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.w + (int64_t)n0 * p.ldw), 0, (int)((int64_t)min(BN, p.n - n0) * p.ldw * 2), qd::RSRC_CFG);
    const int va = (prow * (int)p.lda + pch * 8) * 2, vb = (prow * (int)p.ldw + pch * 8) * 2;
    const int kh_w = wave & 1;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
        if (kt == 1 && nk < 2) break;
        const uint32_t stage = lds0 + kt * G::STAGE;
        const int kb = kt * 128 + kh_w * 64;
#pragma unroll
        for (int u = 0; u < PPW; ++u) {
            const bool is_a = u < NPA / 4;
            const int rg = is_a ? (wave >> 1) + 2 * u : (wave >> 1) + 2 * u - NPA / 2;
            if (is_a)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, LDS_PTR(void, (uintptr_t)(stage + kh_w * BM * 64 + rg * 1024)),
                                                         16, va, rg * 16 * (int)p.lda * 2 + kb, 0, 0);
            else
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rw, LDS_PTR(void, (uintptr_t)(stage + G::A_IMG + kh_w * BN * 64 + rg * 1024)), 16, vb,
                    rg * 16 * (int)p.ldw * 2 + kb, 0, 0);
        }
    }
}

// The quad tile as data-parallel (one tile per block), persistent (p.persist: whole tiles strided over the grid,
// the next tile's first K-tiles prefetched before the epilogue) or stream-K (partial tiles in the SkLayout
// forward-progress order, as phased_sk_kernel).
template <int WM, int WN, int EPI, int NTERM, int STG = 0>
__global__ __launch_bounds__(256, 1) void quad_kernel(EngineArgs p) {
    using G = qd::Cfg<WM, WN>;
    constexpr int TI = G::TI, TJ = G::TJ, BM = G::BM, BN = G::BN, TS = BM * BN;
    __shared__ __attribute__((aligned(16))) char smem[G::LDS];
    if (gated_off(p)) return;
    const int tiles_m = (p.m + BM - 1) / BM, tiles_n = (p.n + BN - 1) / BN;  // (a ragged last column tile:
    const int nwg = gridDim.x, hw = blockIdx.x;                               //  not with the SwiGLU epilogue)
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    const int iters = p.k / 64;
    const int ntiles = tiles_m * tiles_n;
    f32x4 acc[TI][TJ];
    if (p.persist >= 0 && !p.sk_flag) {  // data-parallel (grid = tiles) or persistent (grid < tiles)
        bool pre = false;
        for (int tile = wg; tile < ntiles; tile += nwg) {
            int tm, tn;
            tile_coords(tile, tiles_m, tiles_n, p.group_m, tm, tn);
            if constexpr (STG == 1) {  // register staging: no cross-tile prefetch
                quad_mainloop_reg<WM, WN, NTERM, EPI == E_ADD>(p, smem, tm * BM, tn * BN, 0, iters, acc);
                __syncthreads();  // every wave's last LDS reads of this tile are done before the next tile's writes
                engine_epilogue<G, EPI>(p, tm * BM, tn * BN, acc);
                continue;
            }
            quad_mainloop<WM, WN, NTERM, EPI == E_ADD>(p, smem, tm * BM, tn * BN, 0, iters, acc, pre);
            pre = tile + nwg < ntiles;
            if (pre) {
                int tm2, tn2;
                tile_coords(tile + nwg, tiles_m, tiles_n, p.group_m, tm2, tn2);
                __syncthreads();  // every wave's last LDS reads of this tile are done
                quad_issue01<WM, WN>(p, smem, tm2 * BM, tn2 * BN, iters);
            }
            engine_epilogue<G, EPI>(p, tm * BM, tn * BN, acc);
        }
        return;
    }
    // stream-K over partial tiles (sk_flag set by the host: sk_setup)
    const int64_t ntiles64 = ntiles;
    const SkLayout lay(nwg, ntiles64);
    int grp = 0;
    const int L = lay.logical(hw, &grp);
    const int gend = lay.base(grp) + lay.size(grp);
    int64_t it, it_end;
    const int iters2 = iters / 2;  // stream-K units: pairs of K-tiles (the main loop runs whole pairs)
    lay.equal_range(L, grp, ntiles64, iters2, it, it_end);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    while (it < it_end) {
        const int tile = (int)(it / iters2), kf = (int)(it % iters2);
        const int kl = (int)min((int64_t)iters2, kf + (it_end - it));
        int tm, tn;
        tile_coords(tile, tiles_m, tiles_n, p.group_m, tm, tn);
        const int m0 = tm * BM, n0 = tn * BN;
        wait_vm<0>();
        __syncthreads();  // the previous segment's LDS readers are done
        if constexpr (STG == 1) quad_mainloop_reg<WM, WN, NTERM, EPI == E_ADD>(p, smem, m0, n0, 2 * kf, 2 * kl, acc);
        else quad_mainloop<WM, WN, NTERM, EPI == E_ADD>(p, smem, m0, n0, 2 * kf, 2 * kl, acc);
        if (kf != 0) {
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(p.sk_part + (int64_t)L * TS, 0, TS * 4, qd::RSRC_CFG);
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j) {
                    const int off = (((wave * TI + i) * TJ + j) * 64 + lane) * 16;
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, off, 0, 16);
                }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_store(p.sk_flag + L, p.sk_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (kl < iters2) {
                const int64_t tile_end = (int64_t)(tile + 1) * iters2;
                for (int c = L + 1; c < gend; ++c) {  // the tile's later pieces: lower blockIdx (SkLayout)
                    int64_t cb, ce;
                    lay.equal_range(c, grp, ntiles64, iters2, cb, ce);
                    if (cb >= tile_end) break;
                    if (ce == cb) continue;
                    if (threadIdx.x == 0) {
                        int spins = 0;
                        while (__hip_atomic_load(p.sk_flag + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != p.sk_epoch &&
                               ++spins < p.spin)
                            __builtin_amdgcn_s_sleep(1);
                        if (spins >= p.spin) report_device_error(p.err, RF_DEVERR_SK_GEMM);
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    __syncthreads();
                    const float4* src = reinterpret_cast<const float4*>(p.sk_part + (int64_t)c * TS) + wave * TI * TJ * 64 + lane;
#pragma unroll
                    for (int i = 0; i < TI; ++i)
#pragma unroll
                        for (int j = 0; j < TJ; ++j) {
                            const float4 v = src[(i * TJ + j) * 64];
                            acc[i][j][0] += v.x;
                            acc[i][j][1] += v.y;
                            acc[i][j][2] += v.z;
                            acc[i][j][3] += v.w;
                        }
                }
            }
            engine_epilogue<G, EPI>(p, m0, n0, acc);
        }
        it += kl - kf;
    }
}

// Data-parallel (one output tile per block) or stream-K (SK): the grid's blocks split the
// tiles x K-steps iteration space evenly; a block that starts inside a tile stores its partial
// sum and raises its flag, the block that holds the tile's first K-step (it reaches that tile
// last) folds the partials in and runs the epilogue.  The grid never exceeds the co-resident
// capacity, so every awaited block is running; the spin is bounded regardless.
template <class C, int EPI, int NTERM, bool GATHER, bool SK>
__global__ __launch_bounds__(C::THREADS, 2) void engine_kernel(EngineArgs p) {
    constexpr int BM = C::BM, BN = C::BN, TI = C::TI, TJ = C::TJ;
    constexpr int MAIN = C::STAGES * stage_bytes<C, NTERM>();
    __shared__ __attribute__((aligned(16))) char smem[MAIN + PN_AREA<C, EPI>];
    char* const area = smem + MAIN;
    if (gated_off(p)) return;

    const int tiles_m = (p.m + BM - 1) / BM;
    const int nwg = gridDim.x;
    const int hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    f32x4 acc[TI][TJ];
    if constexpr (!SK) {
        int tm, tn;
        tile_coords(wg, tiles_m, p.n / BN, p.group_m, tm, tn);
        const int m0 = tm * BM, n0 = tn * BN;
        pn_issue<C, EPI>(p, area, m0, n0);
        engine_mainloop<C, NTERM, GATHER, EPI == E_ADD>(p, smem, m0, n0, 0, p.k / (BK * C::KH), acc);
        engine_epilogue<C, EPI>(p, m0, n0, acc, area);
    } else {
        const int iters = p.k / (BK * C::KH);
        const int64_t ntiles64 = (int64_t)tiles_m * (p.n / BN);
        const SkLayout lay(nwg, ntiles64);  // forward-progress layout (common.h)
        int grp = 0;
        const int L = lay.logical(hw, &grp);
        const int gend = lay.base(grp) + lay.size(grp);
        int64_t it, it_end;
        lay.equal_range(L, grp, ntiles64, iters, it, it_end);
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        while (it < it_end) {
            const int tile = (int)(it / iters), kf = (int)(it % iters);
            const int kl = (int)min((int64_t)iters, kf + (it_end - it));
            int tm, tn;
            tile_coords(tile, tiles_m, p.n / BN, p.group_m, tm, tn);
            const int m0 = tm * BM, n0 = tn * BN;
            wait_vm<0>();
            __syncthreads();  // the previous segment's LDS readers are done with the ring
            if (kf == 0) pn_issue<C, EPI>(p, area, m0, n0);  // (only the tile's owner runs its epilogue)
            engine_mainloop<C, NTERM, GATHER, EPI == E_ADD>(p, smem, m0, n0, kf, kl, acc);
            if (kf != 0) {
                // partial tile in accumulator order (1 KiB per wave-instruction), stored write-through
                // (sc1) so no release fence is needed; every storing wave drains, then one lane flags
                // (guide Guideline 16, R1)
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    p.sk_part + (int64_t)L * (BM * BN), 0, BM * BN * 4, 0x00020000);
#pragma unroll
                for (int i = 0; i < TI; ++i)
#pragma unroll
                    for (int j = 0; j < TJ; ++j) {
                        const int off = (((wave * TI + i) * TJ + j) * 64 + lane) * 16;
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, off, 0, 16);
                    }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (threadIdx.x == 0) __hip_atomic_store(p.sk_flag + L, p.sk_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                if (kl < iters) {
                    const int64_t tile_end = (int64_t)(tile + 1) * iters;
                    for (int c = L + 1; c < gend; ++c) {  // the tile's later pieces: lower blockIdx (SkLayout)
                        int64_t cb, ce;
                        lay.equal_range(c, grp, ntiles64, iters, cb, ce);
                        if (cb >= tile_end) break;
                        if (ce == cb) continue;  // empty range: no partial
                        if (threadIdx.x == 0) {
                            int spins = 0;
                            while (__hip_atomic_load(p.sk_flag + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != p.sk_epoch &&
                                   ++spins < p.spin)
                                __builtin_amdgcn_s_sleep(1);
                            if (spins >= p.spin) report_device_error(p.err, RF_DEVERR_SK_GEMM);  // never silent
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // ONE acquire after the match
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        }
                        __syncthreads();
                        const float4* src =
                            reinterpret_cast<const float4*>(p.sk_part + (int64_t)c * (BM * BN)) + wave * TI * TJ * 64 + lane;
#pragma unroll
                        for (int i = 0; i < TI; ++i)
#pragma unroll
                            for (int j = 0; j < TJ; ++j) {
                                const float4 v = src[(i * TJ + j) * 64];
                                acc[i][j][0] += v.x;
                                acc[i][j][1] += v.y;
                                acc[i][j][2] += v.z;
                                acc[i][j][3] += v.w;
                            }
                    }
                }
                engine_epilogue<C, EPI>(p, m0, n0, acc, area);
            }
            it += kl - kf;
        }
    }
}

// Several independent data-parallel launches of one tile configuration as ONE grid (the DPT's four tap
// projections): problem q owns blocks [first[q], first[q + 1]); each block reads its problem's arguments
// from the kernel-argument segment at a wave-uniform index and runs the engine's tile unchanged.  Short
// launches at the DPT's 64^2 level are latency-bound (a fixed ~15 us each), so one grid overlaps them.
constexpr int GROUP_MAX = 4;
struct GroupArgs {
    EngineArgs p[GROUP_MAX];
    int first[GROUP_MAX + 1];
    int n;
};

template <class C, int EPI, int NTERM, bool GATHER>
__global__ __launch_bounds__(C::THREADS, 2) void engine_group_kernel(GroupArgs g) {
    constexpr int BM = C::BM, BN = C::BN, TI = C::TI, TJ = C::TJ;
    __shared__ __attribute__((aligned(16))) char smem[C::STAGES * stage_bytes<C, NTERM>()];
    const int nwg = gridDim.x, hw = blockIdx.x;
    const int xcd = hw & 7, qd = nwg >> 3, rd = nwg & 7;
    const int wg = (xcd < rd ? xcd * (qd + 1) : rd * (qd + 1) + (xcd - rd) * qd) + (hw >> 3);
    int q = 0;
#pragma unroll
    for (int i = 1; i < GROUP_MAX; ++i) q += (i < g.n && wg >= g.first[i]) ? 1 : 0;
    const EngineArgs& p = g.p[q];
    const int local = wg - g.first[q];
    const int tiles_m = (p.m + BM - 1) / BM;
    int tm, tn;
    tile_coords(local, tiles_m, p.n / BN, p.group_m, tm, tn);
    f32x4 acc[TI][TJ];
    engine_mainloop<C, NTERM, GATHER, EPI == E_ADD>(p, smem, tm * BM, tn * BN, 0, p.k / (BK * C::KH), acc);
    engine_epilogue<C, EPI>(p, tm * BM, tn * BN, acc);
}

// ---------------------------------------------------------------------------------------------------
// Halo-tiled 3x3 convolution (stride 1, pad 1, fp16 operands).  The im2col gather of engine_mainloop
// stages every input pixel once per tap (9x the input through L2 -> LDS per output tile); here an output
// tile of BM pixels is a TH x TW block of one image (TW = min(BM, wo), rows of m stay contiguous, so the
// epilogue is unchanged) and, per 32-channel chunk, its (TH+2) x (TW+2) input halo is staged ONCE and
// read by all nine taps at a per-tap row offset (3x the tile's pixels at TH = 1, 2x at TH = 2).  K runs
// chunk-major, tap-minor: W rows (tap * cin_pad + chunk * 32) stream through a 3-stage ring as before;
// the next chunk's halo is issued at the chunk's first tap into the other of two halo buffers and drained
// (vmcnt(0) + barrier) before the step that first reads it.
template <class C>
struct Halo {
    static constexpr int ROWS = (3 * (C::BM + 2) + 15) / 16 * 16;  // >= (TH+2)(TW+2) for every TW | BM, TW >= 16
    static constexpr int BYTES = ROWS * 64;
    static constexpr int PIECES = ROWS / 16;
    static constexpr int PPW = (PIECES + C::NWAVE - 1) / C::NWAVE;  // halo pieces per wave
    static constexpr int BST = 3;                                   // W ring stages
    static constexpr int LDS = 2 * BYTES + BST * C::B_BYTES;
};

template <class C>
RF_DEV void halo_mainloop(const EngineArgs& p, char* smem, int m0, int n0, f32x4 (&acc)[C::TI][C::TJ]) {
    using H = Halo<C>;
    constexpr int TI = C::TI, TJ = C::TJ, PB = C::PB, S = H::BST;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave / C::WGN, wn = wave % C::WGN;
    const int lg = p.halo_lg, tw = 1 << lg, hw2 = tw + 2;
    const int hr_n = ((C::BM >> lg) + 2) * hw2;  // halo rows in use
    const int per_img = p.ho * p.wo;
    const int img = m0 / per_img, rem = m0 - img * per_img;
    const int y0 = rem / p.wo, x0 = rem - y0 * p.wo;

    // halo staging: slot t of this wave is piece wave + NWAVE t (16 rows x 64 B); lane -> (row, chunk)
    int hpix[H::PPW];
#pragma unroll
    for (int t = 0; t < H::PPW; ++t) {
        const int hr = (wave + C::NWAVE * t) * 16 + (lane >> 2);
        int pix = -1;
        if (hr < hr_n) {
            const int hy = hr / hw2, hx = hr - hy * hw2;
            const int iy = y0 + hy - 1, ix = x0 + hx - 1;
            if (iy >= 0 && iy < p.hi && ix >= 0 && ix < p.wi) pix = (img * p.hi + iy) * p.wi + ix;
        }
        hpix[t] = pix;
    }
    int brow[PB], blc[PB];
#pragma unroll
    for (int pc = 0; pc < PB; ++pc) {
        brow[pc] = (wave * PB + pc) * 16 + (lane >> 2);
        blc[pc] = (lane & 3) ^ ((brow[pc] >> 1) & 3);
    }
    auto issue_halo = [&](int chunk, int buf) {
#pragma unroll
        for (int t = 0; t < H::PPW; ++t) {
            const int piece = wave + C::NWAVE * t;
            if (piece < H::PIECES) {
                const int hch = (lane & 3) ^ (((piece * 16 + (lane >> 2)) >> 1) & 3);
                const bf16_t* src = hpix[t] >= 0 ? p.a + (int64_t)hpix[t] * p.cin_pad + chunk * BK + hch * 8 : p.zero;
                __builtin_amdgcn_global_load_lds(GLB_PTR(void, src), LDS_PTR(void, smem + buf * H::BYTES + piece * 1024),
                                                 16, 0, 0);
            }
        }
    };
    auto issue_w = [&](int kt, int stage) {
        const int chunk = kt / 9, tap = kt - 9 * chunk;
        const int k0 = tap * p.cin_pad + chunk * BK;
        char* st = smem + 2 * H::BYTES + stage * C::B_BYTES;
#pragma unroll
        for (int pc = 0; pc < PB; ++pc) {
            const int piece = wave * PB + pc;
            const int64_t woff = (int64_t)(n0 + brow[pc]) * p.ldw + k0 + blc[pc] * 8;
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, p.w + woff), LDS_PTR(void, st + piece * 1024), 16, 0, 0);
        }
    };

#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nch = p.cin_pad / BK, nk = 9 * nch;
    const int frag_row = lane & 15, frag_ch = lane >> 4;
    // halo row of fragment i's output row r at tap (0, 0): r + 2 (r / TW)
    auto base_hr = [&](int i) {
        const int r = wm * C::MW + i * 16 + frag_row;
        return r + ((r >> lg) << 1);
    };
    struct Frags {
        bf16x8 a[TI], w[TJ];
    };
    auto load_frags = [&](int kt, Frags& f) {
        const int chunk = kt / 9, tap = kt - 9 * chunk;
        const int ky = tap / 3, kx = tap - 3 * ky;
        const char* hb = smem + (chunk & 1) * H::BYTES;
        const int toff = ky * hw2 + kx;
#pragma unroll
        for (int i = 0; i < TI; ++i)
            f.a[i] = *reinterpret_cast<const bf16x8*>(hb + lds_off(base_hr(i) + toff, frag_ch));
        const char* st = smem + 2 * H::BYTES + (kt % S) * C::B_BYTES;
#pragma unroll
        for (int j = 0; j < TJ; ++j)
            f.w[j] = *reinterpret_cast<const bf16x8*>(st + lds_off(wn * C::NWD + j * 16 + frag_row, frag_ch));
    };
    auto mma = [&](const Frags& f) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, f.w[j]),
                                                                   __builtin_bit_cast(f16x8, f.a[i]), acc[i][j], 0, 0, 0);
    };
    // W tile kt+1 landed (over-waiting when halo pieces are among the younger DMAs is safe)
    auto wait_w = [&](int younger) {
        if (younger >= 1) wait_vm<PB>();
        else wait_vm<0>();
    };

    issue_halo(0, 0);
#pragma unroll
    for (int st = 0; st < S; ++st) issue_w(st, st);
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    Frags f0, f1;
    load_frags(0, f0);
    auto step = [&](int kt, Frags& cur, Frags& nxt) {
        __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's fragment reads of `cur` are complete
        if (kt + 1 < nk) {
            if ((kt + 1) % 9 == 0) wait_vm<0>();  // tile kt+1 starts a chunk: its halo (and all W) landed
            else wait_w(std::min(S - 2, nk - 2 - kt));
        }
        __builtin_amdgcn_s_barrier();  // every wave's DMA landed and every wave's reads of tile kt are done
        __builtin_amdgcn_sched_barrier(0);
        const int chunk = kt / 9;
        if (kt - 9 * chunk == 0 && chunk + 1 < nch) issue_halo(chunk + 1, (chunk + 1) & 1);
        if (kt + S < nk) issue_w(kt + S, kt % S);
        if (kt + 1 < nk) load_frags(kt + 1, nxt);
        mma(cur);
    };
    for (int kt = 0; kt < nk; kt += 2) {
        step(kt, f0, f1);
        if (kt + 1 < nk) step(kt + 1, f1, f0);
    }
}

template <class C, int EPI>
__global__ __launch_bounds__(C::THREADS, C::BM == 256 ? 1 : 2) void halo_kernel(EngineArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[Halo<C>::LDS];
    if (gated_off(p)) return;
    const int tiles_m = p.m / C::BM;
    const int nwg = gridDim.x;
    const int hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    int tm, tn;
    tile_coords(wg, tiles_m, p.n / C::BN, p.group_m, tm, tn);
    f32x4 acc[C::TI][C::TJ];
    halo_mainloop<C>(p, smem, tm * C::BM, tn * C::BN, acc);
    engine_epilogue<C, EPI>(p, tm * C::BM, tn * C::BN, acc);
}

// ---------------------------------------------------------------------------------------------------
// Halo-tiled 3x3 convolution on 2-D output tiles: 16 x 32 pixels x 128 output channels per block (8 waves,
// each 4 rows x 32 pixels x 64 channels = the phased 256x256 GEMM's 128x64 wave tile).  The 1-row-high
// halo_kernel above re-reads the whole filter bank (K = 9 cin) for every 128 pixels, and at 512^2 that weight
// stream (1.2 GB for output_conv1) bounds it; a 512-pixel block reads the bank 4x less often and its halo is
// 1.2x the tile's pixels instead of 3x.  K runs chunk-major (32 input channels), tap-minor: per chunk the
// 18 x 34 halo is staged once (40 x 1-KiB LDS-DMA pieces, 5 per wave, issued during the previous chunk into
// the other of two buffers) and every tap reads its fragments at a shifted halo index (the XOR image of
// lds_off is bank-conflict-free for 16 consecutive pixels from any start); the 8-KiB W slice of each
// (chunk, tap) step streams through an S-deep ring.  Each step is two phases of 16 MFMAs (fragment rows 0-3,
// then 4-7, sharing the step's four W fragments) in the phased loop's form: load section, barrier, MFMA
// section, barrier, with waves 4-7 one section behind so each SIMD overlaps one wave's LDS reads with its
// partner's MFMAs.  One counted vmcnt per step (h2_wait) publishes the next step's W slice, and at a chunk's
// last tap also the next chunk's halo (issued before that W slice).
namespace h2 {
constexpr int TH = 16, TW = 32, HWID = TW + 2, HPIX = (TH + 2) * HWID;  // 612 halo pixels
// The halo's 16-B chunk XOR key, a function of the halo column hx only (one halo row down is then a constant
// HWID * 64 bytes for every lane).  A fragment read (ds_read_b128: pixel = lane & 15, chunk = lane >> 4) is served
// in four 16-lane groups, each mixing 8 lanes of one chunk over pixels {0-3, 12-15} with 8 lanes of the next chunk
// over pixels 4-11; the key must give those 16 lanes 16 distinct bank quads for every tap shift (0-2) of the column.
// ((hx >> 2) & 3), used through round 4, made every such read 2-way conflicted (SQ_LDS_BANK_CONFLICT = half of
// SQ_LDS_IDX_ACTIVE, profiles/r4_halo_lds.txt); ((hx >> 1) & 2) is conflict-free for all shifts (tools/halo_key.py).
RF_DEV constexpr int hkey(int hx) { return (hx >> 1) & 2; }
constexpr int PIECES = 40, PPW = PIECES / 8;                            // 1-KiB pieces per buffer, per wave
constexpr int HBYTES = PIECES * 1024;                                   // 640 pixel slots x 64 B
static_assert(PIECES * 16 >= HPIX, "halo buffer");
// LDS-DMA left in flight when step t's wait must have landed W(t+1): the issue events after W(t+1) are, per
// step j in [t + 2 - S, t], a halo piece (taps 0-4 of a chunk with a successor) and W(j + S) (if it exists;
// steps before the loop stand for the prologue's W issues)
constexpr int wait_count(int t, int S, bool last) {
    int n = 0;
    for (int j = t + 2 - S; j <= t; ++j) {
        if (last) n += (j < 0 || j + S < 9) ? 1 : 0;
        else n += 1 + ((j >= 0 && j < 5) ? 1 : 0);
    }
    return n;
}
}  // namespace h2
// BN = 128 output channels: 4 x 2 waves of 4 rows x 64 channels; BN = 64 (output_conv2's 32 padded to 64):
// 8 x 1 waves of 2 rows x 64 channels
template <int S, int BN>
struct H2Cfg {
    static constexpr int WGN = BN / 64, WGM = 8 / WGN, RW = h2::TH / WGM;  // tile rows per wave
    static constexpr int TI = 2 * RW, TJ = 4, WBYTES = BN * 64;            // fragments; W stage (BN x 32 ci x 2 B)
    static constexpr int LDS = 2 * h2::HBYTES + S * WBYTES;
    static_assert(BN == 64 || BN == 128, "halo2 channel tile");
};
// the epilogue's view of the block (engine_epilogue reads these members only)
template <int BN>
struct H2Tile {
    static constexpr int WGN = BN / 64, WGM = 8 / WGN, MW = 512 / WGM, NWD = 64, TI = MW / 16, TJ = 4;
};

template <int N>
RF_DEV void wait_vm_rt(int n) {  // vmcnt(n) for a wave-uniform n <= N (the unrolled callers pass constants)
    if constexpr (N > 0) {
        if (n >= N) {
            wait_vm<N>();
            return;
        }
        wait_vm_rt<N - 1>(n);
    } else {
        wait_vm<0>();
    }
}

// DBG (ablation timing only, wrong results): 1 = no MFMAs, 2 = no LDS-DMA after the prologue, 3 = no stagger;
// (right results) 4 = no static priority for the MFMA section, 8 = priority for the load section instead.
// One step = one load section {W fragments + all TI A fragments, the next chunk's halo piece (taps 0-4), W(kt + S - 1)
// into the slot step kt - 1 read, counted wait for W(kt + 1)} and one MFMA section (4 TI MFMAs); with the two halves
// of a step in separate sections (two barriers more per step) the 256^2 conv took 115 instead of 103 us.
template <int S, int BN, int DBG = 0>
RF_DEV void halo2_mainloop(const EngineArgs& p, char* smem, int img, int y0, int x0, int n0,
                           f32x4 (&acc)[H2Cfg<S, BN>::TI][4]) {
    using namespace h2;
    using G = H2Cfg<S, BN>;
    constexpr int TI = G::TI, WBYTES = G::WBYTES;
    static_assert(S >= 3 && S <= 5, "W ring depth (S - 1 slices in flight; the chunk's halo must precede W(next chunk))");
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave / G::WGN, wn = wave % G::WGN;
    // W stage: BN / 16 one-KiB pieces, one per wave of waves 0 .. BN / 16 - 1 (the rest stage no W and count
    // only their halo pieces)
    const bool has_w = BN == 128 || __builtin_amdgcn_readfirstlane(wave) < BN / 16;
    const int nch = p.cin_pad / 32, nk = 9 * nch;
    char* hbuf = smem;                    // two halo buffers
    char* wring = smem + 2 * HBYTES;      // S W stages

    // halo staging: piece wave + 8 t of a buffer holds halo pixels 16 (wave + 8 t) .. + 15 (64 B each, 16-B chunk
    // XOR h2::hkey(column): a function of the halo column only, so one halo row down is a constant HWID * 64 bytes
    // for every lane and a tap's fragment address is a per-(column half, tap column) register plus an immediate
    // (no per-tap address VALU); the fragment reads are conflict-free for every tap shift).  Pixels past the
    // image or past the 612 in use read the zero row
    int hpix[PPW], hch[PPW];
#pragma unroll
    for (int t = 0; t < PPW; ++t) {
        const int hp = (wave + 8 * t) * 16 + (lane >> 2);
        hch[t] = (lane & 3) ^ h2::hkey(hp % HWID);
        int pix = -1;
        if (hp < HPIX) {
            const int hy = hp / HWID, hx = hp - hy * HWID;
            const int iy = y0 + hy - 1, ix = x0 + hx - 1;
            if (iy >= 0 && iy < p.hi && ix >= 0 && ix < p.wi) pix = (img * p.hi + iy) * p.wi + ix;
        }
        hpix[t] = pix;
    }
    auto issue_halo = [&](int chunk, int t) {  // piece t of this wave, chunk's 32 channels, into buffer chunk & 1
        const bf16_t* src = hpix[t] >= 0 ? p.a + (int64_t)hpix[t] * p.cin_pad + hch[t] * 8 + chunk * 32 : p.zero;
        __builtin_amdgcn_global_load_lds(GLB_PTR(void, src),
                                         LDS_PTR(void, hbuf + (chunk & 1) * HBYTES + (wave + 8 * t) * 1024), 16, 0, 0);
    };
    // W staging: wave w fills rows 16 w .. 16 w + 15 of a stage (one 1-KiB piece per lane-instruction)
    const int wrow = 16 * wave + (lane >> 2);
    const bf16_t* wsrc = p.w + (int64_t)(n0 + wrow) * p.ldw + (((lane & 3) ^ ((wrow >> 1) & 3)) * 8);
    auto issue_w = [&](int kt) {
        if (!has_w) return;
        const int chunk = kt / 9, tap = kt - 9 * chunk;
        __builtin_amdgcn_global_load_lds(GLB_PTR(void, wsrc + tap * p.cin_pad + chunk * 32),
                                         LDS_PTR(void, wring + (kt % S) * WBYTES + wave * 1024), 16, 0, 0);
    };

#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int frow = lane & 15, fch = lane >> 4;
    // LDS byte address (in the current halo buffer) of fragment i's lane pixel at tap (ty, tx): tile row
    // RW wm + i / 2 + ty, halo column hx = 16 (i & 1) + frow + tx; = hadr[i & 1][tx] + (i / 2 + ty) HWID 64,
    // the second term an immediate of the unrolled loops.  hadr moves between the two halo buffers per chunk.
    uint32_t hadr[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) {
            const int hx = 16 * h + frow + tx;
            hadr[h][tx] = (uint32_t)(uintptr_t)LDS_PTR(char, hbuf) + ((G::RW * wm) * HWID + hx) * 64 +
                          ((fch ^ h2::hkey(hx)) << 4);
        }
    bf16x8 fa[TI], fb[4];
    auto read_a = [&](int tap) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
            fa[i] = *LDS_PTR(const bf16x8, (uintptr_t)(hadr[i & 1][tap % 3] + ((i >> 1) + tap / 3) * HWID * 64));
    };
    auto read_b = [&](int slot) {
        int soff = slot * WBYTES;
        asm volatile("" : "+s"(soff));
        const char* ws = wring + soff;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            fb[j] = *reinterpret_cast<const bf16x8*>(ws + lds_off(wn * 64 + j * 16 + frow, fch));
    };
    auto mma = [&]() {
        if constexpr (DBG == 1) return;
        if constexpr (DBG != 4 && DBG != 8) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fb[j]),
                                                                   __builtin_bit_cast(f16x8, fa[i]), acc[i][j], 0, 0, 0);
        if constexpr (DBG != 4 && DBG != 8) __builtin_amdgcn_s_setprio(0);
    };
    auto sync_in = [&]() {
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this section's fragments are in registers
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    auto sync_out = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    // prologue: chunk 0's halo and W(0 .. S-2), all landed
#pragma unroll
    for (int t = 0; t < PPW; ++t) issue_halo(0, t);
#pragma unroll
    for (int kt = 0; kt < S - 1; ++kt)
        if (kt < nk) issue_w(kt);
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const bool late = DBG != 3 && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256;  // waves 4-7: one section behind
    if (late) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);

    for (int c = 0; c < nch; ++c) {
        const bool last = c + 1 == nch;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int kt = 9 * c + t;
            if constexpr (DBG == 8) __builtin_amdgcn_s_setprio(1);  // ablation: the load section outranks the MFMAs
            read_b(kt % S);
            read_a(t);
            // slot (kt - 1) % S was read by both wave groups before the barrier this section started after
            if (DBG != 2 && t < PPW && !last) issue_halo(c + 1, t);
            if (DBG != 2 && kt + S - 1 < nk) issue_w(kt + S - 1);
            if (has_w) {
                if (t < 8 || !last) {  // W(kt + 1) landed: the same event count as an (S-1)-stage ring
                    if (last) wait_vm_rt<4>(wait_count(t, S - 1, true));
                    else wait_vm_rt<8>(wait_count(t, S - 1, false));
                }
            } else if (t == 8 && !last) {
                wait_vm<0>();  // no W staged by this wave: only its pieces of the next chunk's halo
            }
            if constexpr (DBG == 8) __builtin_amdgcn_s_setprio(0);
            sync_in();
            mma();
            sync_out();
        }
        const uint32_t step = (c & 1) ? (uint32_t)-HBYTES : (uint32_t)HBYTES;  // next chunk: the other halo buffer
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int tx = 0; tx < 3; ++tx) hadr[h][tx] += step;
    }
    if (!late) __builtin_amdgcn_s_barrier();  // re-align the groups' barrier counts
}

template <int S, int BN, int DBG = 0>
__global__ __launch_bounds__(512, 1) void halo2_kernel(EngineArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[H2Cfg<S, BN>::LDS];
    // XCD-contiguous tile ids (consecutive ids share an XCD's L2: the two channel tiles of one pixel tile and
    // neighbouring pixel tiles, whose halos overlap); tile id = pixel tile * n_tiles + channel tile
    const int nwg = gridDim.x, hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    const int tiles_n = p.n / BN, tx_n = p.wo / h2::TW, ty_n = p.ho / h2::TH;
    const int tn = wg % tiles_n, pt = wg / tiles_n;
    const int tx = pt % tx_n, rest = pt / tx_n;
    const int ty = rest % ty_n, img = rest / ty_n;
    const int y0 = ty * h2::TH, x0 = tx * h2::TW;
    f32x4 acc[H2Cfg<S, BN>::TI][4];
    halo2_mainloop<S, BN, DBG>(p, smem, img, y0, x0, tn * BN, acc);
    engine_epilogue<H2Tile<BN>, E_CONV, h2::TW, BN == 64>(p, (img * p.ho + y0) * p.wo + x0, tn * BN, acc);
}

// ---------------------------------------------------------------------------------------------------
// halo3: halo2's block (16 x 32 pixels x 128 output channels, 8 waves, the same halo image and double buffer) with
// the filter bank read straight from L2 into registers instead of through an LDS ring.  halo2 needed two barriers
// per (chunk, tap) step because the W slice of each step was a shared LDS stage; its ablations showed the
// load / sync skeleton taking half the kernel (58.5 of 114.6 us).  Here the only shared LDS data is
// the halo, so a whole 32-channel chunk (9 taps, 288 MFMAs per wave) runs between two barriers, and the two waves
// of a SIMD interleave freely.  Waves are 2 (rows) x 4 (channels): each owns 8 tile rows (16 pixel fragments) x 32
// channels (2 W fragments), so per tap a wave reads 16 A fragments from LDS (128 KiB per CU per tap: half the LDS
// array's rate at the MFMA's) and 2 W fragments (2 KiB) from the L2-resident bank through a 3-deep register ring,
// two taps ahead.  The bank (9 cin x 128 x 2 B per block, 0.6 MB at cin 256) is read 2x per block from L2.
namespace h3 {
constexpr int WGN = 4, WGM = 2, RW = h2::TH / WGM, TI = 2 * RW, TJ = 2;  // 8 rows x 32 pixels x 32 channels per wave
constexpr int LDS = 2 * h2::HBYTES;                                     // two halo buffers (80 KiB)
}  // namespace h3
struct H3Tile {  // the epilogue's view of the block
    static constexpr int WGN = h3::WGN, WGM = h3::WGM, MW = 512 / h3::WGM, NWD = 128 / h3::WGN, TI = h3::TI,
                         TJ = h3::TJ;
};

// DBG (ablation timing only, wrong results): 1 = no MFMAs, 2 = no W loads in the loop, 4 = no halo DMA in the loop,
// 8 = no chunk-end wait + barrier
template <int DBG = 0>
__global__ __launch_bounds__(512, 1) void halo3_kernel(EngineArgs p) {
    using namespace h2;
    __shared__ __attribute__((aligned(16))) char smem[h3::LDS];
    constexpr int TI = h3::TI;
    // XCD-contiguous tile ids as halo2 (the channel tiles of one pixel tile and neighbouring pixel tiles share an L2)
    const int nwg = gridDim.x, hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    const int tiles_n = p.n / 128, tx_n = p.wo / TW, ty_n = p.ho / TH;
    const int tn = wg % tiles_n, pt = wg / tiles_n;
    const int tx = pt % tx_n, rest = pt / tx_n;
    const int ty = rest % ty_n, img = rest / ty_n;
    const int y0 = ty * TH, x0 = tx * TW, n0 = tn * 128;

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave / h3::WGN, wn = wave % h3::WGN;
    const int nch = p.cin_pad / 32, nk = 9 * nch;
    char* hbuf = smem;

    // halo staging exactly as halo2 (piece wave + 8 t of a buffer = halo pixels 16 (wave + 8 t) .. + 15)
    int hpix[PPW], hch[PPW];
#pragma unroll
    for (int t = 0; t < PPW; ++t) {
        const int hp = (wave + 8 * t) * 16 + (lane >> 2);
        hch[t] = (lane & 3) ^ h2::hkey(hp % HWID);
        int pix = -1;
        if (hp < HPIX) {
            const int hy = hp / HWID, hx = hp - hy * HWID;
            const int iy = y0 + hy - 1, ix = x0 + hx - 1;
            if (iy >= 0 && iy < p.hi && ix >= 0 && ix < p.wi) pix = (img * p.hi + iy) * p.wi + ix;
        }
        hpix[t] = pix;
    }
    // The halo pieces are issued by inline asm: with the builtin, hipcc counts the LDS-DMA as a second kind of
    // vector-memory event and, unable to order it against the W loads, waits vmcnt(0) at every third tap (the
    // W ring's prefetch then never overlaps).  Hidden from it, its vmcnt for a W slot also covers the (older) halo
    // pieces issued between, which only waits for what landed long ago; the chunk-end wait publishes the halo.
    // M0 is clobbered: every M0 use in this kernel is one of these statements.
    const uint32_t hbase = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(char, hbuf) + wave * 1024);
    auto issue_halo = [&](int chunk, int buf, int t) {
        const bf16_t* src = hpix[t] >= 0 ? p.a + (int64_t)hpix[t] * p.cin_pad + hch[t] * 8 + chunk * 32 : p.zero;
        const uint32_t lds = hbase + buf * HBYTES + t * 8 * 1024;
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds)
                     : "memory", "m0");
    };

    const int frow = lane & 15, fch = lane >> 4;
    // W fragment j of this wave: filter rows n0 + 32 wn + 16 j + frow, K = tap * cin_pad + 32 chunk + 8 fch .. + 7
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.w + (int64_t)n0 * p.ldw), 0, (int)((int64_t)128 * p.ldw * 2), qd::RSRC_CFG);
    const int wv0 = ((wn * 32 + frow) * (int)p.ldw + fch * 8) * 2, wv1 = wv0 + 16 * (int)p.ldw * 2;
    u32x4 fb[3][2];  // ring slot kt % 3 (9 taps per chunk: the slot of a tap does not depend on its chunk)
    auto load_b = [&](int kt, int slot) {
        const int chunk = kt / 9, tap = kt - 9 * chunk;
        const int so = (tap * p.cin_pad + chunk * 32) * 2;
        fb[slot][0] = __builtin_amdgcn_raw_buffer_load_b128(rw, wv0, so, 0);
        fb[slot][1] = __builtin_amdgcn_raw_buffer_load_b128(rw, wv1, so, 0);
    };

    f32x4 acc[TI][2];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // LDS byte address of fragment i's lane pixel at tap (ty, tx): tile row RW wm + i / 2 + ty, halo column
    // 16 (i & 1) + frow + tx (halo2's register + immediate form)
    uint32_t hadr[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int tx3 = 0; tx3 < 3; ++tx3) {
            const int hx = 16 * h + frow + tx3;
            hadr[h][tx3] = (uint32_t)(uintptr_t)LDS_PTR(char, hbuf) + ((h3::RW * wm) * HWID + hx) * 64 +
                           ((fch ^ h2::hkey(hx)) << 4);
        }

    // prologue: chunk 0's halo and W(0), W(1)
#pragma unroll
    for (int t = 0; t < PPW; ++t) issue_halo(0, 0, t);
    load_b(0, 0);
    load_b(min(1, nk - 1), 1);
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);

    for (int c = 0; c < ((DBG & 32) ? 0 : nch); ++c) {  // DBG 32 (ablation): prologue + epilogue only
        const bool last = c + 1 == nch;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int kt = 9 * c + t;
            bf16x8 fa[TI];
#pragma unroll
            for (int i = 0; i < TI; ++i) {
                if constexpr (DBG & 16) {  // ablation: no fragment reads (the MFMAs take lane-dependent junk)
                    fa[i] = __builtin_bit_cast(bf16x8, u32x4{(uint32_t)(lane + i), (uint32_t)t, 0u, (uint32_t)c});
                } else {
                    fa[i] = *LDS_PTR(const bf16x8, (uintptr_t)(hadr[i & 1][t % 3] + ((i >> 1) + t / 3) * HWID * 64));
                }
            }
            // branch-free issue (a conditional load makes hipcc's vmcnt accounting fall back to vmcnt(0) at the
            // ring slot's next use): the last chunk re-stages its own halo into the idle buffer and the last two
            // taps re-load the last W slice
            if (!(DBG & 4) && t < PPW) issue_halo(last ? c : c + 1, (c + 1) & 1, t);
            if (!(DBG & 2)) load_b(min(kt + 2, nk - 1), (t + 2) % 3);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if constexpr (DBG & 1) {  // ablation: no MFMAs (the reads stay live)
                        if (j == 0) asm volatile("" ::"v"(fa[i]));
                    } else {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fb[t % 3][j]),
                                                                           __builtin_bit_cast(f16x8, fa[i]), acc[i][j], 0, 0, 0);
                    }
                }
            __builtin_amdgcn_s_setprio(0);
        }
        if (!(DBG & 8) && !last) {
            // the next chunk's halo (and the W loads behind it) landed, and every wave is done reading this chunk's
            // buffer, which the chunk after next overwrites
            wait_vm<0>();
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t step = (c & 1) ? (uint32_t)-HBYTES : (uint32_t)HBYTES;
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int tx3 = 0; tx3 < 3; ++tx3) hadr[h][tx3] += step;
        }
    }
    wait_vm<0>();  // the last chunk's re-staged halo pieces land before the block's LDS is released
    if constexpr ((DBG & 64) != 0) {  // ablation: no epilogue (the accumulators stay live)
#pragma unroll
        for (int i = 0; i < TI; ++i) asm volatile("" ::"v"(acc[i][0]), "v"(acc[i][1]));
        return;
    }
    engine_epilogue<H3Tile, E_CONV, TW, false>(p, (img * p.ho + y0) * p.wo + x0, n0, acc);
}

// ---------------------------------------------------------------------------------------------------
// The DPT's last 3x3 convolution (output_conv2, dpt.py:234-240: <= 32 filters, fp16) with its fused head
// (SiLU -> 1x1 to n_fin -> ELU -> 10^x - 1).  The halo2 kernel pads the 32-filter bank to a 64-wide tile (half
// its MFMAs multiply zeros) and runs 16 MFMAs per barrier-delimited section, which left it bound by its section
// overheads (68 us for 19.3 GFLOP at 512^2).  Here a block is 4 waves (one per SIMD) over a 16 x 32
// pixel tile with exactly 32 output channels: each wave owns 4 tile rows (8 fragments of 16 pixels) x 32
// channels, so one (chunk, tap) step is 16 useful MFMAs per wave, and a whole 32-channel chunk (9 taps, 144
// MFMAs per wave) runs between two barriers.  Per chunk the 18 x 34 halo (40 KiB, halo2's column-keyed XOR
// image: conflict-free fragment reads) and the chunk's 9 W slices (18 KiB) land by LDS-DMA in one of two
// buffers while the previous chunk computes.  The input plane is read ~1.2x (the halo), the bank once per block.
namespace c32 {
constexpr int TH = 16, TW = 32, HWID = TW + 2, HPIX = (TH + 2) * HWID;  // 612 halo pixels
constexpr int HPIECES = 40, WPIECES = 18;                               // 1-KiB pieces per chunk
constexpr int HBYTES = HPIECES * 1024, WBYTES = WPIECES * 1024, BUF = HBYTES + WBYTES;
constexpr int NWAVE = 4, HPW = HPIECES / NWAVE;                         // 10 halo pieces per wave
constexpr int LDS = 2 * BUF;                                             // 116 KiB: one block per CU
constexpr int NFIN = 4;                                                  // head outputs (RGB: 3)
}  // namespace c32

__global__ __launch_bounds__(256, 1) void conv3x3_c32_kernel(EngineArgs p) {
    using namespace c32;
    __shared__ __attribute__((aligned(16))) char smem[LDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-contiguous tile ids (neighbouring tiles, whose halos overlap, share an XCD's L2)
    const int nwg = gridDim.x, hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    const int tx_n = p.wo / TW, ty_n = p.ho / TH;
    const int tx = wg % tx_n, rest = wg / tx_n;
    const int ty = rest % ty_n, img = rest / ty_n;
    const int y0 = ty * TH, x0 = tx * TW;
    const int nch = p.cin_pad / 32;

    // halo piece t of this wave = halo pixels 16 (wave + 4 t) .. + 15, 64 B each (16-B chunk ^ column key)
    int hpix[HPW], hch[HPW];
#pragma unroll
    for (int t = 0; t < HPW; ++t) {
        const int hp = (wave + NWAVE * t) * 16 + (lane >> 2);
        hch[t] = (lane & 3) ^ h2::hkey(hp % HWID);
        int pix = -1;
        if (hp < HPIX) {
            const int hy = hp / HWID, hx = hp - hy * HWID;
            const int iy = y0 + hy - 1, ix = x0 + hx - 1;
            if (iy >= 0 && iy < p.hi && ix >= 0 && ix < p.wi) pix = (img * p.hi + iy) * p.wi + ix;
        }
        hpix[t] = pix;
    }
    // W piece v (0..17) = tap v / 2, output channels 16 (v & 1) .. + 15 (rows of the [cout_pad][9][cin_pad] bank)
    const int wr = lane >> 2;
    auto issue = [&](int chunk, int buf) {
        char* b = smem + buf * BUF;
#pragma unroll
        for (int t = 0; t < HPW; ++t) {
            const bf16_t* src = hpix[t] >= 0 ? p.a + (int64_t)hpix[t] * p.cin_pad + hch[t] * 8 + chunk * 32 : p.zero;
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, src), LDS_PTR(void, b + (wave + NWAVE * t) * 1024), 16, 0, 0);
        }
        for (int v = wave; v < WPIECES; v += NWAVE) {  // waves 0, 1: 5 pieces; 2, 3: 4 (wave-uniform)
            const int tap = v >> 1, row = 16 * (v & 1) + wr;
            const bf16_t* src = p.w + (int64_t)row * p.ldw + tap * p.cin_pad + chunk * 32 + (((lane & 3) ^ ((row >> 1) & 3)) * 8);
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, src), LDS_PTR(void, b + HBYTES + v * 1024), 16, 0, 0);
        }
    };
    const int n_issue = HPW + (WPIECES - wave + NWAVE - 1) / NWAVE;  // LDS-DMA per wave per chunk (14 or 15)

    f32x4 acc[8][2];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int frow = lane & 15, fch = lane >> 4;
    // fragment i = tile row 4 wave + i / 2, columns 16 (i & 1) .. + 15; at tap (ty, tx) its lane's halo pixel is
    // row 4 wave + i / 2 + ty, column hx = 16 (i & 1) + frow + tx: hadr[i & 1][tx] + (i / 2 + ty) HWID 64
    uint32_t hadr[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int hx = 16 * h + frow + t;
            hadr[h][t] = (uint32_t)(uintptr_t)LDS_PTR(char, smem) + ((4 * wave) * HWID + hx) * 64 +
                         ((fch ^ h2::hkey(hx)) << 4);
        }
    const uint32_t wadr = (uint32_t)(uintptr_t)LDS_PTR(char, smem) + HBYTES + lds_off(frow, fch);

    issue(0, 0);
    for (int c = 0; c < nch; ++c) {
        const int buf = c & 1;
        if (c + 1 < nch) {
            issue(c + 1, buf ^ 1);  // lands under this chunk's MFMAs
            wait_vm_rt<16>(n_issue);  // this wave's pieces of chunk c landed (chunk c + 1's still in flight)
        } else {
            wait_vm<0>();
        }
        __builtin_amdgcn_s_barrier();  // every wave's pieces of chunk c landed
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t bo = buf * BUF;
        // one wave per SIMD: tap t + 1's fragments are read under tap t's MFMAs (two register sets)
        bf16x8 fa[2][8], fb[2][2];
        auto rd = [&](int tap, int s) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
                fb[s][j] = *LDS_PTR(const bf16x8, (uintptr_t)(wadr + bo + tap * 2048 + j * 1024));
#pragma unroll
            for (int i = 0; i < 8; ++i)
                fa[s][i] = *LDS_PTR(const bf16x8, (uintptr_t)(hadr[i & 1][tap % 3] + bo + ((i >> 1) + tap / 3) * HWID * 64));
        };
        rd(0, 0);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int s = tap & 1;
            if (tap + 1 < 9) rd(tap + 1, s ^ 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fb[s][j]),
                                                                       __builtin_bit_cast(f16x8, fa[s][i]), acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();  // buffer `buf` is free for chunk c + 2
    }

    // fused head: acc[i][j][e] = conv channel 16 j + 4 (lane >> 4) + e of pixel (tile row 4 wave + i / 2, column
    // 16 (i & 1) + (lane & 15)); s_f = sum_c silu(conv_c + b_c) w_fin[f, c], the 32 channels of a pixel summed over
    // the lane's 8 and the four lane groups
    float bsum[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int col = j * 16 + 4 * (lane >> 4) + e;
            bsum[j][e] = (p.bias && col < p.cout) ? p.bias[col] : 0.f;
        }
    const int hwp = p.ho * p.wo;
    // silu(conv + bias) once per value (64 per lane: one wave per SIMD has the registers), then n_fin dot products
    float sv[8][2][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) sv[i][j][e] = silu(acc[i][j][e] + bsum[j][e]);
    // every head weight is read before the first store: a load issued after a store waits for it (vmcnt counts
    // both in issue order), and b_fin re-read per pixel fragment made each fragment wait for the previous one's
    // stores (n_fin <= c32::NFIN, c32_ok)
    const float* __restrict__ w_fin = p.w_fin;
    const float* __restrict__ b_fin = p.b_fin;
    float* __restrict__ out = reinterpret_cast<float*>(p.c);
    float wf[NFIN][2][4], bf[NFIN];
#pragma unroll
    for (int f = 0; f < NFIN; ++f) {
        bf[f] = f < p.n_fin ? b_fin[f] : 0.f;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int col = j * 16 + 4 * (lane >> 4) + e;
                wf[f][j][e] = (f < p.n_fin && col < p.cout) ? w_fin[f * p.cout + col] : 0.f;
            }
    }
#pragma unroll
    for (int f = 0; f < NFIN; ++f) {
        if (f >= p.n_fin) break;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) s += sv[i][j][e] * wf[f][j][e];
            s += __shfl_xor(s, 16, 64);
            s += __shfl_xor(s, 32, 64);
            if (lane < 16) {
                const int m = (img * p.ho + y0 + 4 * wave + (i >> 1)) * p.wo + x0 + 16 * (i & 1) + lane;
                float y = elu_fast(s + bf[f], p.elu_alpha);
                if (p.flags & RF_CONV_LOG_DECODE) y = pow10m1_fast(y);
                const int64_t o = (p.flags & RF_CONV_NCHW_OUT) ? ((int64_t)(m / hwp) * p.n_fin + f) * hwp + (m % hwp)
                                                              : (int64_t)m * p.n_fin + f;
                out[o] = y;
            }
        }
    }
}

#ifdef RF_STUDY  // conv3x3_hk_kernel (measured slower than halo3): study build only
// ---------------------------------------------------------------------------------------------------
// conv3x3_hk_kernel: the chunk-per-barrier structure of conv3x3_c32_kernel for 3x3 / stride 1 / pad 1 fp16
// convolutions with any multiple of 64 output channels and the full conv epilogue (bias / border-class bias,
// residuals, SiLU, fp32 and fp16-plane outputs): DPT output_conv1 (512^2, 256 -> 128) and the 256^2 level's
// ResidualConvUnits (256 -> 256), which halo2_kernel ran at 0.25-0.31 of peak with two barriers per (chunk,
// tap) step.  A block is 4 waves (one per SIMD, the whole register file) over a 16 x 32 pixel tile and 64
// output channels; each wave owns 4 tile rows (8 fragments of 16 pixels) x 64 channels, so one tap is 32 MFMAs
// per wave and a 32-channel chunk (9 taps, 288 MFMAs) runs between two barriers.  Per chunk the 18 x 34 halo
// (40 KiB, column-keyed XOR image) and the chunk's 9 W slices (36 KiB) land by LDS-DMA in one of two buffers
// (152 KiB in all) while the previous chunk computes.  Blocks walk pixel tile-major (the channel tiles of a
// pixel tile are consecutive ids: same XCD, the halo is read from L2 by the second).
namespace hk {
constexpr int TH = 16, TW = 32, HWID = TW + 2, HPIX = (TH + 2) * HWID;  // 612 halo pixels
constexpr int NCO = 64;                                                  // output channels per block
constexpr int HPIECES = 40, WPIECES = 9 * NCO / 16;                     // 1-KiB pieces per chunk (40 + 36)
constexpr int HBYTES = HPIECES * 1024, WBYTES = WPIECES * 1024, BUF = HBYTES + WBYTES;
constexpr int NWAVE = 4, HPW = HPIECES / NWAVE, WPW = WPIECES / NWAVE;   // 10 + 9 pieces per wave
constexpr int LDS = 2 * BUF;                                             // 152 KiB: one block per CU
static_assert(WPIECES % NWAVE == 0 && LDS <= 160 * 1024, "hk: LDS budget");
}  // namespace hk
// the epilogue's view of the block: 4 waves stacked over the pixel rows, 128 pixels (4 rows of 32) x 64 channels
struct HkTile {
    static constexpr int WGN = 1, WGM = 4, MW = 128, NWD = 64, TI = 8, TJ = 4;
};

__global__ __launch_bounds__(256, 1) void conv3x3_hk_kernel(EngineArgs p) {
    using namespace hk;
    __shared__ __attribute__((aligned(16))) char smem[LDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwg = gridDim.x, hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    const int tiles_n = p.n / NCO, tx_n = p.wo / TW, ty_n = p.ho / TH;
    const int tn = wg % tiles_n, pt = wg / tiles_n;
    const int tx = pt % tx_n, rest = pt / tx_n;
    const int ty = rest % ty_n, img = rest / ty_n;
    const int y0 = ty * TH, x0 = tx * TW, n0 = tn * NCO;
    const int nch = p.cin_pad / 32;

    int hpix[HPW], hch[HPW];
#pragma unroll
    for (int t = 0; t < HPW; ++t) {
        const int hp = (wave + NWAVE * t) * 16 + (lane >> 2);
        hch[t] = (lane & 3) ^ h2::hkey(hp % HWID);
        int pix = -1;
        if (hp < HPIX) {
            const int hy = hp / HWID, hx = hp - hy * HWID;
            const int iy = y0 + hy - 1, ix = x0 + hx - 1;
            if (iy >= 0 && iy < p.hi && ix >= 0 && ix < p.wi) pix = (img * p.hi + iy) * p.wi + ix;
        }
        hpix[t] = pix;
    }
    // W piece v (0..35) = tap v / 4, output channels n0 + 16 (v & 3) .. + 15 of the [cout_pad][9][cin_pad] bank
    const int wr = lane >> 2;
    const bf16_t* wsrc[WPW];
#pragma unroll
    for (int u = 0; u < WPW; ++u) {
        const int v = wave + NWAVE * u, tap = v >> 2, row = 16 * (v & 3) + wr;
        wsrc[u] = p.w + (int64_t)(n0 + row) * p.ldw + tap * p.cin_pad + (((lane & 3) ^ ((row >> 1) & 3)) * 8);
    }
    auto issue = [&](int chunk, int buf) {
        char* b = smem + buf * BUF;
#pragma unroll
        for (int t = 0; t < HPW; ++t) {
            const bf16_t* src = hpix[t] >= 0 ? p.a + (int64_t)hpix[t] * p.cin_pad + hch[t] * 8 + chunk * 32 : p.zero;
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, src), LDS_PTR(void, b + (wave + NWAVE * t) * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < WPW; ++u)
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, wsrc[u] + chunk * 32),
                                             LDS_PTR(void, b + HBYTES + (wave + NWAVE * u) * 1024), 16, 0, 0);
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int frow = lane & 15, fch = lane >> 4;
    // fragment i = tile row 4 wave + i / 2, columns 16 (i & 1) .. + 15; at tap (ty, tx) its lane's halo pixel is
    // hadr[i & 1][tx] + (i / 2 + ty) HWID 64 (see conv3x3_c32_kernel)
    uint32_t hadr[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int hx = 16 * h + frow + t;
            hadr[h][t] = (uint32_t)(uintptr_t)LDS_PTR(char, smem) + ((4 * wave) * HWID + hx) * 64 +
                         ((fch ^ h2::hkey(hx)) << 4);
        }
    const uint32_t wadr = (uint32_t)(uintptr_t)LDS_PTR(char, smem) + HBYTES + lds_off(frow, fch);

    issue(0, 0);
    for (int c = 0; c < nch; ++c) {
        const int buf = c & 1;
        if (c + 1 < nch) {
            issue(c + 1, buf ^ 1);   // lands under this chunk's MFMAs
            wait_vm<HPW + WPW>();    // this wave's pieces of chunk c landed (chunk c + 1's still in flight)
        } else {
            wait_vm<0>();
        }
        __builtin_amdgcn_s_barrier();  // every wave's pieces of chunk c landed
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t bo = buf * BUF;
        // one wave per SIMD: tap t + 1's fragments are read under tap t's MFMAs (two register sets)
        bf16x8 fa[2][8], fb[2][4];
        auto rd = [&](int tap, int s) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                fb[s][j] = *LDS_PTR(const bf16x8, (uintptr_t)(wadr + bo + tap * 4096 + j * 1024));
#pragma unroll
            for (int i = 0; i < 8; ++i)
                fa[s][i] = *LDS_PTR(const bf16x8, (uintptr_t)(hadr[i & 1][tap % 3] + bo + ((i >> 1) + tap / 3) * HWID * 64));
        };
        rd(0, 0);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int s = tap & 1;
            if (tap + 1 < 9) rd(tap + 1, s ^ 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fb[s][j]),
                                                                       __builtin_bit_cast(f16x8, fa[s][i]), acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();  // buffer `buf` is free for chunk c + 2
    }
    engine_epilogue<HkTile, E_CONV, TW, false>(p, (img * p.ho + y0) * p.wo + x0, n0, acc);
}
#endif  // RF_STUDY

// Tile configurations.  T128: 128x128, 4 waves of 64x64, 3-stage ring (48 KiB / 96 KiB LDS).
// T256: 256x256, 8 waves of 128x64, 4-stage ring (128 KiB).  T256x128: 8 waves of 64x64, bf16x3 3-stage (144 KiB).
using T128 = Tile<128, 128, 2, 2, 3>;
using T128w8 = Tile<128, 128, 2, 4, 3>;  // 8 waves of 64x32: two waves per SIMD at one block per CU
using T256 = Tile<256, 256, 2, 4, 4>;
using T256x128 = Tile<256, 128, 4, 2, 3>;
using T256x64 = Tile<256, 64, 4, 1, 4>;  // fp16 convolutions with <= 64 output channels (DPT output_conv2)
// short-M tiles for the N = 1,024 / 3,072 projections: BM chosen so the tile count fills whole rounds of
// 256 CUs (M = 5,649: 59 x 4 = 236 tiles of 96 x 256; M = 4,096: 64 x 4 = 256 tiles of 64 x 256)
using T96x256 = Tile<96, 256, 2, 4, 3>;
using T64x256 = Tile<64, 256, 2, 4, 3>;
using T64x256w4 = Tile<64, 256, 1, 4, 3>;
// deeper rings (cold weights / activations come from HBM or the MALL: more K-steps in flight per block)
using T96x256s5 = Tile<96, 256, 2, 4, 5>;
using T96x256s6 = Tile<96, 256, 2, 4, 6>;
using T64x256s6 = Tile<64, 256, 2, 4, 6>;
using T128s6 = Tile<128, 128, 2, 2, 6>;
using T128w8s6 = Tile<128, 128, 2, 4, 6>;
// 64-deep K-steps (two 32-deep planes per stage: half the barriers)
using T128k2s3 = Tile<128, 128, 2, 2, 3, 2>;
using T128k2s4 = Tile<128, 128, 2, 2, 4, 2>;
using T128w8k2s4 = Tile<128, 128, 2, 4, 4, 2>;
using T96x256k2 = Tile<96, 256, 2, 4, 3, 2>;
using T64x256k2 = Tile<64, 256, 2, 4, 3, 2>;
using T64x256w4k2 = Tile<64, 256, 1, 4, 3, 2>;
// small DPT levels (64^2 / 32^2 / 128^2 convolutions): 4 waves of 32 x 32 (64 x 64) or 32 x 64 (64 x 128) with an
// 8- / 6-deep ring, data-parallel (A/B against the stream-K 128x128 default: RF_CONV_TILE=64 / 6412)
using T64c = Tile<64, 64, 2, 2, 8>;
using T64x128c = Tile<64, 128, 2, 2, 6>;

// a_bytes: the A operand's bytes.  Past 192 MiB (3/4 of the 256 MiB Infinity Cache; config 5's W2 / larger views) A
// streams from HBM and the square
// raster below has an XCD's 32 co-running blocks on 32 different m-tiles of one n column, so every A panel is fetched
// once per n-tile; with few n-tiles (N <= 2,048) the co-running blocks instead take 32 / tiles_n m-tiles x every n
// column, and each A panel is fetched once per XCD (rf_gemm_mx8 W2 at 98,304 rows: 845 -> 748 us, the f16 engine
// 814 -> 762: profiles/r6_mx8_raster.txt)
int pick_group_m(int tiles_m, int tiles_n, int bm, int bn, int64_t per_xcd, int64_t a_bytes = 0) {
    if (const char* env = getenv("RF_GEMM_GROUP_M")) return std::max(1, std::min(tiles_m, atoi(env)));
    static const bool stream_raster = !getenv("RF_GEMM_STREAM_RASTER") || atoi(getenv("RF_GEMM_STREAM_RASTER")) != 0;
    if (stream_raster && a_bytes > (192ll << 20) && tiles_n <= 8) return std::max(1, std::min(tiles_m, 32 / tiles_n));
    const double g = std::sqrt((double)per_xcd * bn / bm);
    int gm = (int)(g + 0.5);
    gm = std::max(1, std::min(gm, tiles_m));
    if ((int64_t)gm * tiles_n < per_xcd / 2) gm = std::min<int64_t>(tiles_m, (per_xcd + tiles_n - 1) / tiles_n);
    return gm;
}

template <class C, int EPI, int NTERM, bool GATHER = false>
int launch(EngineArgs a, void* stream, const char* what) {
    const int tiles_m = (a.m + C::BM - 1) / C::BM, tiles_n = a.n / C::BN;
    const int nwg = tiles_n * tiles_m;
    a.group_m = pick_group_m(tiles_m, tiles_n, C::BM, C::BN, (nwg + 7) / 8, GATHER ? 0 : (int64_t)a.m * a.k * 2);
    RF_LAUNCH((engine_kernel<C, EPI, NTERM, GATHER, false>), dim3(nwg), dim3(C::THREADS), 0, (hipStream_t)stream,
                       a);
    return rf::check_launch(what);
}

// the halo kernel serves this convolution: 3x3, stride 1, pad 1, whole tiles of TW | wo (power of 2) x TH
template <class C>
bool halo_ok(EngineArgs& a) {
    if (a.kw != 3 || a.k != 9 * a.cin_pad || a.stride != 1 || a.pad != 1 || a.ho != a.hi || a.wo != a.wi) return false;
    if (a.cin_pad % BK || a.m % C::BM || (a.ho * a.wo) % C::BM) return false;
    const int tw = std::min(C::BM, a.wo);
    if (tw < 16 || (tw & (tw - 1)) || a.wo % tw || C::BM % tw) return false;
    const int th = C::BM / tw;
    if (a.ho % th || (th + 2) * (tw + 2) > Halo<C>::ROWS) return false;
    a.halo_lg = __builtin_ctz(tw);
    return true;
}

template <class C, int EPI>
int launch_halo(EngineArgs a, void* stream, const char* what) {
    const int tiles_m = a.m / C::BM, tiles_n = a.n / C::BN;
    const int nwg = tiles_n * tiles_m;
    a.group_m = pick_group_m(tiles_m, tiles_n, C::BM, C::BN, (nwg + 7) / 8);
    RF_LAUNCH((halo_kernel<C, EPI>), dim3(nwg), dim3(C::THREADS), 0, (hipStream_t)stream, a);
    return rf::check_launch(what);
}

// the engine's data-parallel conv launch, or the halo kernel when it serves the shape
// Measured (tools/kbench.py conv, RF_CONV_HALO): the halo kernel wins on the 4-wave 128x128 tile at large
// grids (512^2 output_conv1, 256 -> 128: 293 -> 251 us), where the gathered A re-reads dominate; on the
// 8-wave tiles it loses (128^2: 45 -> 49 us; 256^2 256x256: 123 -> 258 us, the tile spills), so by
// default only T128 uses it (RF_CONV_HALO=1: every tile that can, 0: none).
template <class C, int NTERM, bool GATHER>
int launch_conv(EngineArgs& a, void* stream, const char* what) {
    if constexpr (GATHER && NTERM == P_F16) {
        const char* env = getenv("RF_CONV_HALO");
        const bool want = env ? atoi(env) != 0 : (C::BM == 128 && C::NWAVE == 4);
        if (want && halo_ok<C>(a)) return launch_halo<C, E_CONV>(a, stream, what);
    }
    return launch<C, E_CONV, NTERM, GATHER>(a, stream, what);
}

constexpr int SK_MAX_GRID = 768;                                  // 3 blocks of T128 per CU
constexpr int64_t SK_PART_FLOATS = (int64_t)256 * 256 * 256;     // >= grid x BM x BN for every SK config
constexpr int64_t SK_WS_BYTES = SK_PART_FLOATS * 4 + SK_MAX_GRID * 4;

template <class C, int EPI, int NTERM = 1, bool GATHER = false>
int launch_sk(EngineArgs a, int grid, void* stream, const char* what) {
    const int tiles_m = (a.m + C::BM - 1) / C::BM, tiles_n = a.n / C::BN;
    a.group_m = pick_group_m(tiles_m, tiles_n, C::BM, C::BN, ((int64_t)tiles_m * tiles_n + 7) / 8);
    RF_LAUNCH((engine_kernel<C, EPI, NTERM, GATHER, true>), dim3(grid), dim3(C::THREADS), 0,
                       (hipStream_t)stream, a);
    return rf::check_launch(what);
}

// RF_OK, or RF_ERR_LAUNCH when the flag area could not be re-zeroed at an epoch wrap (the launch must not run)
int sk_setup(EngineArgs& p, void* workspace, void* stream) {
    p.sk_part = (float*)workspace;
    p.sk_flag = (int*)(p.sk_part + SK_PART_FLOATS);
    // flags from earlier launches never equal the current epoch (rf::next_epoch re-zeroes the area on a wrap)
    p.sk_epoch = rf::next_epoch(p.sk_flag, SK_MAX_GRID * sizeof(int), (hipStream_t)stream);
    if (p.sk_epoch == 0) return RF_ERR_LAUNCH;
    p.err = rf::device_error_word();
    p.spin = rf::spin_limit();
    // diagnostics: stamps in the last 256 KiB of the partial area (tools/kbench.py skstamps)
    static const bool stamps = getenv("RF_GEMM_STAMPS") && atoi(getenv("RF_GEMM_STAMPS")) != 0;
    p.stamps = stamps ? (uint64_t*)(p.sk_part + SK_PART_FLOATS - 65536) : nullptr;
    return RF_OK;
}


// Stream-K grid for the 128x128 tile, or 0 for the data-parallel launch: used when whole-tile
// rounds of 2 blocks per CU would leave >10% of the slots idle and each block keeps >= 8 K-steps.
int sk_grid(int m, int n, int k) {
    const char* env = getenv("RF_GEMM_SK");
    int grid = 2 * 256;
    if (!env) return 0;  // opt-in until validated on the GPU
    if (env) {
        grid = atoi(env);
        if (grid <= 0) return 0;
        grid = grid > SK_MAX_GRID ? SK_MAX_GRID : grid;
    }
    const int64_t tiles = (int64_t)((m + 127) / 128) * (n / 128);
    const int64_t rounds = (tiles + 511) / 512;
    const double eff = (double)tiles / (rounds * 512);
    if (!env && (eff >= 0.9 || tiles * (k / BK) < 8LL * grid)) return 0;
    return grid;
}

// Tile choice by a measured cost model (tools/kbench.py coldgemm: operands rotated over > 512 MB so every call
// reads them from HBM, as in the frame where each layer's weights are read once; profiles/r2_gemm_cold.log).
// A launch of T tiles takes ceil(T / (256 x slots)) rounds of `fixed + per_k * K/1024 (+ add)` us each, where
// `add` is the residual epilogue's cost (C tile read up front + fp32 store):
//   256   phased 256x256, 2 buffers     11.0 + 20.4   add 5
//   1282  phased 128x256, 2 buffers      2.3 + 18.4   add 5
//   964   phased  96x256, 3 buffers      6.0 + 14.4   add 5    (M = 5,649, N = 1,024: 236 tiles = one round)
//   645   phased  64x256, 3 buffers      6.5 + 11.8   add 5    (M = 4,096, N = 1,024: 256 tiles)
//   962   ring    96x256, 32-deep steps  2.2 + 16.5   add 13
//   12884 ring   128x128, 8 waves, 64-deep steps, 4 stages   6.8 + 10.9   add 5
//   128   ring   128x128, 4 waves: 5.5 + 13.1 at <= 256 tiles, else two blocks per CU 11 + 14 per 512
int pick_cfg(int m, int n, int k, int epilogue = RF_EPI_BF16) {
    if (const char* env = getenv("RF_GEMM_TILE")) return atoi(env);
    const char* ph = getenv("RF_GEMM_PHASED");
    const bool phased = n % 256 == 0 && k % 64 == 0 && (!ph || atoi(ph) != 0);
    const double kk = k / 1024.0;
    const bool add = epilogue == RF_EPI_ADD_F32;
    auto cost = [&](int bm, int bn, int slots, double fixed, double per_k, double add_cost) {
        const int64_t tiles = (int64_t)((m + bm - 1) / bm) * (n / bn);
        const int64_t rounds = (tiles + 256 * slots - 1) / (256 * slots);
        return rounds * (fixed + per_k * kk + (add ? add_cost : 0.0));
    };
    int best = 128;
    const int64_t t128 = (int64_t)((m + 127) / 128) * (n / 128);
    double best_c = t128 <= 256 ? cost(128, 128, 1, 5.5, 13.1, 5.0) : cost(128, 128, 2, 11.0, 14.0, 5.0);
    auto consider = [&](int cfg, double c) {
        if (c < best_c) {
            best_c = c;
            best = cfg;
        }
    };
    if (k % 64 == 0) consider(12884, cost(128, 128, 1, 6.8, 10.9, 5.0));
    if (n % 256 == 0) consider(962, cost(96, 256, 1, 2.2, 16.5, 13.0));
    if (phased) {
        consider(256, cost(256, 256, 1, 11.0, 20.4, 5.0));
        consider(1282, cost(128, 256, 1, 2.3, 18.4, 5.0));
        consider(964, cost(96, 256, 1, 6.0, 14.4, 5.0));
        consider(645, cost(64, 256, 1, 6.5, 11.8, 5.0));
    }
    return best;
}

__device__ __attribute__((aligned(16))) bf16_t g_zero_row[64];  // stays zero: source of padded conv taps

// ---------------------------------------------------------------------------------------------
// MX fp8 GEMM (OCP e4m3 operands, one E8M0 scale per 32 K-elements of every row, fp32 accumulate) on the
// block-scaled v_mfma_scale_f32_16x16x128_f8f6f4: twice the bf16 MFMA rate.  C[M,N] (epilogue) A[M,K] W[N,K]^T
// with A = a * 2^(sa - 127), W = w * 2^(sw - 127) blockwise.  Tile 256x256, 8 waves of 128x64 (8 x 4 MFMAs of
// 16x16x128 per 128-deep K-step), 2-stage LDS ring filled by LDS-DMA: operand rows of 128 B with the 16-B
// chunk index XOR (row & 7) (pre-swizzled source address, the same XOR on the read), and the step's scale
// dwords (4 blocks per row) staged beside them.  Lane l holds row l & 15 (see below for its K bytes); the W
// fragment is the instruction's first operand, so each lane's accumulator holds 4 consecutive output columns
// of one row, as in the bf16 engine (engine_epilogue applies unchanged).  Measured K map (tools/fp8_probe.py,
// structured data): the 16-B halves h = 0, 1 of lane group g = lane >> 4 are K elements 64 h + 16 g .. +15,
// and the scale operand of lane group b scales K block b (elements 32 b .. 32 b + 31) — so a lane reads its
// row's 16-B chunks g and g + 4 and passes the scale byte of block g.
namespace mx {
constexpr int BM = 256, BN = 256, KS = 128;  // KS: K bytes (= elements) per step
constexpr int A_DATA = BM * KS, B_DATA = BN * KS;
constexpr int STAGE = A_DATA + B_DATA + (BM + BN) * 4;
constexpr int TI = 8, TJ = 4;
typedef __attribute__((ext_vector_type(8))) int i32x8;
RF_DEV int off(int row, int ch) { return row * KS + ((ch ^ (row & 7)) << 4); }
}  // namespace mx

template <bool INITC>
RF_DEV void mx8_mainloop(const EngineArgs& p, char* smem, int m0, int n0, int kbeg, int kend,
                         f32x4 (&acc)[mx::TI][mx::TJ]) {
    using namespace mx;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const int nk = kend - kbeg;
    const uint8_t* A = reinterpret_cast<const uint8_t*>(p.a);
    const uint8_t* W = reinterpret_cast<const uint8_t*>(p.w);
    // data pieces: 8 rows x 128 B per wave-instruction; pieces 0..31 = A, 32..63 = W; 8 per wave
    auto issue = [&](int kt, int buf) {
        char* st = smem + buf * STAGE;
        const int64_t k0 = (int64_t)(kbeg + kt) * KS;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int piece = wave * 8 + i;
            const bool is_a = piece < BM / 8;
            const int row = (is_a ? piece : piece - BM / 8) * 8 + (lane >> 3);
            const int ch = (lane & 7) ^ (row & 7);  // logical chunk landing at physical chunk lane & 7
            const uint8_t* src;
            if (is_a) {
                const int m = m0 + row;
                src = A + (int64_t)(m < p.m ? m : p.m - 1) * p.lda + k0 + ch * 16;
            } else {
                src = W + (int64_t)(n0 + row) * p.ldw + k0 + ch * 16;
            }
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, src), LDS_PTR(void, st + (is_a ? 0 : A_DATA) + piece % (BM / 8) * 1024),
                                             16, 0, 0);
        }
        // scales: wave w < 4 stages A rows 64 w + lane, waves 4..7 W rows 64 (w - 4) + lane (one dword each)
        {
            const bool is_a = wave < BM / 64;
            const int row = (is_a ? wave : wave - BM / 64) * 64 + lane;
            const uint8_t* src;
            if (is_a) {
                const int m = m0 + row;
                src = p.sa + (int64_t)(m < p.m ? m : p.m - 1) * p.ld_sa + (kbeg + kt) * 4;
            } else {
                src = p.sw + (int64_t)(n0 + row) * p.ld_sw + (kbeg + kt) * 4;
            }
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, src),
                                             LDS_PTR(void, st + A_DATA + B_DATA + (is_a ? 0 : BM * 4) + (row & ~63) * 4),
                                             4, 0, 0);
        }
    };
    if (INITC && kbeg == 0) {
        load_c_acc<TI, TJ>(p, m0 + wm * 128, n0 + wn * 64, acc);
    } else {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int frow = lane & 15, g = lane >> 4;
    issue(0, 0);
    if (nk > 1) {
        issue(1, 1);
        wait_vm<9>();
    } else {
        wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < nk; ++kt) {
        const char* st = smem + (kt & 1) * STAGE;
        const int* sca = reinterpret_cast<const int*>(st + A_DATA + B_DATA);
        const int* scw = sca + BM;
        i32x8 fa[TI], fw[TJ];
        int sa[TI], sw[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const int row = wm * 128 + i * 16 + frow;
            const u32x4 lo = *reinterpret_cast<const u32x4*>(st + off(row, g));
            const u32x4 hi = *reinterpret_cast<const u32x4*>(st + off(row, g + 4));
            fa[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
            sa[i] = (sca[row] >> (8 * g)) & 0xff;
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            const int row = wn * 64 + j * 16 + frow;
            const u32x4 lo = *reinterpret_cast<const u32x4*>(st + A_DATA + off(row, g));
            const u32x4 hi = *reinterpret_cast<const u32x4*>(st + A_DATA + off(row, g + 4));
            fw[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
            sw[j] = (scw[row] >> (8 * g)) & 0xff;
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fw[j], fa[i], acc[i][j], 0, 0, 0, sw[j], 0,
                                                                             sa[i]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // (every read of stage kt & 1 retired)
        __builtin_amdgcn_s_barrier();
        if (kt + 2 < nk) {
            issue(kt + 2, kt & 1);
            wait_vm<9>();
        } else {
            wait_vm<0>();
        }
        __builtin_amdgcn_s_barrier();
    }
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void mx8_kernel(EngineArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[2 * mx::STAGE];
    const int tiles_m = (p.m + mx::BM - 1) / mx::BM;
    const int nwg = gridDim.x;
    const int hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    int tm, tn;
    tile_coords(wg, tiles_m, p.n / mx::BN, p.group_m, tm, tn);
    f32x4 acc[mx::TI][mx::TJ];
    mx8_mainloop<EPI == E_ADD>(p, smem, tm * mx::BM, tn * mx::BN, 0, p.k / mx::KS, acc);
    engine_epilogue<Tile<256, 256, 2, 4, 4>, EPI>(p, tm * mx::BM, tn * mx::BN, acc);
}

// Staggered three-buffer MX fp8 loop (the default): tile 128 x 256, 8 waves of 64 x 64 (4 x 4 MFMAs of
// 16x16x128 per 128-deep K-step), one load section {ds_read this step's fragments and scales; issue step t+2's
// LDS-DMA into the buffer step t-1 used; counted vmcnt for step t+1} and one MFMA section per step, waves 4-7
// one section behind (on every SIMD one wave's reads overlap its partner's MFMAs), three 49.5-KiB buffers so
// every DMA has a whole step of both groups' MFMA work to land under (the plain loop above reads, then
// computes: the MFMA pipe idles during every read burst).
namespace mx3 {
constexpr int BM = 128, BN = 256, KS = 128;
constexpr int A_DATA = BM * KS, B_DATA = BN * KS;
constexpr int STAGE = A_DATA + B_DATA + (BM + BN) * 4;
constexpr int TI = 4, TJ = 4;
}  // namespace mx3

template <bool INITC>
RF_DEV void mx8_p3_mainloop(const EngineArgs& p, char* smem, int m0, int n0, int kbeg, int kend,
                            f32x4 (&acc)[mx3::TI][mx3::TJ]) {
    using namespace mx3;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const int nk = kend - kbeg;
    const uint8_t* A = reinterpret_cast<const uint8_t*>(p.a);
    const uint8_t* W = reinterpret_cast<const uint8_t*>(p.w);
    const bool has_sc = __builtin_amdgcn_readfirstlane(wave) < (BM + BN) / 64;  // waves 0-5 stage a scale piece
    auto issue = [&](int kt) {
        char* st = smem + (kt % 3) * STAGE;
        const int64_t k0 = (int64_t)(kbeg + kt) * KS;
#pragma unroll
        for (int i = 0; i < 6; ++i) {  // 48 data pieces of 8 rows x 128 B: 0..15 A, 16..47 W
            const int piece = wave * 6 + i;
            const bool is_a = piece < BM / 8;
            const int row = (is_a ? piece : piece - BM / 8) * 8 + (lane >> 3);
            const int ch = (lane & 7) ^ (row & 7);
            const uint8_t* src;
            if (is_a) {
                const int m = m0 + row;
                src = A + (int64_t)(m < p.m ? m : p.m - 1) * p.lda + k0 + ch * 16;
            } else {
                src = W + (int64_t)(n0 + row) * p.ldw + k0 + ch * 16;
            }
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, src),
                                             LDS_PTR(void, st + (is_a ? piece * 1024 : A_DATA + (piece - BM / 8) * 1024)),
                                             16, 0, 0);
        }
        if (has_sc) {  // scale dwords: waves 0-1 A rows 64 w + lane, waves 2-5 W rows 64 (w - 2) + lane
            const bool is_a = wave < BM / 64;
            const int row = (is_a ? wave : wave - BM / 64) * 64 + lane;
            const uint8_t* src;
            if (is_a) {
                const int m = m0 + row;
                src = p.sa + (int64_t)(m < p.m ? m : p.m - 1) * p.ld_sa + (kbeg + kt) * 4;
            } else {
                src = p.sw + (int64_t)(n0 + row) * p.ld_sw + (kbeg + kt) * 4;
            }
            __builtin_amdgcn_global_load_lds(GLB_PTR(void, src),
                                             LDS_PTR(void, st + A_DATA + B_DATA + (is_a ? 0 : BM * 4) + (row & ~63) * 4),
                                             4, 0, 0);
        }
    };
    if (INITC && kbeg == 0) {
        load_c_acc<TI, TJ>(p, m0 + wm * 64, n0 + wn * 64, acc);
    } else {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int frow = lane & 15, g = lane >> 4;
    issue(0);
    if (nk > 1) {
        issue(1);
        if (has_sc) wait_vm<7>();
        else wait_vm<6>();
    } else {
        wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const bool late = __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256;
    if (late) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    mx::i32x8 fa[TI], fw[TJ];
    int sa[TI], sw[TJ];
    for (int kt = 0; kt < nk; ++kt) {
        const char* st = smem + (kt % 3) * STAGE;
        const int* sca = reinterpret_cast<const int*>(st + A_DATA + B_DATA);
        const int* scw = sca + BM;
        // ---- load section
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const int row = wm * 64 + i * 16 + frow;
            const u32x4 lo = *reinterpret_cast<const u32x4*>(st + mx::off(row, g));
            const u32x4 hi = *reinterpret_cast<const u32x4*>(st + mx::off(row, g + 4));
            fa[i] = mx::i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
            sa[i] = (sca[row] >> (8 * g)) & 0xff;
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            const int row = wn * 64 + j * 16 + frow;
            const u32x4 lo = *reinterpret_cast<const u32x4*>(st + A_DATA + mx::off(row, g));
            const u32x4 hi = *reinterpret_cast<const u32x4*>(st + A_DATA + mx::off(row, g + 4));
            fw[j] = mx::i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
            sw[j] = (scw[row] >> (8 * g)) & 0xff;
        }
        if (kt + 2 < nk) {
            issue(kt + 2);
            if (has_sc) wait_vm<7>();  // step kt+1 landed (this wave's part), step kt+2 in flight
            else wait_vm<6>();
        } else {
            wait_vm<0>();
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        // ---- MFMA section
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fw[j], fa[i], acc[i][j], 0, 0, 0, sw[j], 0,
                                                                             sa[i]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    }
    if (!late) __builtin_amdgcn_s_barrier();
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void mx8_p3_kernel(EngineArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[3 * mx3::STAGE];
    const int tiles_m = (p.m + mx3::BM - 1) / mx3::BM;
    const int nwg = gridDim.x;
    const int hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    int tm, tn;
    tile_coords(wg, tiles_m, p.n / mx3::BN, p.group_m, tm, tn);
    f32x4 acc[mx3::TI][mx3::TJ];
    mx8_p3_mainloop<EPI == E_ADD>(p, smem, tm * mx3::BM, tn * mx3::BN, 0, p.k / mx3::KS, acc);
    engine_epilogue<Tile<128, 256, 2, 4, 4>, EPI>(p, tm * mx3::BM, tn * mx3::BN, acc);
}

// MX quantisation of bf16 rows: every 32-element block gets the E8M0 scale 2^e with e = ceil(log2(amax / 448))
// (the block's largest |value| lands in (224, 448], never saturating e4m3), values x / 2^e rounded to nearest
// even e4m3 (hardware v_cvt_pk_fp8_f32).  One thread per block: 64 B in, 32 B + 1 scale byte out.
__global__ __launch_bounds__(256) void quant_mx8_kernel(const bf16_t* __restrict__ x, int64_t ldx, int rows, int cols,
                                                        uint8_t* __restrict__ q, int64_t ldq, uint8_t* __restrict__ sc,
                                                        int64_t lds) {
    const int nb = cols / 32;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)rows * nb) return;
    const int row = (int)(t / nb), b = (int)(t % nb);
    const uint4* src = reinterpret_cast<const uint4*>(x + (int64_t)row * ldx + b * 32);
    float v[32];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint4 u = src[i];
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            v[i * 8 + 2 * e] = __uint_as_float(w[e] << 16);
            v[i * 8 + 2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
        }
    }
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) amax = fmaxf(amax, fabsf(v[i]));
    int e = -127;
    if (amax > 0.f) {
        // smallest e with amax / 2^e <= 448: frexp gives amax = f 2^x (f in [0.5, 1)); 448 = 0.875 2^9
        int ex;
        const float f = frexpf(amax, &ex);
        e = ex - 9 + (f > 0.875f ? 1 : 0);
        e = e < -127 ? -127 : (e > 127 ? 127 : e);
    }
    const float inv = ldexpf(1.0f, -e);
    uint32_t out[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        int pk = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i] * inv, v[4 * i + 1] * inv, 0, false);
        pk = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i + 2] * inv, v[4 * i + 3] * inv, pk, true);
        out[i] = (uint32_t)pk;
    }
    uint4* dst = reinterpret_cast<uint4*>(q + (int64_t)row * ldq + b * 32);
    dst[0] = make_uint4(out[0], out[1], out[2], out[3]);
    dst[1] = make_uint4(out[4], out[5], out[6], out[7]);
    sc[(int64_t)row * lds + b] = (uint8_t)(e + 127);
}

}  // namespace

// Persistent 256x256 phased launches (RF_GEMM_PERSIST=0 turns them off): more than one round of tiles runs as
// one block per CU looping over whole tiles, each block prefetching its next tile's first K-tiles before the
// current tile's epilogue (phased_sk_kernel, p.persist) instead of one block per tile.
bool persist_on() {
    static const bool on = !getenv("RF_GEMM_PERSIST") || atoi(getenv("RF_GEMM_PERSIST")) != 0;
    return on;
}

// A tile count that is not a whole number of 256-block rounds (the stage-1 SwiGLU W13: 736 tiles) runs one block per
// tile by default: the persistent kernel's last round is as ragged as the hardware dispatcher's, and its cross-tile
// prefetch costs registers (phased_sk_kernel spills at 256 VGPRs, phased_kernel<256> does not).  RF_GEMM_PERSIST_RAGGED=1
// restores the persistent launch there (A/B: profiles/r6_w13_persist_ab.txt).
bool persist_ragged() {
    static const bool on = getenv("RF_GEMM_PERSIST_RAGGED") && atoi(getenv("RF_GEMM_PERSIST_RAGGED")) != 0;
    return on;
}

template <int EPI, int NTERM, bool GATHER, int BM = 256>
int launch_phased(EngineArgs a, void* stream, const char* what) {
    const int tiles_m = (a.m + BM - 1) / BM, tiles_n = a.n / 256;
    const int nwg = tiles_n * tiles_m;
    a.group_m = pick_group_m(tiles_m, tiles_n, BM, 256, (nwg + 7) / 8, GATHER ? 0 : (int64_t)a.m * a.k * 2);
    if constexpr (BM == 256 && (NTERM == 1 || NTERM == P_F16) && !GATHER) {
        if (nwg > 256 && persist_on() && (nwg % 256 == 0 || persist_ragged())) {
            a.persist = 1;
            RF_LAUNCH((phased_sk_kernel<EPI, NTERM>), dim3(256), dim3(512), 0, (hipStream_t)stream, a);
            return rf::check_launch(what);
        }
    }
    RF_LAUNCH((phased_kernel<BM, EPI, NTERM, GATHER>), dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    return rf::check_launch(what);
}

#ifdef RF_STUDY
// phased3 loop's L2 run-ahead distance (K-tiles; 0 = off): RF_GEMM_L2PF (study build)
int l2pf_dist() {
    const char* env = getenv("RF_GEMM_L2PF");
    return env ? std::max(0, std::min(8, atoi(env))) : 0;
}
#endif

template <int EPI, int BM, int NT = 1>
int launch_phased3(EngineArgs a, void* stream, const char* what) {
#ifdef RF_STUDY
    a.l2pf = l2pf_dist();
#endif
    const int tiles_m = (a.m + BM - 1) / BM, tiles_n = a.n / 256;
    const int nwg = tiles_n * tiles_m;
    a.group_m = pick_group_m(tiles_m, tiles_n, BM, 256, (nwg + 7) / 8, (int64_t)a.m * a.k * 2);
    RF_LAUNCH((phased3_kernel<BM, EPI, NT>), dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    return rf::check_launch(what);
}

template <int BM, int NT = 1>
int run_phased3(const EngineArgs& p, int epilogue, void* stream) {
    switch (epilogue) {
        case RF_EPI_BF16: return launch_phased3<E_BF16, BM, NT>(p, stream, "rf_gemm");
        case RF_EPI_F32: return launch_phased3<E_F32, BM, NT>(p, stream, "rf_gemm");
        case RF_EPI_ADD_F32: return launch_phased3<E_ADD, BM, NT>(p, stream, "rf_gemm");
        default: return launch_phased3<E_SWIGLU, BM, NT>(p, stream, "rf_gemm");
    }
}

template <int EPI, int NT = 1>
int launch_phased_sk(EngineArgs a, int grid, void* stream, const char* what) {
    const int tiles_m = (a.m + 255) / 256, tiles_n = a.n / 256;
    a.group_m = pick_group_m(tiles_m, tiles_n, 256, 256, ((int64_t)tiles_m * tiles_n + 7) / 8);
    RF_LAUNCH((phased_sk_kernel<EPI, NT>), dim3(grid), dim3(512), 0, (hipStream_t)stream, a);
    return rf::check_launch(what);
}

// the phased 256x256 loop replaces the ring engine's 256x256 tile (RF_GEMM_PHASED=0 restores it)
bool use_phased(int n, int k) {
    const char* env = getenv("RF_GEMM_PHASED");
    return (!env || atoi(env) != 0) && n % 256 == 0 && k % 64 == 0;
}

template <class C, int NT = 1>
int run_dp_cfg(const EngineArgs& p, int epilogue, void* stream) {
    switch (epilogue) {
        case RF_EPI_BF16: return launch<C, E_BF16, NT>(p, stream, "rf_gemm");
        case RF_EPI_F32: return launch<C, E_F32, NT>(p, stream, "rf_gemm");
        case RF_EPI_ADD_F32: return launch<C, E_ADD, NT>(p, stream, "rf_gemm");
        default: return launch<C, E_SWIGLU, NT>(p, stream, "rf_gemm");
    }
}

// fp16 operands (rf_gemm_f16): the loops pick_cfg chooses from, each with fp16 MFMAs (same rate as bf16)
int run_dp_f16(int cfg, const EngineArgs& p, int epilogue, void* stream) {
    constexpr int NT = P_F16;
    if (use_phased(p.n, p.k)) {
        if (cfg == 256) {
            switch (epilogue) {
                case RF_EPI_BF16: return launch_phased<E_BF16, NT, false>(p, stream, "rf_gemm_f16");
                case RF_EPI_F32: return launch_phased<E_F32, NT, false>(p, stream, "rf_gemm_f16");
                case RF_EPI_ADD_F32: return launch_phased<E_ADD, NT, false>(p, stream, "rf_gemm_f16");
                default: return launch_phased<E_SWIGLU, NT, false>(p, stream, "rf_gemm_f16");
            }
        }
        if (cfg == 1282) {
            switch (epilogue) {
                case RF_EPI_BF16: return launch_phased<E_BF16, NT, false, 128>(p, stream, "rf_gemm_f16");
                case RF_EPI_F32: return launch_phased<E_F32, NT, false, 128>(p, stream, "rf_gemm_f16");
                case RF_EPI_ADD_F32: return launch_phased<E_ADD, NT, false, 128>(p, stream, "rf_gemm_f16");
                default: return launch_phased<E_SWIGLU, NT, false, 128>(p, stream, "rf_gemm_f16");
            }
        }
        if (cfg == 1283) return run_phased3<128, NT>(p, epilogue, stream);
        if (cfg == 964) return run_phased3<96, NT>(p, epilogue, stream);
        if (cfg == 645) return run_phased3<64, NT>(p, epilogue, stream);
    }
    if (cfg == 962 && p.n % 256 == 0) return run_dp_cfg<T96x256, NT>(p, epilogue, stream);
    if (cfg == 12884 && p.k % 64 == 0) return run_dp_cfg<T128w8k2s4, NT>(p, epilogue, stream);
    return run_dp_cfg<T128, NT>(p, epilogue, stream);
}

// cfg codes: 128 = T128, 256 = T256 (needs N % 256 == 0), 1284 / 1285 = 128x128 with a 4 / 5-stage ring,
// 2561 = 256x128 (8 waves)
int run_dp(int cfg, const EngineArgs& p, int epilogue, void* stream) {
    if (cfg == 256 && use_phased(p.n, p.k)) {
        switch (epilogue) {
            case RF_EPI_BF16: return launch_phased<E_BF16, 1, false>(p, stream, "rf_gemm_bf16");
            case RF_EPI_F32: return launch_phased<E_F32, 1, false>(p, stream, "rf_gemm_bf16");
            case RF_EPI_ADD_F32: return launch_phased<E_ADD, 1, false>(p, stream, "rf_gemm_bf16");
            default: return launch_phased<E_SWIGLU, 1, false>(p, stream, "rf_gemm_bf16");
        }
    }
    if (cfg == 1282 && use_phased(p.n, p.k)) {
        switch (epilogue) {
            case RF_EPI_BF16: return launch_phased<E_BF16, 1, false, 128>(p, stream, "rf_gemm_bf16");
            case RF_EPI_F32: return launch_phased<E_F32, 1, false, 128>(p, stream, "rf_gemm_bf16");
            case RF_EPI_ADD_F32: return launch_phased<E_ADD, 1, false, 128>(p, stream, "rf_gemm_bf16");
            default: return launch_phased<E_SWIGLU, 1, false, 128>(p, stream, "rf_gemm_bf16");
        }
    }
    if (cfg == 256 && p.n % 256 == 0) return run_dp_cfg<T256>(p, epilogue, stream);
    if (cfg == 1284) return run_dp_cfg<Tile<128, 128, 2, 2, 4>>(p, epilogue, stream);
    if (cfg == 1285) return run_dp_cfg<Tile<128, 128, 2, 2, 5>>(p, epilogue, stream);
    if (cfg == 2561) return run_dp_cfg<T256x128>(p, epilogue, stream);
    if (cfg == 962 && p.n % 256 == 0) return run_dp_cfg<T96x256>(p, epilogue, stream);
    if (cfg == 642 && p.n % 256 == 0) return run_dp_cfg<T64x256>(p, epilogue, stream);
    if (use_phased(p.n, p.k)) {  // three-buffer phased short tiles
        if (cfg == 1283) return run_phased3<128>(p, epilogue, stream);
        if (cfg == 964) return run_phased3<96>(p, epilogue, stream);
        if (cfg == 645) return run_phased3<64>(p, epilogue, stream);
    }
    if (cfg == 963 && use_phased(p.n, p.k)) {  // phased 96x256
        switch (epilogue) {
            case RF_EPI_BF16: return launch_phased<E_BF16, 1, false, 96>(p, stream, "rf_gemm_bf16");
            case RF_EPI_F32: return launch_phased<E_F32, 1, false, 96>(p, stream, "rf_gemm_bf16");
            case RF_EPI_ADD_F32: return launch_phased<E_ADD, 1, false, 96>(p, stream, "rf_gemm_bf16");
            default: return launch_phased<E_SWIGLU, 1, false, 96>(p, stream, "rf_gemm_bf16");
        }
    }
    if (cfg == 643 && use_phased(p.n, p.k)) {  // phased 64x256
        switch (epilogue) {
            case RF_EPI_BF16: return launch_phased<E_BF16, 1, false, 64>(p, stream, "rf_gemm_bf16");
            case RF_EPI_F32: return launch_phased<E_F32, 1, false, 64>(p, stream, "rf_gemm_bf16");
            case RF_EPI_ADD_F32: return launch_phased<E_ADD, 1, false, 64>(p, stream, "rf_gemm_bf16");
            default: return launch_phased<E_SWIGLU, 1, false, 64>(p, stream, "rf_gemm_bf16");
        }
    }
    if (cfg == 644 && p.n % 256 == 0) return run_dp_cfg<T64x256w4>(p, epilogue, stream);
    if (cfg == 965 && p.n % 256 == 0) return run_dp_cfg<T96x256s5>(p, epilogue, stream);
    if (cfg == 966 && p.n % 256 == 0) return run_dp_cfg<T96x256s6>(p, epilogue, stream);
    if (cfg == 646 && p.n % 256 == 0) return run_dp_cfg<T64x256s6>(p, epilogue, stream);
    if (cfg == 1286) return run_dp_cfg<T128s6>(p, epilogue, stream);
    if (cfg == 1288) return run_dp_cfg<T128w8s6>(p, epilogue, stream);
    if (p.k % 64 == 0) {
        if (cfg == 12823) return run_dp_cfg<T128k2s3>(p, epilogue, stream);
        if (cfg == 12824) return run_dp_cfg<T128k2s4>(p, epilogue, stream);
        if (cfg == 12884) return run_dp_cfg<T128w8k2s4>(p, epilogue, stream);
        if (cfg == 9623 && p.n % 256 == 0) return run_dp_cfg<T96x256k2>(p, epilogue, stream);
        if (cfg == 6423 && p.n % 256 == 0) return run_dp_cfg<T64x256k2>(p, epilogue, stream);
        if (cfg == 6443 && p.n % 256 == 0) return run_dp_cfg<T64x256w4k2>(p, epilogue, stream);
    }
    return run_dp_cfg<T128>(p, epilogue, stream);
}

bool sk256(int m, int n, int k) {
    if (const char* env = getenv("RF_GEMM_SK256")) return atoi(env) != 0;
    return false;  // the ring engine's 256x256 stream-K: superseded by the phased one, kept for A/B
}

// Phased 256x256 stream-K over one block per CU (RF_GEMM_SKPH=1/0 forces it on/off).  With partial tiles
// its fix-up costs ~5-10 us per block, and the 128x256 phased tile beat it on every such shape measured
// (texture GEMM 5633x1024x13312: 170 us vs 212 us); when the tile count is a multiple of the 256-block
// grid every block runs whole tiles back to back (no fix-up) and it beats the data-parallel launch
// (stage-2 W13 4096x8192x1024: 68 vs 72.5 us), so that case is the default.
bool skph(int m, int n, int k) {
    if (!use_phased(n, k)) return false;
    if (const char* env = getenv("RF_GEMM_SKPH")) return atoi(env) != 0;
    const int64_t tiles = (int64_t)((m + 255) / 256) * (n / 256);
    return n % 256 == 0 && tiles >= 512 && tiles % 256 == 0;
}

extern "C" int64_t rf_gemm_workspace_bytes(void) { return SK_WS_BYTES; }

#ifdef RF_STUDY  // the 4-wave GEMM (measured slower than the 8-wave engine): study build only
// The 4-wave engine (quad_kernel).  RF_GEMM_QUAD (read per call, for A/B in one process): 0 = off, 1 = data-
// parallel / persistent over whole tiles, 2 = stream-K over 256 blocks in pairs of K-tiles.  RF_GEMM_QUAD_TILE
// picks the block tile (BM x BN): 256x256 (default; 128 x 128 per wave), 192x256, 160x256, 128x192, 128x128.
// Needs K % 128 == 0, a column-tile multiple of N for the SwiGLU epilogue, and operands addressable by 32-bit
// buffer offsets.
static int quad_tile() {
    const char* env = getenv("RF_GEMM_QUAD_TILE");
    if (!env) return 256256;
    int bm = 0, bn = 0;
    if (sscanf(env, "%dx%d", &bm, &bn) != 2) return 256256;
    return bm * 1000 + bn;
}

static int quad_mode(int m, int n, int k, int64_t lda, int64_t ldw, int epilogue) {
    const char* env = getenv("RF_GEMM_QUAD");
    const int mode = env ? atoi(env) : 0;
    if (mode <= 0 || k % 128 || m <= 0) return 0;  // (the loop runs whole pairs of 64-deep K-tiles)
    const int t = quad_tile(), bn = t % 1000;
    if (bn != 256 && bn != 192 && bn != 128) return 0;
    if (epilogue == RF_EPI_SWIGLU && n % bn) return 0;
    if ((int64_t)m * lda * 2 >= 0x7fffffff || (int64_t)n * ldw * 2 >= 0x7fffffff) return 0;
    return mode;
}

template <int WM, int WN, int EPI, int NT, int STG>
static int launch_quad_s(EngineArgs a, int mode, void* workspace, int64_t ws_bytes, void* stream, const char* what);

template <int WM, int WN, int EPI, int NT>
static int launch_quad(EngineArgs a, int mode, void* workspace, int64_t ws_bytes, void* stream, const char* what) {
    // RF_GEMM_QUAD_STG: 0 = LDS-DMA (default), 1 = register staging.  Measured (profiles/r4_quad_reg_study.txt):
    // staging a 64-deep K-tile through registers costs 64 VGPRs a lane at 256x256, which the 256 accumulator
    // AGPRs leave no room for; the loop spills and runs 2-3x slower than the DMA form.
    const char* stg_env = getenv("RF_GEMM_QUAD_STG");
    if (stg_env && atoi(stg_env) == 1) return launch_quad_s<WM, WN, EPI, NT, 1>(a, mode, workspace, ws_bytes, stream, what);
    return launch_quad_s<WM, WN, EPI, NT, 0>(a, mode, workspace, ws_bytes, stream, what);
}

template <int WM, int WN, int EPI, int NT, int STG>
static int launch_quad_s(EngineArgs a, int mode, void* workspace, int64_t ws_bytes, void* stream, const char* what) {
    using G = qd::Cfg<WM, WN>;
    const int tiles_m = (a.m + G::BM - 1) / G::BM, tiles_n = (a.n + G::BN - 1) / G::BN;
    const int64_t tiles = (int64_t)tiles_m * tiles_n;
    const int grid = (int)std::min<int64_t>(tiles, 256);
    a.group_m = pick_group_m(tiles_m, tiles_n, G::BM, G::BN, (grid + 7) / 8);
    if (mode == 2 && workspace && ws_bytes >= SK_WS_BYTES) {
        if (const int rc = sk_setup(a, workspace, stream)) return rc;
        RF_LAUNCH((quad_kernel<WM, WN, EPI, NT, STG>), dim3(256), dim3(256), 0, (hipStream_t)stream, a);
    } else {
        a.sk_flag = nullptr;
        RF_LAUNCH((quad_kernel<WM, WN, EPI, NT, STG>), dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    }
    return rf::check_launch(what);
}

template <int WM, int WN, int NT>
static int run_quad_t(const EngineArgs& p, int epilogue, int mode, void* workspace, int64_t ws_bytes, void* stream,
                      const char* what) {
    switch (epilogue) {
        case RF_EPI_BF16: return launch_quad<WM, WN, E_BF16, NT>(p, mode, workspace, ws_bytes, stream, what);
        case RF_EPI_F32: return launch_quad<WM, WN, E_F32, NT>(p, mode, workspace, ws_bytes, stream, what);
        case RF_EPI_ADD_F32: return launch_quad<WM, WN, E_ADD, NT>(p, mode, workspace, ws_bytes, stream, what);
        default: return launch_quad<WM, WN, E_SWIGLU, NT>(p, mode, workspace, ws_bytes, stream, what);
    }
}

template <int NT>
static int run_quad(const EngineArgs& p, int epilogue, int mode, void* workspace, int64_t ws_bytes, void* stream,
                    const char* what) {
    switch (quad_tile()) {
        case 192256: return run_quad_t<96, 128, NT>(p, epilogue, mode, workspace, ws_bytes, stream, what);
        case 160256: return run_quad_t<80, 128, NT>(p, epilogue, mode, workspace, ws_bytes, stream, what);
        case 128192: return run_quad_t<64, 96, NT>(p, epilogue, mode, workspace, ws_bytes, stream, what);
        case 128128: return run_quad_t<64, 64, NT>(p, epilogue, mode, workspace, ws_bytes, stream, what);
        default: return run_quad_t<128, 128, NT>(p, epilogue, mode, workspace, ws_bytes, stream, what);
    }
}
#endif  // RF_STUDY

// the deferred-RMSNorm operands of one GEMM (rf_gemm_add_prenorm: xg / norm_g / ss_out; rf_gemm_rownorm: rs_*)
struct NormIO {
    void* xg = nullptr;
    int64_t ldxg = 0;
    const float* norm_g = nullptr;
    float* ss_out = nullptr;
    int xg_f16 = 0;
    const float* rs_part = nullptr;
    float rs_n = 0.f, rs_eps = 0.f;
    float* seg_ss = nullptr;
    int seg_w = 0, seg_n = 0;
};

static int gemm_bf16(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc,
                     const float* bias, int m, int n, int k, int epilogue, void* workspace, int64_t ws_bytes,
                     void* stream, const int* gate, bool f16 = false, const NormIO* nio = nullptr) {
    RF_REQUIRE(a && w && c, "rf_gemm_bf16: null pointer");
    int out_f16 = 0;
    if (epilogue == RF_EPI_F16 || epilogue == RF_EPI_SWIGLU_F16) {  // fp16 16-bit outputs
        out_f16 = 1;
        epilogue = epilogue == RF_EPI_F16 ? RF_EPI_BF16 : RF_EPI_SWIGLU;
    }
    RF_REQUIRE(m > 0 && n > 0 && k > 0, "rf_gemm_bf16: empty problem m=%d n=%d k=%d", m, n, k);
    RF_REQUIRE(k % BK == 0, "rf_gemm_bf16: K=%d must be a multiple of %d", k, BK);
    RF_REQUIRE(n % 128 == 0, "rf_gemm_bf16: N=%d must be a multiple of 128", n);
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
    p.gate = gate;
    p.out_f16 = out_f16;
    p.range = out_f16 ? rf::range_word() : nullptr;
    if (nio) {
        p.xg = (bf16_t*)nio->xg;
        p.ldxg = nio->ldxg;
        p.norm_g = nio->norm_g;
        p.ss_out = nio->ss_out;
        p.xg_f16 = nio->xg_f16;
        p.rs_part = nio->rs_part;
        p.rs_n = nio->rs_n;
        p.rs_eps = nio->rs_eps;
        p.seg_ss = nio->seg_ss;
        p.seg_w = nio->seg_w;
        p.seg_n = nio->seg_n;
        if (nio->xg && nio->xg_f16) p.range = rf::range_word();
    }
#ifdef RF_STUDY
    if (const int qm = nio ? 0 : quad_mode(m, n, k, lda, ldw, epilogue)) {  // (the 4-wave epilogue has no norm I/O)
        return f16 ? run_quad<P_F16>(p, epilogue, qm, workspace, ws_bytes, stream, "rf_gemm_f16")
                   : run_quad<1>(p, epilogue, qm, workspace, ws_bytes, stream, "rf_gemm_bf16");
    }
#else
    if (getenv("RF_GEMM_QUAD") && atoi(getenv("RF_GEMM_QUAD")) > 0) return rf::study_only("rf_gemm: RF_GEMM_QUAD");
#endif
    if (workspace && ws_bytes >= SK_WS_BYTES && skph(m, n, k)) {
        if (const int rc = sk_setup(p, workspace, stream)) return rc;
        const int64_t tiles = (int64_t)((m + 255) / 256) * (n / 256);
        p.persist = tiles % 256 == 0 && persist_on();  // whole tiles per block either way: prefetching form
        if (f16) {
            switch (epilogue) {
                case RF_EPI_BF16: return launch_phased_sk<E_BF16, P_F16>(p, 256, stream, "rf_gemm_f16");
                case RF_EPI_F32: return launch_phased_sk<E_F32, P_F16>(p, 256, stream, "rf_gemm_f16");
                case RF_EPI_ADD_F32: return launch_phased_sk<E_ADD, P_F16>(p, 256, stream, "rf_gemm_f16");
                default: return launch_phased_sk<E_SWIGLU, P_F16>(p, 256, stream, "rf_gemm_f16");
            }
        }
        switch (epilogue) {
            case RF_EPI_BF16: return launch_phased_sk<E_BF16>(p, 256, stream, "rf_gemm_bf16");
            case RF_EPI_F32: return launch_phased_sk<E_F32>(p, 256, stream, "rf_gemm_bf16");
            case RF_EPI_ADD_F32: return launch_phased_sk<E_ADD>(p, 256, stream, "rf_gemm_bf16");
            default: return launch_phased_sk<E_SWIGLU>(p, 256, stream, "rf_gemm_bf16");
        }
    }
    const int cfg = pick_cfg(m, n, k, epilogue);
    if (f16) return run_dp_f16(cfg, p, epilogue, stream);
    const bool big = cfg != 128;
    const int grid = (!big && workspace && ws_bytes >= SK_WS_BYTES) ? sk_grid(m, n, k) : 0;
    if (grid) {
        if (const int rc = sk_setup(p, workspace, stream)) return rc;
        switch (epilogue) {
            case RF_EPI_BF16: return launch_sk<T128, E_BF16>(p, grid, stream, "rf_gemm_bf16");
            case RF_EPI_F32: return launch_sk<T128, E_F32>(p, grid, stream, "rf_gemm_bf16");
            case RF_EPI_ADD_F32: return launch_sk<T128, E_ADD>(p, grid, stream, "rf_gemm_bf16");
            default: return launch_sk<T128, E_SWIGLU>(p, grid, stream, "rf_gemm_bf16");
        }
    }
    // 256x256 tiles at one 512-thread block per CU reach ~1.2 PF/s when every CU has work; when the tile count
    // would leave a ragged last round, stream-K the K loop over exactly 256 blocks instead.
    if (workspace && ws_bytes >= SK_WS_BYTES && n % 256 == 0 && sk256(m, n, k)) {
        if (const int rc = sk_setup(p, workspace, stream)) return rc;
        switch (epilogue) {
            case RF_EPI_BF16: return launch_sk<T256, E_BF16>(p, 256, stream, "rf_gemm_bf16");
            case RF_EPI_F32: return launch_sk<T256, E_F32>(p, 256, stream, "rf_gemm_bf16");
            case RF_EPI_ADD_F32: return launch_sk<T256, E_ADD>(p, 256, stream, "rf_gemm_bf16");
            default: return launch_sk<T256, E_SWIGLU>(p, 256, stream, "rf_gemm_bf16");
        }
    }
    return run_dp(cfg, p, epilogue, stream);
}

extern "C" int rf_gemm_bf16(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc,
                            const float* bias, int m, int n, int k, int epilogue, void* workspace, int64_t ws_bytes,
                            void* stream) {
    return gemm_bf16(a, lda, w, ldw, c, ldc, bias, m, n, k, epilogue, workspace, ws_bytes, stream, nullptr);
}

extern "C" int rf_gemm_f16(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc,
                           const float* bias, int m, int n, int k, int epilogue, void* workspace, int64_t ws_bytes,
                           void* stream) {
    return gemm_bf16(a, lda, w, ldw, c, ldc, bias, m, n, k, epilogue, workspace, ws_bytes, stream, nullptr, true);
}

// Deferred RMSNorm (rf.h): the producer.  Every kernel the dispatch below can pick for RF_EPI_ADD_F32 (phased3,
// phased, phased stream-K, ring engine data-parallel / stream-K) runs the engine epilogue with the LDS row-sum
// area; N > RF_PRENORM_SLOTS x 128 (more column tiles than slots) takes the GEMM + rf_prenorm.
extern "C" int rf_gemm_add_prenorm(const void* a, int64_t lda, const void* w, int64_t ldw, float* x, int64_t ldx,
                                   int m, int n, int k, const float* norm_w, void* xg, int64_t ldxg, float* ss,
                                   int operand_dtype, void* workspace, int64_t ws_bytes, void* stream) {
    RF_REQUIRE(x && norm_w && xg && ss, "rf_gemm_add_prenorm: null pointer");
    RF_REQUIRE(operand_dtype == RF_DT_F16 || operand_dtype == RF_DT_BF16, "rf_gemm_add_prenorm: operand_dtype");
    RF_REQUIRE(ldxg >= n && ldxg % 4 == 0 && ((uintptr_t)xg & 7) == 0, "rf_gemm_add_prenorm: xg rows (ldxg >= N, 8-B)");
    RF_REQUIRE(((uintptr_t)ss & 15) == 0 && ((uintptr_t)norm_w & 15) == 0, "rf_gemm_add_prenorm: ss / norm_w 16-B aligned");
    const bool f16 = operand_dtype == RF_DT_F16;
    if (n > PN_SLOTS * 128) {
        const int rc = gemm_bf16(a, lda, w, ldw, x, ldx, nullptr, m, n, k, RF_EPI_ADD_F32, workspace, ws_bytes, stream,
                                 nullptr, f16);
        if (rc != RF_OK) return rc;
        return rf_prenorm(x, ldx, norm_w, xg, ldxg, ss, m, n, operand_dtype, stream);
    }
    NormIO nio;
    nio.xg = xg;
    nio.ldxg = ldxg;
    nio.norm_g = norm_w;
    nio.ss_out = ss;
    nio.xg_f16 = f16;
    return gemm_bf16(a, lda, w, ldw, x, ldx, nullptr, m, n, k, RF_EPI_ADD_F32, workspace, ws_bytes, stream, nullptr,
                     f16, &nio);
}

// Deferred RMSNorm: the consumer (A = the producer's xg, rows scaled by 1 / rms in the epilogue)
extern "C" int rf_gemm_rownorm(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int m,
                               int n, int k, int epilogue, const float* ss, int norm_dim, float eps, float* seg_ss,
                               int seg_w, int n_seg, int operand_dtype, void* workspace, int64_t ws_bytes,
                               void* stream) {
    RF_REQUIRE(ss && ((uintptr_t)ss & 15) == 0, "rf_gemm_rownorm: ss must be 16-B aligned");
    RF_REQUIRE(norm_dim > 0, "rf_gemm_rownorm: norm_dim must be positive");
    RF_REQUIRE(epilogue == RF_EPI_BF16 || epilogue == RF_EPI_F16 || epilogue == RF_EPI_SWIGLU ||
                   epilogue == RF_EPI_SWIGLU_F16,
               "rf_gemm_rownorm: epilogue must be RF_EPI_BF16 / F16 / SWIGLU / SWIGLU_F16 (got %d)", epilogue);
    RF_REQUIRE(operand_dtype == RF_DT_F16 || operand_dtype == RF_DT_BF16, "rf_gemm_rownorm: operand_dtype");
    RF_REQUIRE(!seg_ss || ((epilogue == RF_EPI_BF16 || epilogue == RF_EPI_F16) && ((uintptr_t)seg_ss & 15) == 0 &&
                           seg_w > 0 && seg_w % 256 == 0 && seg_w <= PN_SLOTS * 128 && n_seg >= 1 &&
                           (int64_t)seg_w * n_seg <= n),
               "rf_gemm_rownorm: seg_ss needs a 16-bit (non-SwiGLU) epilogue, 16-B alignment, seg_w %% 256 == 0 and "
               "<= %d, n_seg >= 1 segments inside N", PN_SLOTS * 128);
    NormIO nio;
    nio.rs_part = ss;
    nio.rs_n = (float)norm_dim;
    nio.rs_eps = eps;
    nio.seg_ss = seg_ss;
    nio.seg_w = seg_w;
    nio.seg_n = seg_ss ? n_seg : 0;
    return gemm_bf16(a, lda, w, ldw, c, ldc, nullptr, m, n, k, epilogue, workspace, ws_bytes, stream, nullptr,
                     operand_dtype == RF_DT_F16, &nio);
}

// rf_gemm_qk_rope (rf.h): the q/k/v projection with the attention's q/k norm weight and rotary encoding in the
// epilogue (E_ROPE) on the engine's 96x256 or 8-wave 128x128 tile (the tiles the cost model picks for these shapes).
template <class C, int NT>
static int launch_rope(EngineArgs p, void* stream) {
    return launch<C, E_ROPE, NT>(p, stream, "rf_gemm_qk_rope");
}

extern "C" int rf_gemm_qk_rope(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int m,
                               int n, int k, const float* ss, int norm_dim, float eps, float* seg_ss, int seg_w,
                               int n_seg, const float* norm_w, const float* pos, int64_t ld_pos, int pos_div,
                               const float* freqs, int n_freqs, float q_scale, int operand_dtype, void* workspace,
                               int64_t ws_bytes, void* stream) {
    (void)workspace;
    (void)ws_bytes;
    RF_REQUIRE(a && w && c, "rf_gemm_qk_rope: null pointer");
    RF_REQUIRE(m > 0 && n > 0 && k > 0, "rf_gemm_qk_rope: empty problem m=%d n=%d k=%d", m, n, k);
    RF_REQUIRE(operand_dtype == RF_DT_F16 || operand_dtype == RF_DT_BF16, "rf_gemm_qk_rope: operand_dtype");
    RF_REQUIRE(k % 64 == 0 && n % 128 == 0, "rf_gemm_qk_rope: needs K %% 64 == 0 and N %% 128 == 0");
    RF_REQUIRE(lda % 8 == 0 && ldw % 8 == 0 && lda >= k && ldw >= k && ((uintptr_t)a & 15) == 0 &&
                   ((uintptr_t)w & 15) == 0, "rf_gemm_qk_rope: operands must be 16-B aligned with lda/ldw >= K");
    RF_REQUIRE(ldc >= n && ldc % 4 == 0 && ((uintptr_t)c & 7) == 0, "rf_gemm_qk_rope: ldc too small/unaligned");
    RF_REQUIRE(seg_w > 0 && seg_w % 256 == 0 && seg_w % 128 == 0 && n_seg >= 1 && (int64_t)seg_w * n_seg <= n,
               "rf_gemm_qk_rope: the q/k segments must be whole 256-column tiles inside N");
    RF_REQUIRE(!seg_ss || (((uintptr_t)seg_ss & 15) == 0 && seg_w <= PN_SLOTS * 128),
               "rf_gemm_qk_rope: seg_ss must be 16-B aligned and seg_w <= %d", PN_SLOTS * 128);
    RF_REQUIRE(!ss || (((uintptr_t)ss & 15) == 0 && norm_dim > 0), "rf_gemm_qk_rope: ss must be 16-B aligned");
    RF_REQUIRE(!norm_w || ((uintptr_t)norm_w & 15) == 0, "rf_gemm_qk_rope: norm_w must be 16-B aligned");
    RF_REQUIRE(!pos || (freqs && n_freqs > 0 && 9 * n_freqs <= 64 && ld_pos >= 9 && pos_div >= 1),
               "rf_gemm_qk_rope: pos needs freqs with 9 * n_freqs <= 64, ld_pos >= 9 and pos_div >= 1");
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
    p.rs_part = ss;
    p.rs_n = (float)norm_dim;
    p.rs_eps = eps;
    p.seg_ss = norm_w ? seg_ss : nullptr;  // (no norm: no 1 / rms downstream, no sums)
    p.seg_w = seg_w;
    p.seg_n = n_seg;
    p.rope_pos = pos;
    p.rope_ld = ld_pos;
    p.rope_div = pos ? pos_div : 1;
    p.rope_freqs = freqs;
    p.rope_nf = pos ? n_freqs : 1;
    p.rope_g = norm_w;
    p.rope_qscale = q_scale;
    const bool f16 = operand_dtype == RF_DT_F16;
    const int cfg = pick_cfg(m, n, k, RF_EPI_BF16);
    const bool t96 = n % 256 == 0 && (cfg == 962 || cfg != 12884);
    if (t96) return f16 ? launch_rope<T96x256, P_F16>(p, stream) : launch_rope<T96x256, 1>(p, stream);
    return f16 ? launch_rope<T128w8k2s4, P_F16>(p, stream) : launch_rope<T128w8k2s4, 1>(p, stream);
}

extern "C" int rf_gemm_bf16_if(const int* flag, const void* a, int64_t lda, const void* w, int64_t ldw, void* c,
                               int64_t ldc, const float* bias, int m, int n, int k, int epilogue, void* workspace,
                               int64_t ws_bytes, void* stream) {
    RF_REQUIRE(flag, "rf_gemm_bf16_if: null flag");
    return gemm_bf16(a, lda, w, ldw, c, ldc, bias, m, n, k, epilogue, workspace, ws_bytes, stream, flag);
}

extern "C" int rf_gemm_mx8(const void* a, int64_t lda, const void* sa, int64_t ld_sa, const void* w, int64_t ldw,
                           const void* sw, int64_t ld_sw, void* c, int64_t ldc, const float* bias, int m, int n, int k,
                           int epilogue, void* stream) {
    RF_REQUIRE(a && w && sa && sw && c, "rf_gemm_mx8: null pointer");
    RF_REQUIRE(m > 0 && n > 0 && k > 0, "rf_gemm_mx8: empty problem");
    RF_REQUIRE(k % 128 == 0 && n % 256 == 0, "rf_gemm_mx8: K=%d must be a multiple of 128 and N=%d of 256", k, n);
    RF_REQUIRE(lda % 16 == 0 && ldw % 16 == 0 && lda >= k && ldw >= k, "rf_gemm_mx8: lda/ldw (bytes) >= K, 16-B aligned");
    RF_REQUIRE(ld_sa % 4 == 0 && ld_sw % 4 == 0 && ld_sa >= k / 32 && ld_sw >= k / 32,
               "rf_gemm_mx8: scale rows must hold K/32 bytes, 4-B aligned");
    RF_REQUIRE(((uintptr_t)a & 15) == 0 && ((uintptr_t)w & 15) == 0 && ((uintptr_t)sa & 3) == 0 && ((uintptr_t)sw & 3) == 0,
               "rf_gemm_mx8: operands 16-B / scales 4-B aligned");
    RF_REQUIRE(epilogue >= RF_EPI_BF16 && epilogue <= RF_EPI_SWIGLU, "rf_gemm_mx8: bad epilogue %d", epilogue);
    RF_REQUIRE(ldc >= (epilogue == RF_EPI_SWIGLU ? n / 2 : n) && ldc % 4 == 0, "rf_gemm_mx8: ldc too small/unaligned");
    EngineArgs p{};
    p.a = (const bf16_t*)a;
    p.lda = lda;
    p.w = (const bf16_t*)w;
    p.ldw = ldw;
    p.sa = (const uint8_t*)sa;
    p.sw = (const uint8_t*)sw;
    p.ld_sa = (int)ld_sa;
    p.ld_sw = (int)ld_sw;
    p.m = m;
    p.n = n;
    p.k = k;
    p.c = c;
    p.ldc = ldc;
    p.bias = bias;
    hipStream_t st = (hipStream_t)stream;
    static const bool plain = getenv("RF_MX8_PLAIN") && atoi(getenv("RF_MX8_PLAIN")) != 0;  // A/B: the unstaggered loop
    if (!plain) {
        const int tiles_m = (m + 127) / 128, tiles_n = n / 256;
        const int nwg = tiles_m * tiles_n;
        p.group_m = pick_group_m(tiles_m, tiles_n, 128, 256, (nwg + 7) / 8, (int64_t)m * k);
        const dim3 g(nwg), b(512);
        switch (epilogue) {
            case RF_EPI_BF16: RF_LAUNCH((mx8_p3_kernel<E_BF16>), g, b, 0, st, p); break;
            case RF_EPI_F32: RF_LAUNCH((mx8_p3_kernel<E_F32>), g, b, 0, st, p); break;
            case RF_EPI_ADD_F32: RF_LAUNCH((mx8_p3_kernel<E_ADD>), g, b, 0, st, p); break;
            default: RF_LAUNCH((mx8_p3_kernel<E_SWIGLU>), g, b, 0, st, p); break;
        }
        return rf::check_launch("rf_gemm_mx8");
    }
    const int tiles_m = (m + 255) / 256, tiles_n = n / 256;
    const int nwg = tiles_m * tiles_n;
    p.group_m = pick_group_m(tiles_m, tiles_n, 256, 256, (nwg + 7) / 8, (int64_t)m * k);
    const dim3 g(nwg), b(512);
    switch (epilogue) {
        case RF_EPI_BF16: RF_LAUNCH((mx8_kernel<E_BF16>), g, b, 0, st, p); break;
        case RF_EPI_F32: RF_LAUNCH((mx8_kernel<E_F32>), g, b, 0, st, p); break;
        case RF_EPI_ADD_F32: RF_LAUNCH((mx8_kernel<E_ADD>), g, b, 0, st, p); break;
        default: RF_LAUNCH((mx8_kernel<E_SWIGLU>), g, b, 0, st, p); break;
    }
    return rf::check_launch("rf_gemm_mx8");
}

extern "C" int rf_quant_mx8(const void* x, int64_t ldx, int rows, int cols, void* q, int64_t ldq, void* scales,
                            int64_t ld_s, void* stream) {
    RF_REQUIRE(x && q && scales, "rf_quant_mx8: null pointer");
    RF_REQUIRE(cols % 32 == 0 && ldx % 8 == 0 && ldq % 16 == 0 && ldq >= cols && ld_s >= cols / 32,
               "rf_quant_mx8: cols %% 32, 16-B rows");
    if (rows <= 0) return RF_OK;
    const int64_t n = (int64_t)rows * (cols / 32);
    RF_LAUNCH(quant_mx8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, ldx, rows, cols, (uint8_t*)q, ldq, (uint8_t*)scales, ld_s);
    return rf::check_launch("rf_quant_mx8");
}

// halo2_kernel serves 3x3 / stride 1 / pad 1 fp16 convolutions on whole 16 x 32 tiles with a multiple of 128
// output channels (or 64: output_conv2) when they make at least one block per CU (RF_CONV_HALO2=0: never,
// 1: whenever it can)
static bool halo2_ok(const EngineArgs& a) {
    const char* env = getenv("RF_CONV_HALO2");
    if (env && atoi(env) == 0) return false;
    if (!env && getenv("RF_CONV_TILE")) return false;  // an explicit tile choice (A/B, tests) keeps its kernel
    if (a.kw != 3 || a.k != 9 * a.cin_pad || a.stride != 1 || a.pad != 1 || a.ho != a.hi || a.wo != a.wi) return false;
    if (a.cin_pad % 32 || (a.n % 128 && a.n != 64) || a.ho % h2::TH || a.wo % h2::TW || a.m % 512) return false;
    const int64_t blocks = (int64_t)(a.m / 512) * (a.n == 64 ? 1 : a.n / 128);
    return (env && atoi(env) == 1) || blocks >= 256;
}

static int launch_halo2(EngineArgs a, void* stream, const char* what) {
    const bool n64 = a.n == 64;
    const int nwg = (a.m / 512) * (n64 ? 1 : a.n / 128);
    const char* env = getenv("RF_CONV_H2S");  // W ring depth (slices in flight + 1): 4 (default), 3 or 5
    const int ring = env ? atoi(env) : 4;
    const hipStream_t st = (hipStream_t)stream;
    const int dbg = getenv("RF_H2_DBG") ? atoi(getenv("RF_H2_DBG")) : 0;  // ablation timing only
#ifndef RF_STUDY
    if (dbg) return rf::study_only("rf_conv: RF_H2_DBG (halo2 ablation builds)");
#else
    if (!n64 && ring == 4 && dbg >= 1 && dbg <= 8) {
        if (dbg == 1) RF_LAUNCH((halo2_kernel<4, 128, 1>), dim3(nwg), dim3(512), 0, st, a);
        if (dbg == 2) RF_LAUNCH((halo2_kernel<4, 128, 2>), dim3(nwg), dim3(512), 0, st, a);
        if (dbg == 3) RF_LAUNCH((halo2_kernel<4, 128, 3>), dim3(nwg), dim3(512), 0, st, a);
        if (dbg == 4) RF_LAUNCH((halo2_kernel<4, 128, 4>), dim3(nwg), dim3(512), 0, st, a);
        if (dbg == 8) RF_LAUNCH((halo2_kernel<4, 128, 8>), dim3(nwg), dim3(512), 0, st, a);
        return rf::check_launch(what);
    }
#endif
    if (n64) {
        if (ring == 3) RF_LAUNCH((halo2_kernel<3, 64>), dim3(nwg), dim3(512), 0, st, a);
        else if (ring == 5) RF_LAUNCH((halo2_kernel<5, 64>), dim3(nwg), dim3(512), 0, st, a);
        else RF_LAUNCH((halo2_kernel<4, 64>), dim3(nwg), dim3(512), 0, st, a);
    } else {
        if (ring == 3) RF_LAUNCH((halo2_kernel<3, 128>), dim3(nwg), dim3(512), 0, st, a);
        else if (ring == 5) RF_LAUNCH((halo2_kernel<5, 128>), dim3(nwg), dim3(512), 0, st, a);
        else RF_LAUNCH((halo2_kernel<4, 128>), dim3(nwg), dim3(512), 0, st, a);
    }
    return rf::check_launch(what);
}

// halo3_kernel serves halo2's non-final convolutions with a multiple of 128 output channels (RF_CONV_HALO3=0:
// halo2 instead); the bank must be addressable by 32-bit buffer offsets
static bool halo3_ok(const EngineArgs& a) {
    const char* env = getenv("RF_CONV_HALO3");
    if ((env && atoi(env) == 0) || (a.flags & RF_CONV_FINAL) || a.n % 128 || a.deconv) return false;
    if ((int64_t)128 * a.ldw * 2 >= 0x7fffffff) return false;
    return halo2_ok(a);
}

static int launch_halo3(EngineArgs a, void* stream, const char* what) {
    const int nwg = (a.m / 512) * (a.n / 128);
    const int dbg = getenv("RF_H3_DBG") ? atoi(getenv("RF_H3_DBG")) : 0;  // ablation timing only
#ifndef RF_STUDY
    if (dbg) return rf::study_only("rf_conv: RF_H3_DBG (halo3 ablation builds, garbage results)");
    RF_LAUNCH(halo3_kernel<0>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
#else
    if (dbg == 1) RF_LAUNCH(halo3_kernel<1>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    else if (dbg == 2) RF_LAUNCH(halo3_kernel<2>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    else if (dbg == 4) RF_LAUNCH(halo3_kernel<4>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    else if (dbg == 6) RF_LAUNCH(halo3_kernel<6>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    else if (dbg == 8) RF_LAUNCH(halo3_kernel<8>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    else if (dbg == 14) RF_LAUNCH(halo3_kernel<14>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    else if (dbg == 15) RF_LAUNCH(halo3_kernel<15>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    else if (dbg == 30) RF_LAUNCH(halo3_kernel<30>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    else if (dbg == 16) RF_LAUNCH(halo3_kernel<16>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    else if (dbg == 32) RF_LAUNCH(halo3_kernel<32>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    else if (dbg == 64) RF_LAUNCH(halo3_kernel<64>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    else if (dbg == 96) RF_LAUNCH(halo3_kernel<96>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
    else RF_LAUNCH(halo3_kernel<0>, dim3(nwg), dim3(512), 0, (hipStream_t)stream, a);
#endif
    return rf::check_launch(what);
}

// conv3x3_c32_kernel serves the fused-head 3x3 convolution with <= 32 filters (output_conv2) on whole 16 x 32
// tiles (RF_CONV_C32=0: the halo2 / engine paths instead)
static bool c32_ok(const EngineArgs& a) {
    const char* env = getenv("RF_CONV_C32");
    if ((env && atoi(env) == 0) || !(a.flags & RF_CONV_FINAL) || a.cout > 32 || a.n < 32) return false;
    if (a.kw != 3 || a.k != 9 * a.cin_pad || a.stride != 1 || a.pad != 1 || a.ho != a.hi || a.wo != a.wi) return false;
    return a.cin_pad % 32 == 0 && a.ho % c32::TH == 0 && a.wo % c32::TW == 0 && a.m > 0 && a.n_fin <= c32::NFIN;
}

static int launch_c32(EngineArgs a, void* stream, const char* what) {
    const int nwg = a.m / (c32::TH * c32::TW);
    RF_LAUNCH(conv3x3_c32_kernel, dim3(nwg), dim3(256), 0, (hipStream_t)stream, a);
    return rf::check_launch(what);
}

// conv3x3_hk_kernel serves non-final 3x3 / stride 1 / pad 1 fp16 convolutions on whole 16 x 32 tiles with a
// multiple of 64 output channels and at least one block per CU (RF_CONV_HK=0: the halo2 / engine paths; 1: whenever
// it can)
static bool hk_ok(const EngineArgs& a) {
    const char* env = getenv("RF_CONV_HK");
    if (!env || atoi(env) == 0 || (a.flags & RF_CONV_FINAL) || a.deconv) return false;  // opt-in: see DESIGN §3.4
#ifndef RF_STUDY
    return true;  // (the production build refuses it in launch_hk)
#else
    if (a.kw != 3 || a.k != 9 * a.cin_pad || a.stride != 1 || a.pad != 1 || a.ho != a.hi || a.wo != a.wi) return false;
    if (a.cin_pad % 32 || a.n % hk::NCO || a.ho % hk::TH || a.wo % hk::TW || a.m <= 0) return false;
    return atoi(env) == 1 || (int64_t)(a.m / (hk::TH * hk::TW)) * (a.n / hk::NCO) >= 256;
#endif
}

static int launch_hk(EngineArgs a, void* stream, const char* what) {
#ifdef RF_STUDY
    const int nwg = (a.m / (hk::TH * hk::TW)) * (a.n / hk::NCO);
    RF_LAUNCH(conv3x3_hk_kernel, dim3(nwg), dim3(256), 0, (hipStream_t)stream, a);
    return rf::check_launch(what);
#else
    (void)a, (void)stream, (void)what;
    return rf::study_only("rf_conv: RF_CONV_HK=1 (conv3x3_hk_kernel)");
#endif
}

// fp16 convolutions (one MFMA per product): the 256x256 tile when the filter bank is a multiple of 256
// wide and there is >= one tile per CU (the im2col gather of A is then read once per pixel tile),
// 256x64 for <= 64 output channels, else 128x128 (faster than 256x128 on every DPT shape measured)
template <bool GATHER>
static int conv_f16_dp(EngineArgs& p, void* stream, const char* what, int tile = 0) {
    if (GATHER && c32_ok(p)) return launch_c32(p, stream, what);
    if (GATHER && hk_ok(p)) return launch_hk(p, stream, what);
    if (GATHER && halo3_ok(p)) return launch_halo3(p, stream, what);
    if (GATHER && halo2_ok(p)) return launch_halo2(p, stream, what);
    const char* env = getenv("RF_CONV_TILE");
    const int t = tile ? tile : env ? atoi(env) : 0;
    // (RF_CONV_HALO=1 runs it halo-tiled: 90 -> 140 us at 512^2, 128 -> 32; a 128x64 tile at two blocks per
    // CU measured the same 90 us with or without the halo, so the gathered 256x64 launch stays the default)
    if (p.n == 64) return launch_conv<T256x64, P_F16, GATHER>(p, stream, what);
    if (t == 64 || t == 6464) return launch_conv<T64c, P_F16, GATHER>(p, stream, what);
    if (t == 6412) return launch_conv<T64x128c, P_F16, GATHER>(p, stream, what);
    if (t == 128) return launch_conv<T128, P_F16, GATHER>(p, stream, what);
    if (t == 1288) return launch_conv<T128w8, P_F16, GATHER>(p, stream, what);
    if (p.n % 256 == 0 && (t == 256 || (!t && ((p.m + 255) / 256) * (p.n / 256) >= 256)))
        return (getenv("RF_CONV_PHASED") && atoi(getenv("RF_CONV_PHASED")) && use_phased(p.n, p.k))
                   ? launch_phased<E_CONV, P_F16, GATHER, 256>(p, stream, what)
                   : launch_conv<T256, P_F16, GATHER>(p, stream, what);
    if (t == 2561) return launch<T256x128, E_CONV, P_F16, GATHER>(p, stream, what);
    // up to two 128x128 tiles per CU: the 8-wave tile (two waves per SIMD) hides the gathered staging's
    // latency (128^2 DPT level: 52 -> 41 us); with more tiles the 4-wave tile's extra blocks do that
    const int64_t tiles = (int64_t)((p.m + 127) / 128) * (p.n / 128);
    if (t != 128 && tiles <= 512) return launch_conv<T128w8, P_F16, GATHER>(p, stream, what);
    return launch_conv<T128, P_F16, GATHER>(p, stream, what);
}

template <int NT>
static int conv_dispatch(EngineArgs& p, bool gather, bool big, int64_t sk_grid_n, void* workspace, void* stream,
                         const char* what, int tile = 0) {
    if constexpr (NT == P_F16) {
        if (!sk_grid_n)
            return gather ? conv_f16_dp<true>(p, stream, what, tile) : conv_f16_dp<false>(p, stream, what, tile);
    }
    if (sk_grid_n) {
        if (const int rc = sk_setup(p, workspace, stream)) return rc;
        // fp16 convolutions stream-K over the 8-wave 128x128 tile (64^2 / 32^2 DPT levels: 1.6x / 2.1x)
        if (NT == P_F16 && !(getenv("RF_CONV_SKW8") && atoi(getenv("RF_CONV_SKW8")) == 0))
            return gather ? launch_sk<T128w8, E_CONV, NT, true>(p, (int)sk_grid_n, stream, what)
                          : launch_sk<T128w8, E_CONV, NT, false>(p, (int)sk_grid_n, stream, what);
        return gather ? launch_sk<T128, E_CONV, NT, true>(p, (int)sk_grid_n, stream, what)
                      : launch_sk<T128, E_CONV, NT, false>(p, (int)sk_grid_n, stream, what);
    }
    if (gather)
        return big ? launch<T256x128, E_CONV, NT, true>(p, stream, what) : launch<T128, E_CONV, NT, true>(p, stream, what);
    return big ? launch<T256x128, E_CONV, NT, false>(p, stream, what) : launch<T128, E_CONV, NT, false>(p, stream, what);
}

// nterm: 3 = bf16x3 hi/lo operands, P_F16 = one fp16 plane per operand (w_lo / in_lo unused)
static int conv_common(EngineArgs& p, int nterm, bool gather, const void* w_hi, const void* w_lo, int cout, int cout_pad, float* out,
                       const float* bias, const float* res1, const float* res2, void* p_hi, void* p_lo, int p_ld,
                       int flags, const float* w_fin, const float* b_fin, int n_fin, float elu_alpha, void* workspace,
                       int64_t ws_bytes, void* stream, const char* what) {
    RF_REQUIRE(w_hi && (w_lo || nterm == P_F16), "%s: null weights", what);
    RF_REQUIRE(cout % 4 == 0, "%s: cout must be a multiple of 4", what);
    RF_REQUIRE(out || p_hi, "%s: no output", what);
    RF_REQUIRE(!p_hi || ((p_lo || nterm == P_F16) && p_ld % 4 == 0 && p_ld >= cout), "%s: bad plane output", what);
    RF_REQUIRE(!(flags & RF_CONV_FINAL) || (cout <= 64 && w_fin && b_fin && n_fin > 0 && out),
               "%s: final head needs cout <= 64 and w_fin/b_fin", what);
    RF_REQUIRE(!(flags & RF_CONV_BORDER_BIAS) ||
                   (bias && !(flags & RF_CONV_FINAL) && p.kw == 3 && p.k == 9 * p.cin_pad && p.stride == 1 &&
                    p.pad == 1 && p.ho == p.hi && p.wo == p.wi && p.deconv == 0 && p.ho >= 2 && p.wo >= 2),
               "%s: RF_CONV_BORDER_BIAS needs a 3x3 stride-1 pad-1 convolution of an image of at least 2 x 2 pixels "
               "with its 9-row bias", what);
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
    p.plane_f16 = nterm == P_F16;
    p.range = (p_hi && nterm == P_F16) ? rf::range_word() : nullptr;
    p.cout = cout;
    p.flags = flags;
    p.w_fin = w_fin;
    p.b_fin = b_fin;
    p.n_fin = n_fin;
    p.elu_alpha = elu_alpha;
    if (p.m <= 0) return RF_OK;
    // 256x128 (8 waves) halves the L2 traffic per FLOP of the 128x128 tile but runs one block per CU:
    // use it only when it still yields >= one tile per CU.
    const char* env = getenv("RF_CONV_TILE");
    const bool big = env ? atoi(env) == 256 : ((p.m + 255) / 256) * (p.n / 128) >= 256;
    // Too few 128x128 tiles for 256 CUs (one bf16x3 block per CU): stream-K over the K loop, each block
    // keeping >= 8 K-steps.
    const char* sk_env = getenv("RF_CONV_SK");
    int64_t skg = 0;
    int ct = env ? atoi(env) : 0;
    // small DPT levels (<= 4,096 output pixels per launch: the 64^2 / 32^2 refinenets and their rn convs): the
    // 64x64 tile, data-parallel at K <= 2,304 and stream-K above (GPU time per launch, rocprofv3 over
    // tools/kbench.py conv: 256->256 @32 32.4 -> 26.6 us, @64 30.1 -> 27.6 us, 1024->256 @32 50.4 -> 41.4 us;
    // 1024->256 @64 stays on the default, 54.4 vs 68.1 us).  RF_CONV_SMALL=0 keeps the default tiles.
    static const bool small_on = !getenv("RF_CONV_SMALL") || atoi(getenv("RF_CONV_SMALL")) != 0;
    if (!ct && small_on && nterm == P_F16 && gather && p.kw == 3 && p.n % 64 == 0 && p.m <= 4096 &&
        (p.k <= 2304 || p.m <= 1024))
        ct = p.k <= 2304 ? 64 : 6464;
    if (nterm == P_F16 && ct == 6464 && p.n % 64 == 0 && workspace && ws_bytes >= SK_WS_BYTES) {
        // A/B: stream-K over the 64x64 small-level tile, up to two blocks per CU, >= 12 K-steps per block
        const int64_t tiles = (int64_t)((p.m + 63) / 64) * (p.n / 64);
        const int64_t grid = std::min<int64_t>(512, tiles * (p.k / BK) / 12);
        if (grid > tiles) {
            if (const int rc = sk_setup(p, workspace, stream)) return rc;
            return gather ? launch_sk<T64c, E_CONV, P_F16, true>(p, (int)grid, stream, what)
                          : launch_sk<T64c, E_CONV, P_F16, false>(p, (int)grid, stream, what);
        }
    }
    if (!big && p.n % 128 == 0 && workspace && ws_bytes >= SK_WS_BYTES && !(sk_env && atoi(sk_env) == 0) &&
        !(nterm == P_F16 && (ct == 64 || ct == 6412 || ct == 6464))) {
        const int64_t tiles = (int64_t)((p.m + 127) / 128) * (p.n / 128);
        const int64_t work = tiles * (p.k / BK);
        const int64_t grid = std::min<int64_t>(256, work / 8);
        if (tiles < 192 && grid > tiles) skg = grid;
    }
    return nterm == P_F16 ? conv_dispatch<P_F16>(p, gather, big, skg, workspace, stream, what, ct == 64 ? 64 : 0)
                          : conv_dispatch<3>(p, gather, big, skg, workspace, stream, what);
}

extern "C" int rf_conv2d_bf16x3(const void* in_hi, const void* in_lo, int n_img, int hi, int wi, int cin_pad,
                                const void* w_hi, const void* w_lo, int cout, int cout_pad, int kh, int kw, int stride,
                                int pad, const float* bias, const float* res1, const float* res2, float* out,
                                void* p_hi, void* p_lo, int p_ld, int flags, const float* w_fin, const float* b_fin,
                                int n_fin, float elu_alpha, void* workspace, int64_t ws_bytes, void* stream) {
    RF_REQUIRE(in_hi && in_lo, "rf_conv2d_bf16x3: null input");
    RF_REQUIRE(cin_pad % BK == 0, "rf_conv2d_bf16x3: cin_pad %d must be a multiple of %d", cin_pad, BK);
    RF_REQUIRE(cout_pad % 128 == 0 && cout_pad >= cout, "rf_conv2d_bf16x3: cout_pad %d must be a multiple of 128",
               cout_pad);
    EngineArgs p{};
    p.a = (const bf16_t*)in_hi;
    p.a_lo = (const bf16_t*)in_lo;
    p.hi = hi;
    p.wi = wi;
    p.cin_pad = cin_pad;
    p.cin_m = udiv_magic(cin_pad);
    p.ho = (hi + 2 * pad - kh) / stride + 1;
    p.wo = (wi + 2 * pad - kw) / stride + 1;
    p.kw = kw;
    p.kw_m = udiv_magic(kw);
    p.stride = stride;
    p.pad = pad;
    p.m = n_img * p.ho * p.wo;
    p.k = kh * kw * cin_pad;
    RF_REQUIRE(p.k < 65536, "conv: kh*kw*cin_pad = %d must be < 65536", p.k);
    p.ldw = p.k;
    return conv_common(p, 3, true, w_hi, w_lo, cout, cout_pad, out, bias, res1, res2, p_hi, p_lo, p_ld, flags, w_fin,
                       b_fin, n_fin, elu_alpha, workspace, ws_bytes, stream, "rf_conv2d_bf16x3");
}

extern "C" int rf_conv2d_f16(const void* in, int n_img, int hi, int wi, int cin_pad, const void* w, int cout,
                             int cout_pad, int kh, int kw, int stride, int pad, const float* bias, const float* res1,
                             const float* res2, float* out, void* p_out, int p_ld, int flags, const float* w_fin,
                             const float* b_fin, int n_fin, float elu_alpha, void* workspace, int64_t ws_bytes,
                             void* stream) {
    RF_REQUIRE(in, "rf_conv2d_f16: null input");
    RF_REQUIRE(cin_pad % BK == 0, "rf_conv2d_f16: cin_pad %d must be a multiple of %d", cin_pad, BK);
    RF_REQUIRE((cout_pad % 128 == 0 || cout_pad == 64) && cout_pad >= cout,
               "rf_conv2d_f16: cout_pad %d must be 64 or a multiple of 128", cout_pad);
    EngineArgs p{};
    p.a = (const bf16_t*)in;
    p.hi = hi;
    p.wi = wi;
    p.cin_pad = cin_pad;
    p.cin_m = udiv_magic(cin_pad);
    p.ho = (hi + 2 * pad - kh) / stride + 1;
    p.wo = (wi + 2 * pad - kw) / stride + 1;
    p.kw = kw;
    p.kw_m = udiv_magic(kw);
    p.stride = stride;
    p.pad = pad;
    p.m = n_img * p.ho * p.wo;
    p.k = kh * kw * cin_pad;
    RF_REQUIRE(p.k < 65536, "conv: kh*kw*cin_pad = %d must be < 65536", p.k);
    p.ldw = p.k;
    return conv_common(p, P_F16, true, w, nullptr, cout, cout_pad, out, bias, res1, res2, p_out, nullptr, p_ld, flags,
                       w_fin, b_fin, n_fin, elu_alpha, workspace, ws_bytes, stream, "rf_conv2d_f16");
}

// one grouped-launch member: the fields rf_conv2d_f16 / rf_deconv2d_f16 and conv_common set (the deconvolution
// runs its dense A as a 1x1 gather: the same row addresses), or an error message
static const char* group_member(EngineArgs& p, const rf_conv_desc& d, const void* zero) {
    if (!d.in || !d.w || !(d.out || d.p_out)) return "null pointer";
    if (d.cin_pad % BK) return "cin_pad must be a multiple of 32";
    if (d.cout % 4) return "cout must be a multiple of 4";
    if (d.p_out && (d.p_ld % 4 || d.p_ld < d.cout)) return "bad p_ld";
    if (d.flags & RF_CONV_FINAL) return "the fused final head runs on its own launch";
    p = EngineArgs{};
    p.a = (const bf16_t*)d.in;
    p.cin_pad = d.cin_pad;
    p.cin_m = udiv_magic(d.cin_pad);
    p.zero = (const bf16_t*)zero;
    if (d.deconv_k > 0) {
        p.hi = p.ho = d.hi;
        p.wi = p.wo = d.wi;
        p.kw = 1;
        p.stride = 1;
        p.pad = 0;
        p.deconv = d.deconv_k;
        p.n = d.deconv_k * d.deconv_k * d.cout;
        if (d.flags) return "a deconvolution takes no flags";
    } else {
        p.hi = d.hi;
        p.wi = d.wi;
        p.ho = (d.hi + 2 * d.pad - d.kh) / d.stride + 1;
        p.wo = (d.wi + 2 * d.pad - d.kw) / d.stride + 1;
        p.kw = d.kw;
        p.stride = d.stride;
        p.pad = d.pad;
        p.n = d.cout_pad;
        if (d.cout_pad < d.cout) return "cout_pad < cout";
        if ((d.flags & RF_CONV_BORDER_BIAS) &&
            !(d.bias && d.kh == 3 && d.kw == 3 && d.stride == 1 && d.pad == 1 && d.hi >= 2 && d.wi >= 2))
            return "RF_CONV_BORDER_BIAS needs a 3x3 stride-1 pad-1 convolution of an image of at least 2 x 2 pixels "
                   "with its 9-row bias";
    }
    p.kw_m = udiv_magic(p.kw);
    p.m = d.n_img * p.ho * p.wo;
    p.k = (d.deconv_k > 0 ? 1 : d.kh * d.kw) * d.cin_pad;
    if (p.k >= 65536) return "kh*kw*cin_pad must be < 65536";
    if (p.n % T128w8::BN) return "output channels (k*k*cout for a deconvolution) must be a multiple of 128";
    p.ldw = p.k;
    p.w = (const bf16_t*)d.w;
    p.c = d.out;
    p.bias = d.bias;
    p.p_hi = (bf16_t*)d.p_out;
    p.p_ld = d.p_ld;
    p.plane_f16 = 1;
    p.range = d.p_out ? rf::range_word() : nullptr;
    p.cout = d.cout;
    p.flags = d.flags;
    return nullptr;
}

// dense: every member is a 1x1 stride-1 convolution over unpadded pixels (A = dense rows of cin_pad, K a
// multiple of 64): the 128x128 tile with 64-deep steps on plain rows (the stage-2 projections' loop) instead of
// the gathered 32-deep one
template <bool DENSE>
static int conv_group_launch(int n_conv, const rf_conv_desc* convs, void* stream, const char* what) {
    RF_REQUIRE(n_conv >= 1 && n_conv <= GROUP_MAX && convs, "%s: 1..%d convolutions", what, GROUP_MAX);
    static void* z = nullptr;
    if (!z && hipGetSymbolAddress(&z, HIP_SYMBOL(g_zero_row)) != hipSuccess) {
        z = nullptr;
        rf::set_error("%s: zero row symbol", what);
        return RF_ERR_LAUNCH;
    }
    using C = std::conditional_t<DENSE, T128w8k2s4, T128w8>;
    GroupArgs g{};
    g.n = n_conv;
    int blocks = 0;
    for (int q = 0; q < n_conv; ++q) {
        const char* err = group_member(g.p[q], convs[q], z);
        RF_REQUIRE(!err, "%s: conv %d: %s", what, q, err ? err : "");
        EngineArgs& p = g.p[q];
        if constexpr (DENSE) {
            RF_REQUIRE(convs[q].kh == 1 && convs[q].kw == 1 && convs[q].stride == 1 && convs[q].pad == 0 &&
                           !convs[q].deconv_k && p.k % (BK * C::KH) == 0,
                       "%s: conv %d: dense members are 1x1 stride-1 convolutions with cin_pad %% 64 == 0", what, q);
            p.lda = p.cin_pad;
        }
        const int tiles_m = (p.m + C::BM - 1) / C::BM, tiles_n = p.n / C::BN;
        p.group_m = pick_group_m(tiles_m, tiles_n, C::BM, C::BN, ((int64_t)tiles_m * tiles_n + 7) / 8);
        g.first[q] = blocks;
        blocks += tiles_m * tiles_n;
    }
    g.first[n_conv] = blocks;
    if (blocks == 0) return RF_OK;
    RF_LAUNCH((engine_group_kernel<C, E_CONV, P_F16, !DENSE>), dim3(blocks), dim3(C::THREADS), 0, (hipStream_t)stream,
              g);
    return rf::check_launch(what);
}

extern "C" int rf_conv2d_f16_group(int n_conv, const rf_conv_desc* convs, void* stream) {
    return conv_group_launch<false>(n_conv, convs, stream, "rf_conv2d_f16_group");
}

extern "C" int rf_conv1x1_f16_group(int n_conv, const void* const* in, const int* cin_pad, const void* const* w,
                                    const int* cout, const int* cout_pad, const float* const* bias,
                                    void* const* p_out, const int* p_ld, int n_img, int hi, int wi, void* stream) {
    RF_REQUIRE(n_conv >= 1 && n_conv <= GROUP_MAX, "rf_conv1x1_f16_group: 1..%d convolutions", GROUP_MAX);
    RF_REQUIRE(in && cin_pad && w && cout && cout_pad && p_out && p_ld, "rf_conv1x1_f16_group: null array");
    rf_conv_desc d[GROUP_MAX] = {};
    for (int q = 0; q < n_conv; ++q) {
        d[q].in = in[q];
        d[q].w = w[q];
        d[q].bias = bias ? bias[q] : nullptr;
        d[q].p_out = p_out[q];
        d[q].n_img = n_img;
        d[q].hi = hi;
        d[q].wi = wi;
        d[q].cin_pad = cin_pad[q];
        d[q].cout = cout[q];
        d[q].cout_pad = cout_pad[q];
        d[q].kh = d[q].kw = d[q].stride = 1;
        d[q].p_ld = p_ld[q];
    }
    // (RF_CONV_GROUP_DENSE=0: the gathered 32-deep loop, A/B)
    static const bool dense = !getenv("RF_CONV_GROUP_DENSE") || atoi(getenv("RF_CONV_GROUP_DENSE")) != 0;
    bool ok = dense;
    for (int q = 0; q < n_conv; ++q) ok = ok && cin_pad[q] % 64 == 0;
    return ok ? conv_group_launch<true>(n_conv, d, stream, "rf_conv1x1_f16_group")
              : conv_group_launch<false>(n_conv, d, stream, "rf_conv1x1_f16_group");
}

extern "C" int rf_deconv2d_bf16x3(const void* in_hi, const void* in_lo, int n_img, int hi, int wi, int cin_pad,
                                  const void* w_hi, const void* w_lo, int cout, int k, const float* bias, float* out,
                                  void* p_hi, void* p_lo, int p_ld, void* workspace, int64_t ws_bytes, void* stream) {
    RF_REQUIRE(in_hi && in_lo, "rf_deconv2d_bf16x3: null input");
    RF_REQUIRE(cin_pad % BK == 0, "rf_deconv2d_bf16x3: cin_pad must be a multiple of %d", BK);
    RF_REQUIRE((k * k * cout) % 128 == 0 && cout < 65536, "rf_deconv2d_bf16x3: k*k*cout must be a multiple of 128");
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
    return conv_common(p, 3, false, w_hi, w_lo, cout, k * k * cout, out, bias, nullptr, nullptr, p_hi, p_lo, p_ld, 0,
                       nullptr, nullptr, 0, 0.f, workspace, ws_bytes, stream, "rf_deconv2d_bf16x3");
}

extern "C" int rf_deconv2d_f16(const void* in, int n_img, int hi, int wi, int cin_pad, const void* w, int cout, int k,
                               const float* bias, float* out, void* p_out, int p_ld, void* workspace, int64_t ws_bytes,
                               void* stream) {
    RF_REQUIRE(in, "rf_deconv2d_f16: null input");
    RF_REQUIRE(cin_pad % BK == 0, "rf_deconv2d_f16: cin_pad must be a multiple of %d", BK);
    RF_REQUIRE((k * k * cout) % 128 == 0 && cout < 65536, "rf_deconv2d_f16: k*k*cout must be a multiple of 128");
    EngineArgs p{};
    p.a = (const bf16_t*)in;
    p.lda = cin_pad;
    p.ho = hi;
    p.wo = wi;
    p.m = n_img * hi * wi;
    p.k = cin_pad;
    p.ldw = cin_pad;
    p.deconv = k;
    return conv_common(p, P_F16, false, w, nullptr, cout, k * k * cout, out, bias, nullptr, nullptr, p_out, nullptr,
                       p_ld, 0, nullptr, nullptr, 0, 0.f, workspace, ws_bytes, stream, "rf_deconv2d_f16");
}
