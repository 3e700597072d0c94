// bf16 MFMA GEMM  C[M,N] (epilogue) A[M,K] * W[N,K]^T  for gfx950.
//
// Both operands are K-contiguous (nn.Linear weight layout [out, in]), which is
// the natural MFMA operand order: no transposes anywhere.
//
// Tile 128x128x64, 256 threads = 4 waves in a 2x2 grid, each wave 64x64 out
// of 4x4 v_mfma_f32_16x16x32_bf16 tiles (64 accumulator VGPRs).  Operands are
// staged global->LDS with global_load_lds_dwordx4 (no VGPR round trip) into
// two LDS buffers; the LDS image is row-major [128][64] bf16 (128-B rows) with
// the 16-B chunk index XOR-swizzled by (row & 7) — applied on the *source*
// address because LDS-DMA writes lane-linearly — which makes the fragment
// ds_read_b128s conflict-free (checked with tools/banks model, 4 LDS cycles
// per read).  blockIdx is remapped so each XCD walks a contiguous band of
// output tiles (shared A rows / W columns stay in that XCD's L2).
//
// Epilogues fuse the bias, fp32 residual accumulation (x += proj) and SwiGLU
// (silu(w1 x) * w3 x with the two weight halves interleaved in 16-row groups),
// so no intermediate [M, 2F] tensor ever reaches HBM.
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int THREADS = 256;
constexpr int TILE_BYTES = BM * BK * 2;  // 16 KiB per operand tile

struct GemmArgs {
    const bf16_t* a;
    const bf16_t* w;
    void* c;
    const float* bias;
    int64_t lda, ldw, ldc;
    int m, n, k;
};

// Stage one BK-slice of a 128-row operand panel into LDS (lane-linear image, swizzled source).
RF_DEV void stage_panel(const bf16_t* base, int64_t ld, int row0, int row_max, int k0, char* lds_tile, int wave,
                        int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int piece = wave * 4 + i;          // 1 KiB piece = 8 rows x 128 B
        const int chunk = piece * 64 + lane;     // 16-B chunk index in the tile image
        const int row = chunk >> 3;
        const int lc = (chunk & 7) ^ (row & 7);  // logical k-chunk held at this physical slot
        int grow = row0 + row;
        grow = grow < row_max ? grow : row_max - 1;
        const bf16_t* src = base + (int64_t)grow * ld + k0 + lc * 8;
        __builtin_amdgcn_global_load_lds(GLB_PTR(void, src), LDS_PTR(void, lds_tile + piece * 1024), 16, 0, 0);
    }
}

RF_DEV bf16x8 read_frag(const char* tile, int row, int kchunk) {
    const int off = row * 128 + ((kchunk ^ (row & 7)) << 4);
    return *reinterpret_cast<const bf16x8*>(tile + off);
}

RF_DEV float silu(float x) { return x / (1.0f + __expf(-x)); }

template <int EPI>
__global__ __launch_bounds__(THREADS, 2) void gemm_bf16_kernel(GemmArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];  // [buf][A|B]

    const int tiles_n = p.n / BN;
    const int tiles_m = (p.m + BM - 1) / BM;
    const int nwg = tiles_n * tiles_m;
    // XCD-aware bijective remap: consecutive hardware ids round-robin over 8 XCDs;
    // give each XCD a contiguous run of logical tiles.
    const int hw = blockIdx.x;
    const int xcd = hw & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (hw >> 3);
    // tiles walked column-band major so neighbouring tiles share W panels
    const int tm = wg % tiles_m;
    const int tn = wg / tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = p.k / BK;
    stage_panel(p.a, p.lda, m0, p.m, 0, smem, wave, lane);
    stage_panel(p.w, p.ldw, n0, p.n, 0, smem + TILE_BYTES, wave, lane);
    wait_vmcnt0();
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
        char* cur = smem + (kt & 1) * 2 * TILE_BYTES;
        if (kt + 1 < nk) {
            char* nxt = smem + ((kt + 1) & 1) * 2 * TILE_BYTES;
            stage_panel(p.a, p.lda, m0, p.m, (kt + 1) * BK, nxt, wave, lane);
            stage_panel(p.w, p.ldw, n0, p.n, (kt + 1) * BK, nxt + TILE_BYTES, wave, lane);
        }
        const char* ta = cur;
        const char* tb = cur + TILE_BYTES;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int kc = ks * 4 + (lane >> 4);
            bf16x8 fa[4], fb[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) fa[i] = read_frag(ta, wm * 64 + i * 16 + (lane & 15), kc);
#pragma unroll
            for (int j = 0; j < 4; ++j) fb[j] = read_frag(tb, wn * 64 + j * 16 + (lane & 15), kc);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        wait_vmcnt0();
        __syncthreads();
    }

    // ------------------------------------------------------------------ epilogue
    const int col_l = lane & 15;
    const int row_q = (lane >> 4) * 4;
    if constexpr (EPI == RF_EPI_SWIGLU) {
        bf16_t* c = reinterpret_cast<bf16_t*>(p.c);
#pragma unroll
        for (int pair = 0; pair < 2; ++pair) {
            const int gcol = n0 + wn * 64 + pair * 32;       // start of a 32-row interleave group
            const int ocol = (gcol >> 5) * 16 + col_l;        // output feature index
            const float b1 = p.bias ? p.bias[gcol + col_l] : 0.f;
            const float b3 = p.bias ? p.bias[gcol + 16 + col_l] : 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int row = m0 + wm * 64 + i * 16 + row_q + rr;
                    if (row < p.m) {
                        const float g = acc[i][2 * pair][rr] + b1;
                        const float u = acc[i][2 * pair + 1][rr] + b3;
                        c[(int64_t)row * p.ldc + ocol] = f32_to_bf16(silu(g) * u);
                    }
                }
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = n0 + wn * 64 + j * 16 + col_l;
            const float b = p.bias ? p.bias[col] : 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int row = m0 + wm * 64 + i * 16 + row_q + rr;
                    if (row < p.m) {
                        const float v = acc[i][j][rr] + b;
                        const int64_t o = (int64_t)row * p.ldc + col;
                        if constexpr (EPI == RF_EPI_BF16) {
                            reinterpret_cast<bf16_t*>(p.c)[o] = f32_to_bf16(v);
                        } else if constexpr (EPI == RF_EPI_F32) {
                            reinterpret_cast<float*>(p.c)[o] = v;
                        } else {
                            reinterpret_cast<float*>(p.c)[o] += v;
                        }
                    }
                }
        }
    }
}

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
    RF_REQUIRE(ldc >= (epilogue == RF_EPI_SWIGLU ? n / 2 : n), "rf_gemm_bf16: ldc too small");
    GemmArgs p{(const bf16_t*)a, (const bf16_t*)w, c, bias, lda, ldw, ldc, m, n, k};
    const int nwg = (n / BN) * ((m + BM - 1) / BM);
    hipStream_t s = (hipStream_t)stream;
    switch (epilogue) {
        case RF_EPI_BF16: hipLaunchKernelGGL(gemm_bf16_kernel<RF_EPI_BF16>, dim3(nwg), dim3(THREADS), 0, s, p); break;
        case RF_EPI_F32: hipLaunchKernelGGL(gemm_bf16_kernel<RF_EPI_F32>, dim3(nwg), dim3(THREADS), 0, s, p); break;
        case RF_EPI_ADD_F32: hipLaunchKernelGGL(gemm_bf16_kernel<RF_EPI_ADD_F32>, dim3(nwg), dim3(THREADS), 0, s, p); break;
        default: hipLaunchKernelGGL(gemm_bf16_kernel<RF_EPI_SWIGLU>, dim3(nwg), dim3(THREADS), 0, s, p); break;
    }
    return rf::check_launch("rf_gemm_bf16");
}
