// hipBLASLt backend for the plain projection GEMMs (guide: "hipBLASLt/rocBLAS only for plain library
// GEMMs"): C[M,N] = A[M,K]·W[N,K]^T with a bf16 result, an fp32 result (+ optional fp32 bias per
// column), or an fp32 residual accumulate C += A·W^T (beta 1, C == D).  Fused epilogues (SwiGLU, the
// DPT convolutions) stay on the hand-written engine.
//
// Row-major C[M,N] is column-major C^T[N,M]: D = op(A_l)·op(B_l) with A_l = W viewed col-major
// [K x N] (transposed), B_l = A viewed col-major [K x M], so m_l = N, n_l = M.
// One handle per device and one algorithm per (device, shape, epilogue), chosen once by hipBLASLt's
// heuristic under the caller's workspace size and cached (the "lazily initialised per-device cache" of
// the ABI contract); nothing is allocated on the device by this file.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "common.h"

namespace {

struct Plan {
    hipblasLtMatmulDesc_t desc = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
    hipblasLtMatmulAlgo_t algo;
    size_t ws = 0;
    bool ok = false;
};

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;
std::map<std::tuple<int, int, int, int, int64_t, int64_t, int64_t, int, bool, int>, Plan> g_plans;

// RF_BLASLT_ALGO=i (tuning/diagnostics, tools/kbench.py blaslt): use the i-th heuristic candidate instead
// of the first
int algo_choice() {
    const char* e = getenv("RF_BLASLT_ALGO");
    return e ? atoi(e) : 0;
}

// One-time tuning of a bf16-output plan (the QKV / Q / KV projections): hipBLASLt's first heuristic pick
// is up to 15 % off the best of its top candidates on the path's shapes (tools/kbench.py blaslt), so the
// first call per shape times TUNE_CANDIDATES of them on the caller's buffers (beta = 0: the output is
// rewritten by the real call that follows) and keeps the fastest.  This synchronises the stream once per
// shape; RF_BLASLT_TUNE=0 disables it, and it is skipped while the stream is being captured.  The
// residual-accumulate plans (beta = 1) are never tuned: their output is live (and the first pick was the
// fastest on every path shape).
constexpr int TUNE_CANDIDATES = 8;

bool tune_enabled(hipStream_t stream) {
    const char* e = getenv("RF_BLASLT_TUNE");
    if (e && atoi(e) == 0) return false;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
    return true;
}

int fastest(hipblasLtHandle_t h, const Plan& pl, const hipblasLtMatmulHeuristicResult_t* res, int found,
            const void* w, const void* a, void* c, uint64_t wmax, void* workspace, hipStream_t stream) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 0;
    const float alpha = 1.0f, beta = 0.0f;
    int best = 0;
    float best_ms = 1e30f;
    for (int i = 0; i < found; ++i) {
        if (res[i].workspaceSize > wmax) continue;
        auto run = [&]() {
            return hipblasLtMatmul(h, pl.desc, &alpha, w, pl.la, a, pl.lb, &beta, c, pl.lc, c, pl.lc, &res[i].algo,
                                   workspace, res[i].workspaceSize, stream) == HIPBLAS_STATUS_SUCCESS;
        };
        if (!run()) continue;  // warm-up (and validity)
        bool ok = hipEventRecord(e0, stream) == hipSuccess;
        for (int r = 0; r < 4 && ok; ++r) ok = run();
        ok = ok && hipEventRecord(e1, stream) == hipSuccess;
        float ms = 0.f;
        if (!ok || hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) continue;
        if (ms < best_ms) {
            best_ms = ms;
            best = i;
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return best;
}

hipblasLtHandle_t handle_for(int dev) {
    auto it = g_handles.find(dev);
    if (it != g_handles.end()) return it->second;
    hipblasLtHandle_t h = nullptr;
    if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) return nullptr;
    g_handles[dev] = h;
    return h;
}

}  // namespace

namespace rf {

// mode: RF_EPI_BF16, RF_EPI_F32 (bias optional) or RF_EPI_ADD_F32.
// returns RF_OK, or -1 when hipBLASLt has no algorithm for the case (caller falls back to its own kernel)
int blaslt_gemm(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int m, int n, int k,
                int mode, const float* bias, void* workspace, int64_t ws_bytes, void* stream) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    std::lock_guard<std::mutex> lock(g_mu);
    hipblasLtHandle_t h = handle_for(dev);
    if (!h) return -1;
    const int choice = algo_choice();
    const auto key = std::make_tuple(dev, m, n, k, lda, ldw, ldc, mode, bias != nullptr, choice);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
        Plan pl;
        const hipDataType ct = mode == RF_EPI_BF16 ? HIP_R_16BF : HIP_R_32F;
        bool good = hipblasLtMatmulDescCreate(&pl.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS;
        const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
        good = good && hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)) ==
                           HIPBLAS_STATUS_SUCCESS;
        good = good && hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)) ==
                           HIPBLAS_STATUS_SUCCESS;
        if (bias) {
            const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
            const hipDataType bt = HIP_R_32F;
            good = good && hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)) ==
                               HIPBLAS_STATUS_SUCCESS;
            good = good && hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt,
                                                           sizeof(bt)) == HIPBLAS_STATUS_SUCCESS;
        }
        good = good && hipblasLtMatrixLayoutCreate(&pl.la, HIP_R_16BF, k, n, ldw) == HIPBLAS_STATUS_SUCCESS;
        good = good && hipblasLtMatrixLayoutCreate(&pl.lb, HIP_R_16BF, k, m, lda) == HIPBLAS_STATUS_SUCCESS;
        good = good && hipblasLtMatrixLayoutCreate(&pl.lc, ct, n, m, ldc) == HIPBLAS_STATUS_SUCCESS;
        hipblasLtMatmulPreference_t pref = nullptr;
        good = good && hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS;
        uint64_t wmax = workspace ? (uint64_t)ws_bytes : 0;
        good = good && hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wmax,
                                                             sizeof(wmax)) == HIPBLAS_STATUS_SUCCESS;
        hipblasLtMatmulHeuristicResult_t res[32];
        int found = 0;
        const bool tune = choice == 0 && mode == RF_EPI_BF16 && tune_enabled((hipStream_t)stream);
        const int want = tune ? TUNE_CANDIDATES : std::min(choice + 1, 32);
        good = good && hipblasLtMatmulAlgoGetHeuristic(h, pl.desc, pl.la, pl.lb, pl.lc, pl.lc, pref, want, res,
                                                       &found) == HIPBLAS_STATUS_SUCCESS;
        if (pref) hipblasLtMatmulPreferenceDestroy(pref);
        if (good && found > 0) {
            int i = std::max(0, std::min(choice, found - 1));
            if (tune && found > 1) i = fastest(h, pl, res, found, w, a, c, wmax, workspace, (hipStream_t)stream);
            pl.algo = res[i].algo;
            pl.ws = res[i].workspaceSize;
            pl.ok = pl.ws <= wmax;
        }
        it = g_plans.emplace(key, pl).first;
    }
    const Plan& pl = it->second;
    if (!pl.ok) return -1;
    if (bias && hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)) !=
                    HIPBLAS_STATUS_SUCCESS)
        return -1;
    const float alpha = 1.0f, beta = mode == RF_EPI_ADD_F32 ? 1.0f : 0.0f;
    const hipblasStatus_t st = hipblasLtMatmul(h, pl.desc, &alpha, w, pl.la, a, pl.lb, &beta, c, pl.lc, c, pl.lc,
                                               &pl.algo, workspace, pl.ws, (hipStream_t)stream);
    if (st != HIPBLAS_STATUS_SUCCESS) {
        set_error("rf_gemm_bf16: hipblasLtMatmul failed (status %d)", (int)st);
        return RF_ERR_LAUNCH;
    }
    return RF_OK;
}

}  // namespace rf
