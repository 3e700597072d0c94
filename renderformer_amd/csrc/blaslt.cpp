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
std::map<std::tuple<int, int, int, int, int64_t, int64_t, int64_t, int, bool>, Plan> g_plans;

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
    const auto key = std::make_tuple(dev, m, n, k, lda, ldw, ldc, mode, bias != nullptr);
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
        hipblasLtMatmulHeuristicResult_t res[1];
        int found = 0;
        good = good && hipblasLtMatmulAlgoGetHeuristic(h, pl.desc, pl.la, pl.lb, pl.lc, pl.lc, pref, 1, res, &found) ==
                           HIPBLAS_STATUS_SUCCESS;
        if (pref) hipblasLtMatmulPreferenceDestroy(pref);
        if (good && found > 0) {
            pl.algo = res[0].algo;
            pl.ws = res[0].workspaceSize;
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
