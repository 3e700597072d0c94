// Error plumbing shared by every entry point of librfhip (thread-local last error).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace rf {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// one mapped, portable host word for the process: kernels on any device store error codes into it, the host
// reads it with a plain load (no device sync)
static volatile int* g_dev_err_host = nullptr;
static int* g_dev_err_dev = nullptr;
static std::once_flag g_dev_err_once;

int* device_error_word() {
    std::call_once(g_dev_err_once, [] {
        void* h = nullptr;
        if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess)
            return;
        memset(h, 0, 64);
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return;
        g_dev_err_host = (volatile int*)h;
        g_dev_err_dev = (int*)d;
    });
    return g_dev_err_dev;
}

// The fp16 range word the calling thread's launches raise: the word bound by rf_range_word_bind (one per frame,
// the model's), else word 1 of the error allocation (the process-wide rf_f16_range_flag).  Thread-local: a render
// issues all its launches from one thread, so two renders on two threads (or one after the other on one thread,
// each binding its own word) never share a word.
static thread_local int* g_bound_range = nullptr;

int* range_word() {
    if (g_bound_range) return g_bound_range;
    int* w = device_error_word();
    return w ? w + 1 : nullptr;
}

struct RangeWord {
    volatile int* host;  // mapped, coherent: kernels store, the host reads with a plain load
    int* dev;
};

// Hand-off flag epochs of the stream-K kernels (attention and GEMM/conv): every launch gets a fresh flag value,
// so flags need no re-arm and no memset between launches.  Values are 1 + (counter mod 2^B) (B = 30, or
// RF_EPOCH_BITS for tests), i.e. they repeat every 2^B launches; a flag slot written 2^B launches ago and never
// since could then equal the current value and let an owner fold a stale partial.  So per flag area the
// generation (counter >> B) of its last launch is remembered, and the first launch of a new generation on an area
// re-zeroes the area first (stream-ordered hipMemsetAsync; zero is never an epoch).  Thread-safe; 64-bit counter.
int next_epoch(void* flags, size_t bytes, hipStream_t st) {
    static std::mutex mu;
    static uint64_t counter = 0;
    static std::unordered_map<void*, uint64_t> gen_of;
    const char* env = getenv("RF_EPOCH_BITS");  // (read per launch: tests shrink the period to force wraps)
    const int bits = env ? std::min(30, std::max(2, atoi(env))) : 30;
    std::lock_guard<std::mutex> lk(mu);
    const uint64_t c = counter++;
    const uint64_t gen = c >> bits;
    auto it = gen_of.find(flags);
    if (it == gen_of.end()) {
        gen_of.emplace(flags, gen);  // a new area is zero-filled by its owner (rf.h workspace contract)
    } else if (it->second != gen) {
        // a failed re-zero would leave last generation's flags in place, where one can equal a new epoch: the
        // generation stays unchanged and the launch is refused (0 is never an epoch; callers return the error)
        if (hipMemsetAsync(flags, 0, bytes, st) != hipSuccess) {
            set_error("stream-K flag area re-zero (hipMemsetAsync) failed at an epoch generation wrap");
            return 0;
        }
        it->second = gen;
    }
    return 1 + (int)(c & ((1ull << bits) - 1));
}

int study_only(const char* what) {
    set_error("%s is a study kernel: this librfhip is the production build; use the study build "
              "(make -C renderformer_amd/csrc study -> lib/librfhip_study.so, selected with RF_LIB)", what);
    return RF_ERR_UNSUPPORTED;
}

int spin_limit() {
    static const int lim = [] {
        const char* e = getenv("RF_SPIN_LIMIT");
        return e ? atoi(e) : (1 << 24);
    }();
    return lim;
}

int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return RF_ERR_LAUNCH;
    }
    if (g_dev_err_host && *g_dev_err_host != 0) {
        set_error("%s: an earlier launch reported device error %d (%s); its outputs are invalid and the stream-K "
                  "workspaces must be re-zeroed (rf_clear_device_error)", what, *g_dev_err_host,
                  *g_dev_err_host == RF_DEVERR_SK_GEMM ? "GEMM stream-K partial not published within the spin bound"
                  : *g_dev_err_host == RF_DEVERR_SK_ATTN ? "attention stream-K partial not published within the spin "
                                                            "bound" : "debug");
        return RF_ERR_DEVICE;
    }
    return RF_OK;
}

// kernel timer: event pairs created by rf_ktimer_arm on the caller's current device, taken by the next launch
struct KTimer {
    std::vector<hipEvent_t> start, stop;  // one pair per armed launch, in launch order
    bool armed = false;
};
static thread_local KTimer g_kt;

bool ktimer_take(hipEvent_t* s, hipEvent_t* e) {
    if (!g_kt.armed) return false;
    g_kt.armed = false;
    *s = g_kt.start.back();
    *e = g_kt.stop.back();
    return true;
}

__global__ void raise_error_kernel(int* err, int code) {
    if (threadIdx.x == 0) report_device_error(err, code);
}
}  // namespace rf

extern "C" int rf_device_error(void) {
    rf::device_error_word();
    return rf::g_dev_err_host ? *rf::g_dev_err_host : 0;
}

extern "C" int rf_clear_device_error(void) {
    rf::device_error_word();
    if (rf::g_dev_err_host) *rf::g_dev_err_host = 0;
    return RF_OK;
}

extern "C" int rf_f16_range_flag(void) {
    rf::device_error_word();
    return rf::g_dev_err_host ? rf::g_dev_err_host[1] : 0;
}

extern "C" int rf_clear_f16_range_flag(void) {
    rf::device_error_word();
    if (rf::g_dev_err_host) rf::g_dev_err_host[1] = 0;
    return RF_OK;
}

extern "C" int rf_range_word_new(void** handle) {
    RF_REQUIRE(handle, "rf_range_word_new: null handle pointer");
    *handle = nullptr;
    void* h = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess) {
        rf::set_error("rf_range_word_new: hipHostMalloc failed");
        return RF_ERR_LAUNCH;
    }
    memset(h, 0, 64);
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipHostFree(h);
        rf::set_error("rf_range_word_new: hipHostGetDevicePointer failed");
        return RF_ERR_LAUNCH;
    }
    *handle = new rf::RangeWord{(volatile int*)h, (int*)d};
    return RF_OK;
}

extern "C" int rf_range_word_bind(void* handle) {
    rf::g_bound_range = handle ? ((rf::RangeWord*)handle)->dev : nullptr;
    return RF_OK;
}

extern "C" int rf_range_word_read(void* handle) {
    if (!handle) return rf_f16_range_flag();
    return *((rf::RangeWord*)handle)->host;
}

extern "C" int rf_range_word_clear(void* handle) {
    if (!handle) return rf_clear_f16_range_flag();
    *((rf::RangeWord*)handle)->host = 0;
    return RF_OK;
}

extern "C" int rf_range_word_free(void* handle) {
    if (!handle) return RF_OK;
    rf::RangeWord* r = (rf::RangeWord*)handle;
    if (rf::g_bound_range == r->dev) rf::g_bound_range = nullptr;
    (void)hipHostFree((void*)r->host);
    delete r;
    return RF_OK;
}

extern "C" int rf_debug_raise_device_error(int code, void* stream) {
    int* w = rf::device_error_word();
    RF_REQUIRE(w, "rf_debug_raise_device_error: no mapped error word");
    RF_LAUNCH(rf::raise_error_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, w, code);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        rf::set_error("rf_debug_raise_device_error: launch failed: %s", hipGetErrorString(e));
        return RF_ERR_LAUNCH;
    }
    return RF_OK;
}

extern "C" int rf_ktimer_arm(void) {
    hipEvent_t a = nullptr, b = nullptr;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
        rf::set_error("rf_ktimer_arm: hipEventCreate failed");
        return RF_ERR_LAUNCH;
    }
    if (rf::g_kt.armed) {  // the previous arm was never taken by a launch: drop its pair
        (void)hipEventDestroy(rf::g_kt.start.back());
        (void)hipEventDestroy(rf::g_kt.stop.back());
        rf::g_kt.start.pop_back();
        rf::g_kt.stop.pop_back();
    }
    rf::g_kt.start.push_back(a);
    rf::g_kt.stop.push_back(b);
    rf::g_kt.armed = true;
    return RF_OK;
}

extern "C" int rf_ktimer_read(float* ms, int max_n) {
    rf::KTimer& t = rf::g_kt;
    const int n = (int)t.start.size() - (t.armed ? 1 : 0);
    RF_REQUIRE(ms || max_n == 0, "rf_ktimer_read: null output");
    int rc = n;
    for (int i = 0; i < n; ++i) {
        float v = -1.f;
        if (hipEventSynchronize(t.stop[i]) != hipSuccess || hipEventElapsedTime(&v, t.start[i], t.stop[i]) != hipSuccess)
            v = -1.f;
        if (i < max_n) ms[i] = v;
        (void)hipEventDestroy(t.start[i]);
        (void)hipEventDestroy(t.stop[i]);
    }
    t.start.clear();
    t.stop.clear();
    t.armed = false;
    return rc;
}

extern "C" const char* rf_last_error(void) { return rf::g_err; }
extern "C" int rf_abi_version(void) { return RF_ABI_VERSION; }
extern "C" int rf_build_flags(void) {
#ifdef RF_STUDY
    return RF_BUILD_STUDY;
#else
    return 0;
#endif
}
