// Shared device/host helpers for librfhip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include "../../include/rf.h"

#define RF_DEV __device__ __forceinline__

typedef uint16_t bf16_t;  // raw bf16 bits in memory
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;  // MFMA A/B fragment (4 VGPRs)
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;  // fp16 MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))
#define GLB_PTR(T, p) ((const __attribute__((address_space(1))) T*)(p))

RF_DEV float bf16_to_f32(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even f32 -> bf16 (NaN-preserving via the hardware cvt when available)
RF_DEV bf16_t f32_to_bf16(float f) {
    __bf16 b = (__bf16)f;
    return *reinterpret_cast<bf16_t*>(&b);
}

RF_DEV uint32_t pack_bf16x2(float lo, float hi) {
    return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

// f32 -> the raw bits of a 16-bit operand: fp16 when f16, else bf16 (both round to nearest even)
RF_DEV uint16_t f32_to_16(float v, bool f16) {
    if (f16) {
        _Float16 h = (_Float16)v;
        return __builtin_bit_cast(uint16_t, h);
    }
    return f32_to_bf16(v);
}

// round-to-nearest-even f32 -> fp16 pair (overflow -> inf, like a torch .half() cast)
RF_DEV uint32_t pack_f16x2(float lo, float hi) {
    _Float16 a = (_Float16)lo, b = (_Float16)hi;
    return (uint32_t)*reinterpret_cast<uint16_t*>(&a) | ((uint32_t)*reinterpret_cast<uint16_t*>(&b) << 16);
}

// fp16 bits -> f32 (exact)
RF_DEV float f16_bits_to_f32(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }

RF_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

RF_DEV float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

RF_DEV void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// silu(x) = x / (1 + e^-x) on the hardware exp2 and reciprocal (~1 ulp each; every caller rounds the result
// to bf16/fp16 or adds it into an fp32 stream right after): 4 VALU ops instead of libm expf + an IEEE
// division (~25).  In the SwiGLU / conv epilogues the precise form cost 15 us of an 80 us GEMM.
RF_DEV float silu(float x) {
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
// (The conv epilogues use silu() too since round 4.  The libm form was once kept for the 256x256 engine conv tile,
// whose main loop spilled with the short one; the large DPT levels now run halo3_kernel<0> / conv3x3_c32_kernel,
// whose resource usage with silu() shows no scratch (hipcc -Rpass-analysis=kernel-resource-usage, round 5).)
// The DPT head's output transforms on the hardware exp2 (~1 ulp, v_exp_f32): ELU's negative branch
// alpha (e^y - 1) and the log decode 10^y - 1 (rendering_pipeline.py:119-123).  The libm expm1f / powf they
// replace cost ~70 VALU per output value, a third of the fused-head conv's time; the difference is ~1e-7
// absolute (y near 0) / relative, far inside the frame's 1e-3 bar.
RF_DEV float elu_fast(float y, float alpha) {
    return y > 0.f ? y : alpha * (__builtin_amdgcn_exp2f(y * 1.4426950408889634f) - 1.0f);
}
RF_DEV float pow10m1_fast(float y) { return __builtin_amdgcn_exp2f(y * 3.3219280948873623f) - 1.0f; }

// Device-side error word (host-pinned, mapped): a stream-K owner whose partial never arrived within the
// spin bound stores a code here instead of failing silently; every later entry point returns
// RF_ERR_DEVICE until rf_clear_device_error().  A vector (per-lane address) system-scope store.
RF_DEV void report_device_error(int* err, int code) {
    if (err) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// fp16 range flag (rf_f16_range_flag): a writer of fp16 operands that met a value it cannot represent (|x| >
// 65504, inf included) stores its code; the values it wrote are inf.  Plain vector system-scope store, like the
// error word (only ever taken on the failing path).
RF_DEV void report_f16_range(int* w, int code) {
    if (w) __hip_atomic_store(w, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// |x| <= 65504 (fp16's largest finite value) for a running max of |x| (an inf input fails it)
RF_DEV bool f16_in_range(float amax) { return amax <= 65504.0f; }
// running max of |a|, |b| (v_max3_f32 with abs source modifiers).  A NaN operand is ignored: NaNs come from NaN
// inputs (the reference propagates them too, and bf16 operands would not remove them), while an overflow is caught
// where the finite value that exceeds fp16's range is produced
RF_DEV float amax3(float m, float a, float b) {
    return __builtin_fmaxf(__builtin_fmaxf(m, __builtin_fabsf(a)), __builtin_fabsf(b));
}
#define RF_RANGE_GEMM 1      // rf_gemm_f16 / rf_gemm_bf16 RF_EPI_F16 / RF_EPI_SWIGLU_F16 outputs
#define RF_RANGE_RMSNORM 2   // rf_rmsnorm_f16
#define RF_RANGE_ATTN 4      // attention / Swin O written as fp16
#define RF_RANGE_CONV 8      // DPT fp16 planes (conv epilogue plane, rf_split_planes)
#define RF_DEVERR_SK_GEMM 1
#define RF_DEVERR_SK_ATTN 2
#define RF_DEVERR_SK_SCHED 3  // a stream-K range table that does not cover the launch's tiles (rejected in-kernel)
#define RF_DEVERR_SCENE_POS 4  // rf_scene_pos: a set holds more triangles than the max_tris it was launched for

// ------------------------------------------------------------------------------------------------------
// Stream-K block layout with forward progress (attention, GEMM and conv stream-K kernels).  The block that
// holds a unit's first iteration (the owner: it reaches that piece last in its range) waits for the partials
// of the blocks holding the unit's later iterations.  Every such wait goes to a block with a LOWER blockIdx,
// i.e. one dispatched earlier, and the awaited piece is always the first piece of its block's range (published
// before that block waits on anything).  So the lowest-numbered waiting block only ever waits on a block that
// is already resident and never blocks: the launch drains whatever else occupies the chip (two renders on two
// streams, or fewer CUs than blocks), with no co-residency assumption.
// Layout: blocks carry XCD labels x = blockIdx % nx (blocks b and b + 8 share an XCD's L2); the labels are
// cut into G groups and the units into G contiguous chunks, one per group, so no unit spans two groups (a
// group's blocks share one XCD's L2 when G = 8); inside a group the LOGICAL order, in which ranges are laid
// out, is DESCENDING blockIdx.  Logical index L = group base + rank; the host scheduler (rf_attn_schedule)
// and the kernels share these formulas.
#define RF_HD __host__ __device__ __forceinline__
struct SkLayout {
    int nwg, nx, G;
    RF_HD SkLayout(int nwg_, int64_t units) : nwg(nwg_), nx(nwg_ < 8 ? nwg_ : 8), G(1) {
        G = units < (int64_t)nx ? (int)(units > 0 ? units : 1) : nx;
    }
    RF_HD int cnt(int x) const { return (nwg - x + nx - 1) / nx; }       // blocks with label x
    RF_HD int xlo(int g) const { return (g * nx + G - 1) / G; }          // first label of group g
    RF_HD int group_of(int x) const { return x * G / nx; }
    RF_HD int base(int g) const {  // first logical index of group g
        int s = 0;
        for (int x = 0; x < xlo(g); ++x) s += cnt(x);
        return s;
    }
    RF_HD int size(int g) const {
        int s = 0;
        for (int x = xlo(g); x < xlo(g + 1); ++x) s += cnt(x);
        return s;
    }
    // logical index of block hw: its group's base + the number of the group's blocks with a larger blockIdx
    RF_HD int logical(int hw, int* grp = nullptr) const {
        const int x = hw % nx, g = group_of(x);
        int rank = 0;
        for (int y = xlo(g); y < xlo(g + 1); ++y) {
            const int jmin = hw - y >= 0 ? (hw - y) / nx + 1 : 0;  // blocks nx j + y > hw
            const int c = cnt(y);
            rank += c > jmin ? c - jmin : 0;
        }
        if (grp) *grp = g;
        return base(g) + rank;
    }
    // equal split (no host schedule): group g takes units [U g / G, U (g+1) / G), its blocks equal shares of
    // their iterations (units of `per` iterations each)
    RF_HD void equal_range(int L, int g, int64_t units, int64_t per, int64_t& b, int64_t& e) const {
        const int64_t u0 = units * g / G, u1 = units * (g + 1) / G;
        const int64_t t0 = u0 * per, tn = (u1 - u0) * per;
        const int nb = size(g), li = L - base(g);
        b = t0 + tn * li / nb;
        e = t0 + tn * (li + 1) / nb;
    }
};

// ------------------------------------------------------------------------- host side
namespace rf {
// stream-K attention geometry shared by the kernel (attention.hip) and its host schedule (attn_sched.cpp)
constexpr int ATTN_KT = 64;         // keys per tile
constexpr int ATTN_QB = 256;        // query rows per unit (8 waves x 32)
constexpr int ATTN_MAX_GRID = 512;  // workgroups per launch (partial slots / flags in the workspace)
void set_error(const char* fmt, ...);
int check_launch(const char* what);
int* device_error_word();  // device pointer of the mapped error word (nullptr if it could not be allocated)
int* range_word();         // device pointer of the mapped fp16 range flag (rf_f16_range_flag)
// Study-only kernels (measured slower than the defaults, or ablation builds whose results are garbage) are compiled
// only with -DRF_STUDY (make study -> librfhip_study.so); a production build asked for one refuses: sets the error
// and returns RF_ERR_UNSUPPORTED (capi.cpp)
int study_only(const char* what);
int spin_limit();          // stream-K hand-off spin bound (RF_SPIN_LIMIT, default 2^24 polls)
// fresh hand-off flag value (>= 1) for a stream-K launch on the flag area [flags, flags + bytes); re-zeroes the
// area on the stream when the epoch sequence wraps (capi.cpp)
int next_epoch(void* flags, size_t bytes, hipStream_t st);
// Kernel timer (rf_ktimer_arm / rf_ktimer_read): when armed, the next library launch takes a start/stop event
// pair that the dispatch packet itself timestamps (hipExtLaunchKernel), so the measured duration is the
// kernel's own, as in a rocprofv3 kernel trace, with no extra packets in the queue.
bool ktimer_take(hipEvent_t* start, hipEvent_t* stop);
}  // namespace rf

#define RF_REQUIRE(cond, ...)                          \
    do {                                               \
        if (!(cond)) {                                 \
            rf::set_error(__VA_ARGS__);                \
            return RF_ERR_INVALID;                     \
        }                                              \
    } while (0)

// Every library launch goes through RF_LAUNCH: a plain launch unless the kernel timer is armed.
#define RF_LAUNCH(kernel, grid, block, shmem, stream, ...)                                                  \
    do {                                                                                                 \
        hipEvent_t rf_ev0_, rf_ev1_;                                                                     \
        if (rf::ktimer_take(&rf_ev0_, &rf_ev1_))                                                         \
            hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, rf_ev0_, rf_ev1_, 0, __VA_ARGS__); \
        else                                                                                             \
            hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                         \
    } while (0)
