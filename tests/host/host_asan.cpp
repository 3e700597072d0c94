// Host-side memory and undefined-behaviour check of librfhip's pointer-heavy host code (SURVEY §5 "Race
// detection / sanitizers": AddressSanitizer for host C++; GPU sanitizers are not available on this pool).
// Built by `make -C renderformer_amd/csrc asan`: capi.cpp, stage.cpp and attn_sched.cpp with
// -fsanitize=address,undefined on the host side (hipcc -Xarch_host), linked with the library's other objects and
// run WITHOUT a GPU (tests/test_host_asan.py).  It drives:
//   * rf_attn_schedule over random varlen problem tables (the cost-balanced stream-K ranges: bisection, backward
//     fill, unit lookup), checking the table invariants the kernel relies on;
//   * the stream-K epoch table (rf::next_epoch) through generation wraps (RF_EPOCH_BITS=2), where the flag area
//     re-zero fails without a device and the launch must be refused (epoch 0);
//   * the per-render fp16 range words and the process words (allocation failure paths);
//   * the stage-level descriptor walkers (rf_encoder_forward / rf_decoder_forward / rf_decoder_workspace_bytes)
//     on valid and malformed descriptors: validation, layout arithmetic, layer / tap walks up to the first launch.
// Exit status 0 and no sanitizer report = pass.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "rf.h"

namespace rf {
int next_epoch(void* flags, size_t bytes, hipStream_t st);  // capi.cpp
}

static int g_fails = 0;
#define CHECK(c)                                                                   \
    do {                                                                           \
        if (!(c)) {                                                                \
            fprintf(stderr, "CHECK failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fails;                                                             \
        }                                                                          \
    } while (0)

static void schedule_tables() {
    std::mt19937 rng(1234);
    int cases = 0;
    for (int seed = 0; seed < 300; ++seed) {
        const int n_prob = 1 + (int)(rng() % 40);
        const int heads = 1 + (int)(rng() % 16);
        const int grid = 1 + (int)(rng() % 512);
        std::vector<int32_t> prob(5 * n_prob);
        int64_t total = 0;
        for (int i = 0; i < n_prob; ++i) {
            const int ql = (int)(rng() % 3000), kl = (rng() % 5 == 0) ? 0 : (int)(rng() % 12000);
            prob[5 * i + 0] = (int)(rng() % 1000);
            prob[5 * i + 1] = ql;
            prob[5 * i + 2] = (int)(rng() % 1000);
            prob[5 * i + 3] = kl;
            prob[5 * i + 4] = (int)(rng() % 1000);
            const int64_t nt = (kl + 63) / 64, nu = nt > 0 ? (int64_t)heads * ((ql + 255) / 256) : 0;
            total += nu * nt;
        }
        std::vector<int64_t> b(grid + 1, -7);
        const int rc = rf_attn_schedule(prob.data(), n_prob, heads, grid, b.data());
        CHECK(rc == RF_OK);
        if (rc != RF_OK) continue;
        CHECK(b[0] == 0 && b[grid] == total);
        for (int w = 0; w < grid; ++w) CHECK(b[w] <= b[w + 1]);
        ++cases;
    }
    // the bench shape (stage 1: S = 5,649, 8 heads, 256 workgroups) and config 5's cross-attention (24 views)
    {
        const int32_t p1[5] = {0, 5649, 0, 5649, 0};
        std::vector<int64_t> b(257);
        CHECK(rf_attn_schedule(p1, 1, 8, 256, b.data()) == RF_OK);
        CHECK(b[0] == 0 && b[256] == 8 * 23 * 89);
        std::vector<int32_t> p2;
        for (int v = 0; v < 24; ++v) {
            const int32_t row[5] = {v * 16384, 16384, 0, 5649, 0};
            p2.insert(p2.end(), row, row + 5);
        }
        CHECK(rf_attn_schedule(p2.data(), 24, 8, 256, b.data()) == RF_OK);
        CHECK(b[256] == (int64_t)24 * 8 * 64 * 89);
    }
    // malformed arguments are refused, nothing is written past the table
    {
        const int32_t bad[5] = {0, -1, 0, 10, 0};
        std::vector<int64_t> b(9);
        CHECK(rf_attn_schedule(bad, 1, 8, 8, b.data()) == RF_ERR_INVALID);
        const int32_t ok[5] = {0, 100, 0, 100, 0};
        CHECK(rf_attn_schedule(ok, 1, 8, 0, b.data()) == RF_ERR_INVALID);
        CHECK(rf_attn_schedule(ok, 1, 8, 513, b.data()) == RF_ERR_INVALID);
        CHECK(rf_attn_schedule(nullptr, 1, 8, 8, b.data()) == RF_ERR_INVALID);
        CHECK(strlen(rf_last_error()) > 0);
    }
    printf("schedule: %d random tables + bench / config-5 shapes + malformed arguments\n", cases);
}

static void epochs() {
    setenv("RF_EPOCH_BITS", "2", 1);
    std::vector<int> area(512, 0);
    int zeros = 0, seen = 0;
    for (int i = 0; i < 40; ++i) {  // 2-bit epochs: a generation wrap every 4 launches (re-zero needs a device here)
        const int e = rf::next_epoch(area.data(), area.size() * sizeof(int), nullptr);
        CHECK(e >= 0 && e <= 4);
        zeros += e == 0;
        seen += e > 0;
    }
    unsetenv("RF_EPOCH_BITS");
    CHECK(seen >= 4);  // the first generation is served without a re-zero
    printf("epochs: %d served, %d refused at a wrap whose re-zero failed\n", seen, zeros);
}

static void range_words() {
    void* h = (void*)0x1;
    const int rc = rf_range_word_new(&h);
    if (rc == RF_OK) {  // (a machine with a device)
        CHECK(h != nullptr && rf_range_word_read(h) == 0);
        CHECK(rf_range_word_bind(h) == RF_OK && rf_range_word_bind(nullptr) == RF_OK);
        CHECK(rf_range_word_free(h) == RF_OK);
    } else {
        CHECK(h == nullptr);
    }
    CHECK(rf_range_word_new(nullptr) == RF_ERR_INVALID);
    CHECK(rf_range_word_bind(nullptr) == RF_OK && rf_range_word_free(nullptr) == RF_OK);
    CHECK(rf_range_word_read(nullptr) >= 0 && rf_range_word_clear(nullptr) == RF_OK);
    CHECK(rf_device_error() >= 0 && rf_clear_device_error() == RF_OK);
    printf("range words: allocation %s\n", rc == RF_OK ? "succeeded" : "refused (no device)");
}

static void stages() {
    const int L = 3, T = 300, D = 256, H = 2, F = 512;
    // host stand-ins for the device buffers: the walkers never dereference them on the host
    std::vector<char> dummy(1 << 16);
    void* p = dummy.data();
    std::vector<rf_encoder_layer> el(L);
    for (auto& l : el) {
        l.attn_norm = (const float*)p;
        l.w_qkv = p;
        l.qk_norm = (const float*)p;
        l.w_out = p;
        l.ffn_norm = (const float*)p;
        l.w13 = p;
        l.w2 = p;
    }
    void* ws = aligned_alloc(256, 1 << 16);
    rf_encoder_desc e{};
    e.n_layers = L;
    e.rows = T;
    e.dim = D;
    e.n_heads = H;
    e.ffn_dim = F;
    e.operand_dtype = RF_DT_F16;
    e.eps = 1e-6f;
    e.layers = el.data();
    e.pos = (const float*)p;
    e.ld_pos = 9;
    e.freqs = (const float*)p;
    e.n_freqs = 6;
    e.problems = (const int32_t*)p;
    e.n_problems = 1;
    e.workspace = ws;
    e.attn_ws = p;
    float* x = (float*)p;
    CHECK(rf_encoder_forward(x, D, nullptr, nullptr) == RF_ERR_INVALID);
    CHECK(rf_encoder_workspace_bytes(T, D, F, RF_DT_F16) > 0 && rf_encoder_workspace_bytes(0, D, F, 0) == 0);
    const int rc_e = rf_encoder_forward(x, D, &e, nullptr);  // valid: runs to the first launch (fails: no device)
    CHECK(rc_e != RF_ERR_INVALID);
    rf_encoder_desc bad = e;
    bad.dim = 250;
    CHECK(rf_encoder_forward(x, D, &bad, nullptr) == RF_ERR_INVALID);
    bad = e;
    bad.layers = nullptr;
    CHECK(rf_encoder_forward(x, D, &bad, nullptr) == RF_ERR_INVALID);
    std::vector<rf_encoder_layer> el_null = el;
    el_null[L - 1].w2 = nullptr;
    bad = e;
    bad.layers = el_null.data();
    CHECK(rf_encoder_forward(x, D, &bad, nullptr) == RF_ERR_INVALID);
    bad = e;
    bad.n_layers = 0;
    CHECK(rf_encoder_forward(x, D, &bad, nullptr) == RF_OK);

    std::vector<rf_decoder_layer> dl(L);
    for (auto& l : dl) {
        memset(&l, 0, sizeof(l));
        l.query_norm = (const float*)p;
        l.w_q = p;
        l.q_norm = (const float*)p;
        l.w_out = p;
        l.self_norm = (const float*)p;
        l.w_self_in = p;
        l.self_qk_norm = (const float*)p;
        l.w_self_out = p;
        l.ffn_norm = (const float*)p;
        l.w13 = p;
        l.w2 = p;
    }
    std::vector<rf_decoder_tap> taps(2);
    for (int i = 0; i < 2; ++i) {
        taps[i].layer = i + 1;
        taps[i].p_ld = D;
        taps[i].p_hi = p;
        taps[i].p_lo = nullptr;
    }
    rf_decoder_desc d{};
    d.n_layers = L;
    d.rows = 64 * 4;
    d.dim = D;
    d.n_heads = H;
    d.ffn_dim = F;
    d.operand_dtype = RF_DT_F16;
    d.eps = 1e-6f;
    d.layers = dl.data();
    d.ctx = (const float*)p;
    d.ld_ctx = D;
    d.ctx_rows = T;
    d.ctx_dim = D;
    d.ctx_norm = (const float*)p;
    d.w_kv_all = p;
    d.kv_rows = T;
    d.kv_src_rows = (const int32_t*)p;
    d.kv_pos = (const float*)p;
    d.ld_kv_pos = 9;
    d.k_batch = 1;
    d.freqs = (const float*)p;
    d.n_freqs = 6;
    d.ray_pos = (const float*)p;
    d.ld_ray_pos = 9;
    d.ray_pos_div = 64;
    d.cross_problems = (const int32_t*)p;
    d.n_cross = 4;
    d.swin = 1;
    d.n_images = 4;
    d.grid_h = 8;
    d.grid_w = 8;
    d.window = 8;
    d.shift = 4;
    d.taps = taps.data();
    d.n_taps = 2;
    d.workspace = ws;
    d.attn_ws = p;
    const int64_t wsb = rf_decoder_workspace_bytes(&d);
    CHECK(wsb > 0);
    CHECK(rf_decoder_workspace_bytes(nullptr) == 0);
    CHECK(rf_decoder_forward(x, D, nullptr, nullptr) == RF_ERR_INVALID);
    const int rc_d = rf_decoder_forward(x, D, &d, nullptr);
    CHECK(rc_d != RF_ERR_INVALID);
    rf_decoder_desc bd = d;
    bd.n_taps = 2;
    std::vector<rf_decoder_tap> bad_taps = taps;
    bad_taps[1].layer = L + 5;  // a tap after the last layer
    bd.taps = bad_taps.data();
    CHECK(rf_decoder_forward(x, D, &bd, nullptr) == RF_ERR_INVALID);
    bd = d;
    bd.swin = 1;
    bd.grid_h = 7;  // not a multiple of the window
    CHECK(rf_decoder_forward(x, D, &bd, nullptr) == RF_ERR_INVALID);
    free(ws);
    printf("stages: encoder rc %d, decoder rc %d (valid descriptors run to the first launch), workspace %lld B\n",
           rc_e, rc_d, (long long)wsb);
}

int main() {
    schedule_tables();
    epochs();
    range_words();
    stages();
    float ms[4];
    CHECK(rf_ktimer_read(ms, 4) >= 0);
    if (g_fails) {
        fprintf(stderr, "%d checks failed\n", g_fails);
        return 1;
    }
    printf("host_asan: all checks passed\n");
    return 0;
}
