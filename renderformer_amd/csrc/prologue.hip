// Pre/post-processing kernels around the two transformer stages.
//
// These are all HBM/latency-bound elementwise passes; the point of having them
// on the device is that the product path never round-trips scene data through
// the host and never materialises the reference's intermediate
// repeat_interleave / cat / padded tensors.
#include <math.h>

#include "common.h"

namespace {

// ----------------------------------------------------------------------------- texture
// rendering_pipeline.py:67-68 (in-place log10(x+1) of the emission channels, all rows)
// + renderformer.py:145-147 flatten to [N, C*P*P], compacted to valid rows, bf16.
__global__ __launch_bounds__(256) void texture_pack_kernel(float* __restrict__ tex, int channels, int patch_elems,
                                                           int log_from, const int32_t* __restrict__ dst_row,
                                                           bf16_t* __restrict__ out, int64_t ldo, const int* gate) {
    if (gate && *gate == 0) return;
    const int64_t r = blockIdx.x;
    const int n4 = channels * patch_elems / 4;
    float4* row = reinterpret_cast<float4*>(tex + r * (int64_t)channels * patch_elems);
    const int d = dst_row ? dst_row[r] : (int)r;
    bf16_t* o = d >= 0 ? out + (int64_t)d * ldo : nullptr;
    for (int i = threadIdx.x; i < n4; i += blockDim.x) {
        float4 v = row[i];
        if ((i * 4) / patch_elems >= log_from) {
            v.x = log10f(v.x + 1.0f);
            v.y = log10f(v.y + 1.0f);
            v.z = log10f(v.z + 1.0f);
            v.w = log10f(v.w + 1.0f);
            row[i] = v;
        }
        if (o) {
            uint2 pk;
            pk.x = pack_bf16x2(v.x, v.y);
            pk.y = pack_bf16x2(v.z, v.w);
            *reinterpret_cast<uint2*>(o + i * 4) = pk;
        }
    }
}

// Texture encoder fast path.  Every texture written by scene_processor/to_h5.py:41-66 is, per triangle and
// channel, one constant times the fixed patch mask {(i, j) : i + j <= 32} of the 32x32 patch, so the
// texture Linear(C*1024 -> D) of renderformer.py:145-147 reduces exactly to a C-wide product with the
// mask-summed weights.  The scan proves that form for every valid row (exact float
// compares after the in-place log encode; NaN fails) and raises *flag otherwise; the consumers are gated
// on the flag on the device, so no host round trip decides the path.
constexpr int TEX_SIDE = 32;  // to_h5.py:41

RF_DEV bool tex_in_mask(int e) { return (e >> 5) + (e & 31) <= TEX_SIDE; }

// one block per texture row (all n_rows rows are log-encoded, like rendering_pipeline.py:67-68); thread t
// owns texels 4t..4t+3 of every channel (patch row t >> 3)
__global__ __launch_bounds__(256) void texture_scan_kernel(float* __restrict__ tex, int channels, int log_from,
                                                           const int32_t* __restrict__ dst_row,
                                                           float* __restrict__ coef, int64_t ldc, int* flag,
                                                           int* flag_clear) {
    const int64_t r = blockIdx.x;
    const int t = threadIdx.x;
    if (r == 0 && t == 0 && flag_clear) *flag_clear = 0;  // the other frame-parity flag (rf_texture_scan2)
    float* base = tex + r * (int64_t)channels * (TEX_SIDE * TEX_SIDE);
    __shared__ float c_raw[32];
    if (t < channels) c_raw[t] = base[t * TEX_SIDE * TEX_SIDE];  // texel (0, 0): inside the mask
    __syncthreads();  // read before any thread rewrites it in place
    const int e0 = 4 * t;
    const bool m0 = tex_in_mask(e0), m1 = tex_in_mask(e0 + 1), m2 = tex_in_mask(e0 + 2), m3 = tex_in_mask(e0 + 3);
    bool ok = true;
    for (int ch = 0; ch < channels; ++ch) {
        float4* p4 = reinterpret_cast<float4*>(base + ch * TEX_SIDE * TEX_SIDE) + t;
        float4 v = *p4;
        float c = c_raw[ch];
        if (ch >= log_from) {
            v.x = log10f(v.x + 1.0f);
            v.y = log10f(v.y + 1.0f);
            v.z = log10f(v.z + 1.0f);
            v.w = log10f(v.w + 1.0f);
            *p4 = v;
            c = log10f(c + 1.0f);  // the same op on the same input as texel (0, 0) above: bit-identical
        }
        ok = ok && v.x == (m0 ? c : 0.f) && v.y == (m1 ? c : 0.f) && v.z == (m2 ? c : 0.f) && v.w == (m3 ? c : 0.f);
    }
    const int d = dst_row ? dst_row[r] : (int)r;
    if (d < 0) return;  // block-uniform: padded rows are only log-encoded
    if (!__syncthreads_and(ok) && t == 0) *flag = 1;
    if (t < channels) {
        const float c = c_raw[t];
        coef[(int64_t)d * ldc + t] = t >= log_from ? log10f(c + 1.0f) : c;
    }
}

// out[r, o] = bias[o] + sum_c coef[r, c] * wsum[c, o]   (fast path; no-op when *flag != 0).  Thread t keeps
// columns 4t..4t+3 of wsum (<= 16 channels) in registers for TL_ROWS rows; the rows' coefficients go
// through LDS, so wsum is read once per block (not once per row).
constexpr int TL_ROWS = 16, TL_MAXC = 16;
__global__ __launch_bounds__(256) void texture_linear_kernel(const float* __restrict__ coef, int64_t ldc, int rows,
                                                             int channels, const float* __restrict__ wsum,
                                                             const float* __restrict__ bias, float* __restrict__ out,
                                                             int64_t ldo, int n, const int* flag) {
    if (*flag != 0) return;
    __shared__ float cs[TL_ROWS][TL_MAXC];
    const int r0 = blockIdx.x * TL_ROWS;
    const int t = threadIdx.x;
    {
        const int rr = t / TL_MAXC, c = t % TL_MAXC;
        cs[rr][c] = (r0 + rr < rows && c < channels) ? coef[(int64_t)(r0 + rr) * ldc + c] : 0.f;
    }
    __syncthreads();
    for (int o = 4 * t; o < n; o += 1024) {
        float4 w[TL_MAXC];
#pragma unroll
        for (int c = 0; c < TL_MAXC; ++c)
            w[c] = c < channels ? *reinterpret_cast<const float4*>(wsum + (int64_t)c * n + o) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 b4 = bias ? *reinterpret_cast<const float4*>(bias + o) : make_float4(0.f, 0.f, 0.f, 0.f);
        for (int rr = 0; rr < TL_ROWS && r0 + rr < rows; ++rr) {
            float4 acc = b4;
#pragma unroll
            for (int c = 0; c < TL_MAXC; ++c) {
                const float k = cs[rr][c];
                acc.x = fmaf(k, w[c].x, acc.x);
                acc.y = fmaf(k, w[c].y, acc.y);
                acc.z = fmaf(k, w[c].z, acc.z);
                acc.w = fmaf(k, w[c].w, acc.w);
            }
            *reinterpret_cast<float4*>(out + (int64_t)(r0 + rr) * ldo + o) = acc;
        }
    }
}

// ----------------------------------------------------------------------------- vertex normals
// NeRFEncoding(in_dim=9, L, include_input) (nerf_encoding.py:76-84): [x, sin(x_d 2^l), sin(x_d 2^l + pi/2)]
__global__ __launch_bounds__(256) void vn_encode_kernel(const float* __restrict__ vn, int64_t n_rows,
                                                        const int32_t* __restrict__ dst_row, int L,
                                                        bf16_t* __restrict__ out, int64_t ldo, int f16) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const int d = dst_row ? dst_row[r] : (int)r;
    if (d < 0) return;
    const float* x = vn + r * 9;
    const int n_sin = 9 * L;
    for (int e = lane; e < ldo; e += 64) {
        float val = 0.f;
        if (e < 9) {
            val = x[e];
        } else if (e < 9 + 2 * n_sin) {
            const int j = (e - 9) % n_sin;
            const float s = x[j / L] * exp2f((float)(j % L));
            val = (e - 9) < n_sin ? sinf(s) : sinf(s + 1.5707963267948966f);
        }
        out[(int64_t)d * ldo + e] = f32_to_16(val, f16);
    }
}

// ----------------------------------------------------------------------------- rays
// RayGenerator (ray_generator.py:31-50) + rearrange 'b (h p1) (w p2) c -> b (h w) (c p1 p2)'
__global__ __launch_bounds__(256) void ray_tokens_kernel(const float* __restrict__ c2w, const float* __restrict__ fov,
                                                         int res, int patch, bf16_t* __restrict__ out,
                                                         float* __restrict__ ray_pos, int f16) {
    const int view = blockIdx.y;
    const int pix = blockIdx.x * blockDim.x + threadIdx.x;
    const float* m = c2w + view * 16;
    if (pix == 0 && ray_pos) {
        for (int c = 0; c < 9; ++c) ray_pos[view * 9 + c] = m[(c % 3) * 4 + 3];
    }
    if (pix >= res * res) return;
    const int y = pix / res, x = pix % res;
    const float fov_rad = fov[view] / 180.0f * 3.14159265358979323846f;
    const float f = (float)res / 2.0f / tanf(0.5f * fov_rad);
    const float c = (float)res / 2.0f;
    const float dx = ((float)x + 0.5f - c) / f;
    const float dy = -(((float)y + 0.5f - c) / f);
    const float dz = -1.0f;
    float r0 = dx * m[0] + dy * m[1] + dz * m[2];
    float r1 = dx * m[4] + dy * m[5] + dz * m[6];
    float r2 = dx * m[8] + dy * m[9] + dz * m[10];
    const float nrm = fmaxf(sqrtf(r0 * r0 + r1 * r1 + r2 * r2), 1e-12f);
    r0 /= nrm;
    r1 /= nrm;
    r2 /= nrm;
    const int pw = res / patch;
    const int tok = (y / patch) * pw + (x / patch);
    const int pp = patch * patch;
    const int feat = (y % patch) * patch + (x % patch);
    bf16_t* o = out + ((int64_t)view * pw * pw + tok) * (3 * pp);
    o[feat] = f32_to_16(r0, f16);
    o[pp + feat] = f32_to_16(r1, f16);
    o[2 * pp + feat] = f32_to_16(r2, f16);
}

__global__ __launch_bounds__(256) void patchify_rays_kernel(const float* __restrict__ rays, int res, int patch,
                                                            bf16_t* __restrict__ out, int f16) {
    const int view = blockIdx.y;
    const int pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= res * res) return;
    const int y = pix / res, x = pix % res;
    const float* r = rays + ((int64_t)view * res * res + pix) * 3;
    const int pw = res / patch, pp = patch * patch;
    const int tok = (y / patch) * pw + (x / patch);
    const int feat = (y % patch) * patch + (x % patch);
    bf16_t* o = out + ((int64_t)view * pw * pw + tok) * (3 * pp);
    o[feat] = f32_to_16(r[0], f16);
    o[pp + feat] = f32_to_16(r[1], f16);
    o[2 * pp + feat] = f32_to_16(r[2], f16);
}

// ----------------------------------------------------------------------------- RoPE positions
// trans_to_cam_coord (transform.py:24-27: p -> R^T p - R^T t) and process_tri_vpos_list
// (renderformer.py:111-122: register rows = masked mean position, averaged over the 3 vertices).
// Triangle positions + register-token centres in two launches (deterministic, no atomics):
//   1. scene_pos_tri_kernel, grid (ceil(max_n / 256), sets): one thread per triangle writes its (camera-frame)
//      9 coordinates and each block writes the 9 sums of its triangles to partial[set][block];
//   2. scene_pos_center_kernel, one wave per set: sums the block partials in block order and writes the
//      n_reg centre rows (renderformer.py:113-116: mean over valid triangles / (n + 1e-5), vertex-averaged).
// (one 1,024-thread block per set took ~19 us: each thread walked ~6 triangles through dependent loads)
__global__ __launch_bounds__(256) void scene_pos_tri_kernel(const float* __restrict__ tris,
                                                            const int32_t* __restrict__ valid_idx,
                                                            const int32_t* __restrict__ scene_off,
                                                            const float* __restrict__ c2w, int n_views, int n_reg,
                                                            float* __restrict__ pos_out,
                                                            const int32_t* __restrict__ set_off,
                                                            float* __restrict__ partial) {
    __shared__ float red[4][9];
    const int set = blockIdx.y;
    const int scene = c2w ? set / n_views : set;
    const int t0 = scene_off[scene], n = scene_off[scene + 1] - t0;
    const int i = blockIdx.x * 256 + threadIdx.x;
    float v[9];
    for (int c = 0; c < 9; ++c) v[c] = 0.f;
    if (i < n) {
        const float* src = tris + (int64_t)valid_idx[t0 + i] * 9;
        for (int c = 0; c < 9; ++c) v[c] = src[c];
        if (c2w) {
            const float* m = c2w + set * 16;
            float rt[9], tinv[3];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) rt[a * 3 + b] = m[b * 4 + a];
            for (int a = 0; a < 3; ++a) tinv[a] = -(rt[a * 3 + 0] * m[3] + rt[a * 3 + 1] * m[7] + rt[a * 3 + 2] * m[11]);
            float w[9];
            for (int vert = 0; vert < 3; ++vert)
                for (int a = 0; a < 3; ++a)
                    w[vert * 3 + a] = rt[a * 3 + 0] * v[vert * 3 + 0] + rt[a * 3 + 1] * v[vert * 3 + 1] +
                                      rt[a * 3 + 2] * v[vert * 3 + 2] + tinv[a];
            for (int c = 0; c < 9; ++c) v[c] = w[c];
        }
        float* dst = pos_out + (int64_t)(set_off[set] + n_reg + i) * 9;
        for (int c = 0; c < 9; ++c) dst[c] = v[c];
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int c = 0; c < 9; ++c) {
        const float sm = wave_sum(v[c]);
        if (lane == 0) red[wave][c] = sm;
    }
    __syncthreads();
    if (threadIdx.x < 9)
        partial[((int64_t)set * gridDim.x + blockIdx.x) * 9 + threadIdx.x] =
            (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

__global__ __launch_bounds__(64) void scene_pos_center_kernel(const int32_t* __restrict__ scene_off, int n_views,
                                                              int has_c2w, int n_reg, int n_blocks,
                                                              const float* __restrict__ partial,
                                                              float* __restrict__ pos_out,
                                                              const int32_t* __restrict__ set_off, int* err) {
    const int set = blockIdx.x;
    const int scene = has_c2w ? set / n_views : set;
    const int n = scene_off[scene + 1] - scene_off[scene];
    // blocks that held triangles of this set (the rest wrote zeros).  A set with more triangles than the
    // max_tris the caller sized the launch for would read the next set's partials and leave positions past
    // n_blocks * 256 unwritten: clamp to this set's slots and raise the device error word instead.
    int nb = (n + 255) / 256;
    if (nb > n_blocks) {
        nb = n_blocks;
        if (threadIdx.x == 0) report_device_error(err, RF_DEVERR_SCENE_POS);
    }
    // the partials of 64 blocks at a time come in with one load round trip (lane b loads block b's 9 sums into
    // LDS), then lane c < 9 adds them in block order: the same sums in the same order as a serial loop (whose
    // ~200 dependent loads took 11 us), so the result is bit-identical to it
    __shared__ float part_lds[64][9];
    const int lane = threadIdx.x;
    float acc = 0.f;  // lane c < 9: channel c
    for (int b0 = 0; b0 < nb; b0 += 64) {
        const int b = b0 + lane;
        if (b < nb) {
            const float* src = partial + ((int64_t)set * n_blocks + b) * 9;
#pragma unroll
            for (int c = 0; c < 9; ++c) part_lds[lane][c] = src[c];
        }
        __syncthreads();
        if (lane < 9) {
            const int m = min(64, nb - b0);
            for (int j = 0; j < m; ++j) acc += part_lds[j][lane];
        }
        __syncthreads();
    }
    __shared__ float tot_lds[9];
    if (lane < 9) tot_lds[lane] = acc / ((float)n + 1e-5f);
    __syncthreads();
    float tot[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) tot[c] = tot_lds[c];
    for (int t = threadIdx.x; t < n_reg * 9; t += 64) {
        const int k = t % 3;
        pos_out[(int64_t)set_off[set] * 9 + t] = (tot[k] + tot[3 + k] + tot[6 + k]) / 3.0f;
    }
}

// ----------------------------------------------------------------------------- output
// ELU(alpha) (view_transformer.py:86,122), permute [n,c,h,w] -> [n,h,w,c] and 10^x - 1 (rendering_pipeline.py:119-123)
__global__ __launch_bounds__(256) void hdr_output_kernel(const float* __restrict__ logits, float* __restrict__ out,
                                                         int64_t n_pix, int c, int hw, float alpha, int log_decode,
                                                         int channels_last) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pix) return;
    const int64_t img = i / hw, px = i % hw;
    for (int ch = 0; ch < c; ++ch) {
        float y = logits[(img * c + ch) * hw + px];
        y = y > 0.f ? y : alpha * expm1f(y);
        if (log_decode) y = powf(10.0f, y) - 1.0f;
        out[channels_last ? i * c + ch : (img * c + ch) * hw + px] = y;
    }
}

}  // namespace

extern "C" int rf_texture_pack(float* texture, int64_t n_rows, int channels, int patch_elems, int log_channels,
                               const int32_t* dst_row, void* out, int64_t ldo, void* stream) {
    RF_REQUIRE(texture && out, "rf_texture_pack: null pointer");
    RF_REQUIRE(patch_elems % 4 == 0 && ((uintptr_t)texture & 15) == 0, "rf_texture_pack: need 16-B aligned rows");
    RF_REQUIRE(ldo >= (int64_t)channels * patch_elems && ldo % 4 == 0, "rf_texture_pack: bad ldo");
    RF_REQUIRE(n_rows < (1ll << 31), "rf_texture_pack: too many rows");
    if (n_rows <= 0) return RF_OK;
    RF_LAUNCH(texture_pack_kernel, dim3((unsigned)n_rows), dim3(256), 0, (hipStream_t)stream, texture,
                       channels, patch_elems, channels - log_channels, dst_row, (bf16_t*)out, ldo, nullptr);
    return rf::check_launch("rf_texture_pack");
}

extern "C" int rf_texture_pack_if(const int* flag, float* texture, int64_t n_rows, int channels, int patch_elems,
                                  int log_channels, const int32_t* dst_row, void* out, int64_t ldo, void* stream) {
    RF_REQUIRE(flag && texture && out, "rf_texture_pack_if: null pointer");
    RF_REQUIRE(patch_elems % 4 == 0 && ((uintptr_t)texture & 15) == 0, "rf_texture_pack_if: need 16-B aligned rows");
    RF_REQUIRE(ldo >= (int64_t)channels * patch_elems && ldo % 4 == 0, "rf_texture_pack_if: bad ldo");
    RF_REQUIRE(n_rows < (1ll << 31), "rf_texture_pack_if: too many rows");
    if (n_rows <= 0) return RF_OK;
    RF_LAUNCH(texture_pack_kernel, dim3((unsigned)n_rows), dim3(256), 0, (hipStream_t)stream, texture,
                       channels, patch_elems, channels - log_channels, dst_row, (bf16_t*)out, ldo, flag);
    return rf::check_launch("rf_texture_pack_if");
}

extern "C" int rf_texture_scan(float* texture, int64_t n_rows, int channels, int patch_elems, int log_channels,
                               const int32_t* dst_row, float* coef, int64_t ldc, int* flag, void* stream) {
    RF_REQUIRE(texture && coef && flag, "rf_texture_scan: null pointer");
    RF_REQUIRE(patch_elems == TEX_SIDE * TEX_SIDE, "rf_texture_scan: patch_elems must be %d", TEX_SIDE * TEX_SIDE);
    RF_REQUIRE(channels >= 1 && channels <= 32 && ldc >= channels, "rf_texture_scan: bad channels/ldc");
    RF_REQUIRE(log_channels >= 0 && log_channels <= channels, "rf_texture_scan: bad log_channels");
    RF_REQUIRE(((uintptr_t)texture & 15) == 0, "rf_texture_scan: texture must be 16-B aligned");
    RF_REQUIRE(n_rows < (1ll << 31), "rf_texture_scan: too many rows");
    if (hipMemsetAsync(flag, 0, sizeof(int), (hipStream_t)stream) != hipSuccess) {
        rf::set_error("rf_texture_scan: flag reset failed");
        return RF_ERR_LAUNCH;
    }
    if (n_rows <= 0) return RF_OK;
    RF_LAUNCH(texture_scan_kernel, dim3((unsigned)n_rows), dim3(256), 0, (hipStream_t)stream, texture,
                       channels, channels - log_channels, dst_row, coef, ldc, flag, (int*)nullptr);
    return rf::check_launch("rf_texture_scan");
}

// rf_texture_scan without the flag reset in the queue (the hipMemsetAsync above is a ~5 us blit kernel in
// every frame): *flag must be 0 on entry, and the kernel zeroes *flag_clear — the caller alternates two
// flags by frame parity, so each frame clears the flag the next frame raises into.
extern "C" int rf_texture_scan2(float* texture, int64_t n_rows, int channels, int patch_elems, int log_channels,
                                const int32_t* dst_row, float* coef, int64_t ldc, int* flag, int* flag_clear,
                                void* stream) {
    RF_REQUIRE(texture && coef && flag && flag_clear && flag != flag_clear, "rf_texture_scan2: null or aliased pointer");
    RF_REQUIRE(patch_elems == TEX_SIDE * TEX_SIDE, "rf_texture_scan2: patch_elems must be %d", TEX_SIDE * TEX_SIDE);
    RF_REQUIRE(channels >= 1 && channels <= 32 && ldc >= channels, "rf_texture_scan2: bad channels/ldc");
    RF_REQUIRE(log_channels >= 0 && log_channels <= channels, "rf_texture_scan2: bad log_channels");
    RF_REQUIRE(((uintptr_t)texture & 15) == 0, "rf_texture_scan2: texture must be 16-B aligned");
    RF_REQUIRE(n_rows > 0 && n_rows < (1ll << 31), "rf_texture_scan2: need 1 .. 2^31 rows");
    RF_LAUNCH(texture_scan_kernel, dim3((unsigned)n_rows), dim3(256), 0, (hipStream_t)stream, texture,
                       channels, channels - log_channels, dst_row, coef, ldc, flag, flag_clear);
    return rf::check_launch("rf_texture_scan2");
}

extern "C" int rf_texture_linear(const float* coef, int64_t ldc, int rows, int channels, const float* wsum,
                                 const float* bias, float* out, int64_t ldo, int n, const int* flag, void* stream) {
    RF_REQUIRE(coef && wsum && out && flag, "rf_texture_linear: null pointer");
    RF_REQUIRE(n % 4 == 0 && ldo % 4 == 0 && ldo >= n && ldc >= channels, "rf_texture_linear: bad n/ldo/ldc");
    RF_REQUIRE(channels >= 1 && channels <= TL_MAXC, "rf_texture_linear: channels must be in [1, %d]", TL_MAXC);
    RF_REQUIRE(((uintptr_t)out & 15) == 0 && ((uintptr_t)wsum & 15) == 0 && (!bias || ((uintptr_t)bias & 15) == 0),
               "rf_texture_linear: out/wsum/bias must be 16-B aligned");
    if (rows <= 0) return RF_OK;
    RF_LAUNCH(texture_linear_kernel, dim3((unsigned)((rows + TL_ROWS - 1) / TL_ROWS)), dim3(256), 0,
                       (hipStream_t)stream,
                       coef, ldc, rows, channels, wsum, bias, out, ldo, n, flag);
    return rf::check_launch("rf_texture_linear");
}

extern "C" int rf_vn_encode_dt(const float* vn, int64_t n_rows, const int32_t* dst_row, int n_freqs, void* out,
                               int64_t ldo, int out_dtype, void* stream) {
    RF_REQUIRE(vn && out, "rf_vn_encode: null pointer");
    RF_REQUIRE(ldo >= 9 * (2 * n_freqs + 1), "rf_vn_encode: ldo too small");
    RF_REQUIRE(out_dtype == RF_DT_BF16 || out_dtype == RF_DT_F16, "rf_vn_encode: bad out_dtype");
    if (n_rows <= 0) return RF_OK;
    RF_LAUNCH(vn_encode_kernel, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, vn,
                       n_rows, dst_row, n_freqs, (bf16_t*)out, ldo, (int)(out_dtype == RF_DT_F16));
    return rf::check_launch("rf_vn_encode");
}

extern "C" int rf_vn_encode(const float* vn, int64_t n_rows, const int32_t* dst_row, int n_freqs, void* out,
                            int64_t ldo, void* stream) {
    return rf_vn_encode_dt(vn, n_rows, dst_row, n_freqs, out, ldo, RF_DT_BF16, stream);
}

extern "C" int rf_ray_tokens_dt(const float* c2w, const float* fov_deg, int n_views, int res, int patch, void* out,
                                float* ray_pos, int out_dtype, void* stream) {
    RF_REQUIRE(c2w && fov_deg && out, "rf_ray_tokens: null pointer");
    RF_REQUIRE(res % patch == 0, "rf_ray_tokens: resolution %d not divisible by patch %d", res, patch);
    RF_REQUIRE(out_dtype == RF_DT_BF16 || out_dtype == RF_DT_F16, "rf_ray_tokens: bad out_dtype");
    if (n_views <= 0) return RF_OK;
    dim3 grid((res * res + 255) / 256, n_views);
    RF_LAUNCH(ray_tokens_kernel, grid, dim3(256), 0, (hipStream_t)stream, c2w, fov_deg, res, patch,
                       (bf16_t*)out, ray_pos, (int)(out_dtype == RF_DT_F16));
    return rf::check_launch("rf_ray_tokens");
}

extern "C" int rf_ray_tokens(const float* c2w, const float* fov_deg, int n_views, int res, int patch, void* out,
                             float* ray_pos, void* stream) {
    return rf_ray_tokens_dt(c2w, fov_deg, n_views, res, patch, out, ray_pos, RF_DT_BF16, stream);
}

extern "C" int rf_patchify_rays_dt(const float* rays_d, int n_views, int res, int patch, void* out, int out_dtype,
                                   void* stream) {
    RF_REQUIRE(rays_d && out, "rf_patchify_rays: null pointer");
    RF_REQUIRE(res % patch == 0, "rf_patchify_rays: resolution %d not divisible by patch %d", res, patch);
    RF_REQUIRE(out_dtype == RF_DT_BF16 || out_dtype == RF_DT_F16, "rf_patchify_rays: bad out_dtype");
    if (n_views <= 0) return RF_OK;
    dim3 grid((res * res + 255) / 256, n_views);
    RF_LAUNCH(patchify_rays_kernel, grid, dim3(256), 0, (hipStream_t)stream, rays_d, res, patch, (bf16_t*)out,
              (int)(out_dtype == RF_DT_F16));
    return rf::check_launch("rf_patchify_rays");
}

extern "C" int rf_patchify_rays(const float* rays_d, int n_views, int res, int patch, void* out, void* stream) {
    return rf_patchify_rays_dt(rays_d, n_views, res, patch, out, RF_DT_BF16, stream);
}

extern "C" int rf_scene_pos(const float* tris, const int32_t* valid_idx, const int32_t* scene_off, const float* c2w,
                            int n_scenes, int n_views, int n_reg, float* pos_out, const int32_t* set_off, int max_tris,
                            float* partials, int64_t partial_floats, void* stream) {
    RF_REQUIRE(tris && valid_idx && scene_off && pos_out && set_off && partials, "rf_scene_pos: null pointer");
    RF_REQUIRE(n_reg >= 0 && max_tris >= 0, "rf_scene_pos: negative sizes");
    const int sets = c2w ? n_scenes * n_views : n_scenes;
    if (sets <= 0) return RF_OK;
    const int nb = max_tris > 0 ? (max_tris + 255) / 256 : 1;
    RF_REQUIRE(partial_floats >= (int64_t)sets * nb * 9, "rf_scene_pos: partials need sets x ceil(max_tris/256) x 9 "
               "floats (rf_scene_pos_partials)");
    RF_LAUNCH(scene_pos_tri_kernel, dim3(nb, sets), dim3(256), 0, (hipStream_t)stream, tris, valid_idx,
                       scene_off, c2w, n_views, n_reg, pos_out, set_off, partials);
    RF_LAUNCH(scene_pos_center_kernel, dim3(sets), dim3(64), 0, (hipStream_t)stream, scene_off, n_views,
                       c2w ? 1 : 0, n_reg, nb, partials, pos_out, set_off, rf::device_error_word());
    return rf::check_launch("rf_scene_pos");
}

extern "C" int64_t rf_scene_pos_partials(int sets, int max_tris) {
    return (int64_t)(sets > 0 ? sets : 0) * (max_tris > 0 ? (max_tris + 255) / 256 : 1) * 9;
}

extern "C" int rf_hdr_output(const float* logits, float* out, int n, int c, int h, int w, float elu_alpha,
                             int log_decode, int channels_last, void* stream) {
    RF_REQUIRE(logits && out, "rf_hdr_output: null pointer");
    const int64_t n_pix = (int64_t)n * h * w;
    if (n_pix <= 0) return RF_OK;
    RF_LAUNCH(hdr_output_kernel, dim3((unsigned)((n_pix + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       logits, out, n_pix, c, h * w, elu_alpha, log_decode, channels_last);
    return rf::check_launch("rf_hdr_output");
}
