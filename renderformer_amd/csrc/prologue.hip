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
                                                           bf16_t* __restrict__ out, int64_t ldo) {
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

// ----------------------------------------------------------------------------- vertex normals
// NeRFEncoding(in_dim=9, L, include_input) (nerf_encoding.py:76-84): [x, sin(x_d 2^l), sin(x_d 2^l + pi/2)]
__global__ __launch_bounds__(256) void vn_encode_kernel(const float* __restrict__ vn, int64_t n_rows,
                                                        const int32_t* __restrict__ dst_row, int L,
                                                        bf16_t* __restrict__ out, int64_t ldo) {
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
        out[(int64_t)d * ldo + e] = f32_to_bf16(val);
    }
}

// ----------------------------------------------------------------------------- rays
// RayGenerator (ray_generator.py:31-50) + rearrange 'b (h p1) (w p2) c -> b (h w) (c p1 p2)'
__global__ __launch_bounds__(256) void ray_tokens_kernel(const float* __restrict__ c2w, const float* __restrict__ fov,
                                                         int res, int patch, bf16_t* __restrict__ out,
                                                         float* __restrict__ ray_pos) {
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
    o[feat] = f32_to_bf16(r0);
    o[pp + feat] = f32_to_bf16(r1);
    o[2 * pp + feat] = f32_to_bf16(r2);
}

__global__ __launch_bounds__(256) void patchify_rays_kernel(const float* __restrict__ rays, int res, int patch,
                                                            bf16_t* __restrict__ out) {
    const int view = blockIdx.y;
    const int pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= res * res) return;
    const int y = pix / res, x = pix % res;
    const float* r = rays + ((int64_t)view * res * res + pix) * 3;
    const int pw = res / patch, pp = patch * patch;
    const int tok = (y / patch) * pw + (x / patch);
    const int feat = (y % patch) * patch + (x % patch);
    bf16_t* o = out + ((int64_t)view * pw * pw + tok) * (3 * pp);
    o[feat] = f32_to_bf16(r[0]);
    o[pp + feat] = f32_to_bf16(r[1]);
    o[2 * pp + feat] = f32_to_bf16(r[2]);
}

// ----------------------------------------------------------------------------- RoPE positions
// trans_to_cam_coord (transform.py:24-27: p -> R^T p - R^T t) and process_tri_vpos_list
// (renderformer.py:111-122: register rows = masked mean position, averaged over the 3 vertices).
__global__ __launch_bounds__(256) void scene_pos_kernel(const float* __restrict__ tris,
                                                        const int32_t* __restrict__ valid_idx,
                                                        const int32_t* __restrict__ scene_off,
                                                        const float* __restrict__ c2w, int n_views, int n_reg,
                                                        float* __restrict__ pos_out,
                                                        const int32_t* __restrict__ set_off) {
    __shared__ float red[256 / 64][9];
    const int set = blockIdx.x;
    const int scene = c2w ? set / n_views : set;
    const int t0 = scene_off[scene], n = scene_off[scene + 1] - t0;
    float rt[9], tinv[3];
    if (c2w) {
        const float* m = c2w + set * 16;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) rt[i * 3 + j] = m[j * 4 + i];
        for (int i = 0; i < 3; ++i) tinv[i] = -(rt[i * 3 + 0] * m[3] + rt[i * 3 + 1] * m[7] + rt[i * 3 + 2] * m[11]);
    }
    float acc[9];
    for (int c = 0; c < 9; ++c) acc[c] = 0.f;
    float* dst = pos_out + (int64_t)(set_off[set] + n_reg) * 9;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float* src = tris + (int64_t)valid_idx[t0 + i] * 9;
        float v[9];
        for (int c = 0; c < 9; ++c) v[c] = src[c];
        if (c2w) {
            float w[9];
            for (int vert = 0; vert < 3; ++vert)
                for (int a = 0; a < 3; ++a)
                    w[vert * 3 + a] = rt[a * 3 + 0] * v[vert * 3 + 0] + rt[a * 3 + 1] * v[vert * 3 + 1] +
                                      rt[a * 3 + 2] * v[vert * 3 + 2] + tinv[a];
            for (int c = 0; c < 9; ++c) v[c] = w[c];
        }
        for (int c = 0; c < 9; ++c) {
            dst[(int64_t)i * 9 + c] = v[c];
            acc[c] += v[c];
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int c = 0; c < 9; ++c) {
        const float s = wave_sum(acc[c]);
        if (lane == 0) red[wave][c] = s;
    }
    __syncthreads();
    if (threadIdx.x < n_reg * 9) {
        const float wgt = 1.0f / ((float)n + 1e-5f);
        float tot[9];
        for (int c = 0; c < 9; ++c) tot[c] = (red[0][c] + red[1][c] + red[2][c] + red[3][c]) * wgt;
        const int k = threadIdx.x % 3;
        const float ctr = (tot[k] + tot[3 + k] + tot[6 + k]) / 3.0f;
        pos_out[(int64_t)set_off[set] * 9 + threadIdx.x] = ctr;
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
    hipLaunchKernelGGL(texture_pack_kernel, dim3((unsigned)n_rows), dim3(256), 0, (hipStream_t)stream, texture,
                       channels, patch_elems, channels - log_channels, dst_row, (bf16_t*)out, ldo);
    return rf::check_launch("rf_texture_pack");
}

extern "C" int rf_vn_encode(const float* vn, int64_t n_rows, const int32_t* dst_row, int n_freqs, void* out,
                            int64_t ldo, void* stream) {
    RF_REQUIRE(vn && out, "rf_vn_encode: null pointer");
    RF_REQUIRE(ldo >= 9 * (2 * n_freqs + 1), "rf_vn_encode: ldo too small");
    if (n_rows <= 0) return RF_OK;
    hipLaunchKernelGGL(vn_encode_kernel, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, vn,
                       n_rows, dst_row, n_freqs, (bf16_t*)out, ldo);
    return rf::check_launch("rf_vn_encode");
}

extern "C" int rf_ray_tokens(const float* c2w, const float* fov_deg, int n_views, int res, int patch, void* out,
                             float* ray_pos, void* stream) {
    RF_REQUIRE(c2w && fov_deg && out, "rf_ray_tokens: null pointer");
    RF_REQUIRE(res % patch == 0, "rf_ray_tokens: resolution %d not divisible by patch %d", res, patch);
    if (n_views <= 0) return RF_OK;
    dim3 grid((res * res + 255) / 256, n_views);
    hipLaunchKernelGGL(ray_tokens_kernel, grid, dim3(256), 0, (hipStream_t)stream, c2w, fov_deg, res, patch,
                       (bf16_t*)out, ray_pos);
    return rf::check_launch("rf_ray_tokens");
}

extern "C" int rf_patchify_rays(const float* rays_d, int n_views, int res, int patch, void* out, void* stream) {
    RF_REQUIRE(rays_d && out, "rf_patchify_rays: null pointer");
    RF_REQUIRE(res % patch == 0, "rf_patchify_rays: resolution %d not divisible by patch %d", res, patch);
    if (n_views <= 0) return RF_OK;
    dim3 grid((res * res + 255) / 256, n_views);
    hipLaunchKernelGGL(patchify_rays_kernel, grid, dim3(256), 0, (hipStream_t)stream, rays_d, res, patch, (bf16_t*)out);
    return rf::check_launch("rf_patchify_rays");
}

extern "C" int rf_scene_pos(const float* tris, const int32_t* valid_idx, const int32_t* scene_off, const float* c2w,
                            int n_scenes, int n_views, int n_reg, float* pos_out, const int32_t* set_off, void* stream) {
    RF_REQUIRE(tris && valid_idx && scene_off && pos_out && set_off, "rf_scene_pos: null pointer");
    RF_REQUIRE(n_reg * 9 <= 256, "rf_scene_pos: too many register tokens");
    const int sets = c2w ? n_scenes * n_views : n_scenes;
    if (sets <= 0) return RF_OK;
    hipLaunchKernelGGL(scene_pos_kernel, dim3(sets), dim3(256), 0, (hipStream_t)stream, tris, valid_idx, scene_off,
                       c2w, n_views, n_reg, pos_out, set_off);
    return rf::check_launch("rf_scene_pos");
}

extern "C" int rf_hdr_output(const float* logits, float* out, int n, int c, int h, int w, float elu_alpha,
                             int log_decode, int channels_last, void* stream) {
    RF_REQUIRE(logits && out, "rf_hdr_output: null pointer");
    const int64_t n_pix = (int64_t)n * h * w;
    if (n_pix <= 0) return RF_OK;
    hipLaunchKernelGGL(hdr_output_kernel, dim3((unsigned)((n_pix + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       logits, out, n_pix, c, h * w, elu_alpha, log_decode, channels_last);
    return rf::check_launch("rf_hdr_output");
}
