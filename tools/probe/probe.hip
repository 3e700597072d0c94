#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

// A[16][32] row-major bf16, B[32][16] (stored as Bt[16][32], i.e. n-major k-contig), C[16][16] f32
__global__ void mfma16(const __hip_bfloat16* A, const __hip_bfloat16* Bt, float* C) {
  int l = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = *(const __bf16*)&A[(l & 15) * 32 + 8 * (l >> 4) + j];
    b[j] = *(const __bf16*)&Bt[(l & 15) * 32 + 8 * (l >> 4) + j];
  }
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}
__global__ void mfma32(const __hip_bfloat16* A, const __hip_bfloat16* Bt, float* C) {
  int l = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = *(const __bf16*)&A[(l & 31) * 16 + 8 * (l >> 5) + j];
    b[j] = *(const __bf16*)&Bt[(l & 31) * 16 + 8 * (l >> 5) + j];
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) C[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}
// f32 16x16x4: A[16][4], Bt[16][4]
__global__ void mfmaf32(const float* A, const float* Bt, float* C) {
  int l = threadIdx.x;
  float a = A[(l & 15) * 4 + (l >> 4)];
  float b = Bt[(l & 15) * 4 + (l >> 4)];
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}
extern "C" int probe_run(int which, const void* A, const void* Bt, float* C, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (which == 0) hipLaunchKernelGGL(mfma16, dim3(1), dim3(64), 0, s, (const __hip_bfloat16*)A, (const __hip_bfloat16*)Bt, C);
  else if (which == 1) hipLaunchKernelGGL(mfma32, dim3(1), dim3(64), 0, s, (const __hip_bfloat16*)A, (const __hip_bfloat16*)Bt, C);
  else hipLaunchKernelGGL(mfmaf32, dim3(1), dim3(64), 0, s, (const float*)A, (const float*)Bt, C);
  return (int)hipGetLastError();
}
