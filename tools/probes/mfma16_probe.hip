// Probe: the fp16 conv's K-remainder path (fdr_impala_h.hip rem_fragment + v_mfma_f32_16x16x16_f16) against
// a CPU reference: D = A (16 x 16) * B (16 x 16) where A's K = 16 values of row o sit in the K = 32 fragment
// layout of the pack (lane (o, g) halves jj: k = 8g + jj, g < 2; zeros for g >= 2), B in the K = 16 layout.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const _Float16* A, const _Float16* B, float* D, float* D32) {
  const int lane = threadIdx.x, g = lane >> 4, o = lane & 15;
  h8 a8;
  for (int jj = 0; jj < 8; ++jj) { const int kk = 8 * g + jj; a8[jj] = kk < 16 ? A[o * 16 + kk] : (_Float16)0.f; }
  // reference path: K = 32 MFMA with B padded by zeros (b8: k = 8g + jj)
  h8 b8;
  for (int jj = 0; jj < 8; ++jj) { const int kk = 8 * g + jj; b8[jj] = kk < 16 ? B[kk * 16 + o] : (_Float16)0.f; }
  f32x4 r32 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, f32x4{0, 0, 0, 0}, 0, 0, 0);
  const int src = ((lane & 15) + 16 * (g >> 1)) * 4;
  const u32x4 d = __builtin_bit_cast(u32x4, a8);
  const unsigned x0 = __builtin_amdgcn_ds_bpermute(src, d[0]), x1 = __builtin_amdgcn_ds_bpermute(src, d[1]);
  const unsigned x2 = __builtin_amdgcn_ds_bpermute(src, d[2]), x3 = __builtin_amdgcn_ds_bpermute(src, d[3]);
  const h8 w = __builtin_bit_cast(h8, u32x4{(g & 1) ? x2 : x0, (g & 1) ? x3 : x1, 0u, 0u});
  h4 b4;
  for (int j = 0; j < 4; ++j) b4[j] = B[(4 * g + j) * 16 + o];
  f32x4 r = __builtin_amdgcn_mfma_f32_16x16x16f16(h4{w[0], w[1], w[2], w[3]}, b4, f32x4{0, 0, 0, 0}, 0, 0, 0);
  for (int j = 0; j < 4; ++j) { D[(4 * g + j) * 16 + o] = r[j]; D32[(4 * g + j) * 16 + o] = r32[j]; }
}

int main() {
  _Float16 hA[256], hB[256];
  for (int i = 0; i < 256; ++i) { hA[i] = (_Float16)((i * 37 % 17) / 8.f - 1.f); hB[i] = (_Float16)((i * 11 % 13) / 6.f - 1.f); }
  _Float16 *dA, *dB; float *dD, *dD32;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 1024); hipMalloc(&dD32, 1024);
  hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD, dD32);
  float D[256], D32[256];
  hipMemcpy(D, dD, 1024, hipMemcpyDeviceToHost); hipMemcpy(D32, dD32, 1024, hipMemcpyDeviceToHost);
  double e16 = 0, e32 = 0;
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
    double ref = 0; for (int kk = 0; kk < 16; ++kk) ref += (double)(float)hA[i * 16 + kk] * (double)(float)hB[kk * 16 + j];
    e16 = fmax(e16, fabs(D[i * 16 + j] - ref)); e32 = fmax(e32, fabs(D32[i * 16 + j] - ref));
  }
  printf("max err x16 path %.3g, x32 path %.3g\n", e16, e32);
  return 0;
}
