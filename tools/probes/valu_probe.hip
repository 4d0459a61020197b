// Probe: issue throughput of v_fmac_f32 vs v_fmac_f32_dpp (row_newbcast) vs v_permlane swaps,
// at 1, 2, 4, 8 waves per SIMD.  Prints ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../dfd-starter_amd/csrc/fdr_dpp_gen.h"

template <int MODE>
__global__ void k(float* out, int iters) {
  float w[64];
  for (int i = 0; i < 64; ++i) w[i] = out[i] * 1e-3f + i;
  float X0 = threadIdx.x, X1 = X0 + 1, X2 = X0 + 2, X3 = X0 + 3;
  float a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {  // 64 plain FMAs, 4 accumulators
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a0) : "v"(X0), "v"(w[c]));
        asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a1) : "v"(X1), "v"(w[16 + c]));
        asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a2) : "v"(X2), "v"(w[32 + c]));
        asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a3) : "v"(X3), "v"(w[48 + c]));
      }
    } else if constexpr (MODE == 1) {  // the 64-FMA DPP block of the rollout
      fdr::dpp_fma_64x4(a0, a1, a2, a3, X0, X1, X2, X3, w);
    } else {  // 64 permlane swaps
#pragma unroll
      for (int c = 0; c < 32; ++c)
        asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(X0), "+v"(X1));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + X0 + X1;
}

int main() {
  float* d;
  hipMalloc(&d, 1 << 26);
  hipMemset(d, 0, 1 << 26);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 2000;
  const char* names[3] = {"v_fmac_f32", "v_fmac_f32_dpp", "permlane swap"};
  for (int mode = 0; mode < 3; ++mode)
    for (int wps : {1, 2, 4, 8}) {
      const int blocks = 256 * wps;  // 256 CUs x wps blocks of 256 threads = wps waves per SIMD
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, d, iters);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, d, iters);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, d, iters);
      };
      launch();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      double instr_per_simd = (double)iters * 64 * wps;  // per SIMD (4 waves/block -> 1 per SIMD)
      printf("%-16s waves/SIMD=%d  %.3f ms  %.3f ns/instr/SIMD  (%.2f cycles @2.4GHz)\n", names[mode], wps, ms,
             ms * 1e6 / instr_per_simd, ms * 1e6 / instr_per_simd * 2.4);
    }
  return 0;
}
