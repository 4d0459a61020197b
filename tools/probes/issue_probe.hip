// Probe: SIMD issue cost (cycles per wave-instruction per SIMD) of the instruction kinds the MLP
// rollout step is built from, at 4 waves/SIMD (the rollout's occupancy).  Each mode issues 64
// independent instructions per iteration (8 rotating destinations).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/issue_probe.hip -o tools/probes/issue_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a[8], w[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = f2{out[i] * 1e-3f, out[i + 8]};
    w[i] = f2{threadIdx.x * 1e-3f + i, 1.f};
  }
  f2 x = f2{threadIdx.x * 1e-4f, 0.5f};
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
#define PK(i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(w[i]), "v"(x));
#define FMA(i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i].x) : "v"(w[i].x), "v"(x.x));
#define EXP(i) asm volatile("v_exp_f32 %0, %1" : "=v"(a[i].x) : "v"(w[i].x));
#define RL(i) { int sv; asm volatile("v_readlane_b32 %0, %1, %2" : "=s"(sv) : "v"(w[i].x), "i"(i)); acc += __builtin_bit_cast(float, sv); }
#define DPPADD(i) asm volatile("v_add_f32_dpp %0, %1, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "+v"(a[i].x) : "v"(w[i].x));
#define PKSG(i) { asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(w[i]), "s"(x)); }
      if constexpr (MODE == 0) { REP8(PK) }
      if constexpr (MODE == 1) { REP8(FMA) }
      if constexpr (MODE == 2) { REP8(EXP) }
      if constexpr (MODE == 3) { REP8(RL) }
      if constexpr (MODE == 4) { REP8(DPPADD) }
      if constexpr (MODE == 5) { REP8(PKSG) }
    }
  }
  float s = acc;
  for (int i = 0; i < 8; ++i) s += a[i].x + a[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* d;
  hipMalloc(&d, 1 << 26);
  hipMemset(d, 0, 1 << 26);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  const char* names[6] = {"v_pk_fma_f32", "v_fma_f32", "v_exp_f32", "v_readlane_b32", "v_add_f32_dpp",
                          "v_pk_fma_f32 (sgpr)"};
  for (int mode = 0; mode < 6; ++mode)
    for (int wps : {1, 4}) {
      const int blocks = 256 * wps;
      auto launch = [&]() {
        switch (mode) {
          case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          default: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
        }
      };
      launch();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double instr_per_simd = (double)iters * 64 * wps;
      printf("%-22s waves/SIMD=%d  %.3f ns/instr/SIMD  (%.2f cycles @2.4GHz)\n", names[mode], wps,
             ms * 1e6 / instr_per_simd, ms * 1e6 / instr_per_simd * 2.4);
    }
  return 0;
}
