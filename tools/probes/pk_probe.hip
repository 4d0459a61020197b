// Probe: issue cost of v_pk_fma_f32 operand patterns vs v_fma_f32 at 1 / 2 / 4 waves per SIMD, with
// the s_memtime tick rate calibrated against wall time (ticks per ns).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/pk_probe.hip -o tools/probes/pk_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define REP16(X) REP8(X) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

__device__ unsigned long long g_ticks;

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a[16], w[16], xs[16];
  for (int i = 0; i < 16; ++i) {
    a[i] = f2{out[i] * 1e-3f, out[i + 16]};
    w[i] = f2{threadIdx.x * 1e-3f + i, 1.f};
    xs[i] = f2{threadIdx.x * 1e-4f + i, 0.5f};
  }
  f2 x = f2{threadIdx.x * 1e-4f, 0.5f};
  unsigned long long t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
  for (int it = 0; it < iters; ++it) {
#define PK(i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(w[i]), "v"(x));
#define PKX(i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(w[i]), "v"(xs[i]));
#define PKB(i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(a[i]) : "v"(w[i]), "v"(x));
#define FMA2(i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i].x) : "v"(w[i].x), "v"(x.x)); \
                asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i].y) : "v"(w[i].y), "v"(x.x));
#define FMAC2(i) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[i].x) : "v"(w[i].x), "v"(x.x)); \
                 asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[i].y) : "v"(w[i].y), "v"(x.x));
    if constexpr (MODE == 0) { REP16(PK) }
    if constexpr (MODE == 1) { REP16(PKX) }
    if constexpr (MODE == 2) { REP16(PKB) }
    if constexpr (MODE == 3) { REP16(FMA2) }
    if constexpr (MODE == 4) { REP16(FMAC2) }
  }
  unsigned long long t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
  if (blockIdx.x == 0 && threadIdx.x == 0) g_ticks = t1 - t0;
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += a[i].x + a[i].y;
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
  const char* names[5] = {"pk_fma (shared x)", "pk_fma (x per acc)", "pk_fma op_sel_hi bcast", "2x v_fma_f32",
                          "2x v_fmac_f32"};
  const int per_iter[5] = {16, 16, 16, 32, 32};
  for (int mode = 0; mode < 5; ++mode)
    for (int wps : {1, 2, 4}) {
      const int blocks = 256 * wps;
      auto launch = [&]() {
        switch (mode) {
          case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          default: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
        }
      };
      launch();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long ticks;
      hipMemcpyFromSymbol(&ticks, HIP_SYMBOL(g_ticks), sizeof(ticks));
      const double instr_per_simd = (double)iters * per_iter[mode] * wps;
      const double ticks_per_instr = (double)ticks / (iters * per_iter[mode]);  // one wave's view
      printf("%-24s waves/SIMD=%d  %.3f ns/instr/SIMD  wave0: %.2f ticks/own-instr, ticks/ns %.3f\n", names[mode],
             wps, ms * 1e6 / instr_per_simd, ticks_per_instr, ticks / (ms * 1e6));
    }
  return 0;
}
