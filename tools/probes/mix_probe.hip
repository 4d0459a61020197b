// Probe: issue cost per wave-instruction per SIMD of every instruction kind in rollout_pair_kernel's loop
// (DESIGN.md 3.0 ceiling table), at 1 / 2 / 4 waves per SIMD.  Each mode issues 64 independent instructions
// per iteration (8 rotating accumulators, operands in distinct registers), timed by HIP events over the
// whole grid (256 CUs x 4 SIMDs x W waves).  ns per instruction per SIMD; cycles at the clock given on the
// command line (the rollout's loaded clock from its PMC, GRBM_GUI_ACTIVE / 8 / duration).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/mix_probe.hip -o tools/probes/mix_probe && ./mix_probe 2.13
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  __shared__ float4 lds[64];
  f2 a[8], w[8];
  float b[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = f2{out[i] * 1e-3f, out[i + 8]};
    w[i] = f2{threadIdx.x * 1e-3f + i, 1.f + i};
    b[i] = out[i + 16] + 0.5f;
  }
  if (threadIdx.x < 64) lds[threadIdx.x] = float4{1.f, 2.f, 3.f, 4.f};
  __syncthreads();
  f2 x = f2{threadIdx.x * 1e-4f, 0.5f};
  float4 acc4 = float4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
#define PK(i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(w[i]), "v"(x));
#define FMA(i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i].x) : "v"(w[i].y), "v"(b[i]));
#define ADD(i) asm volatile("v_add_f32 %0, %1, %0" : "+v"(a[i].x) : "v"(w[i].y));
#define MOV(i) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i].x) : "v"(w[i].y));
#define FMACDPP(i) asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a[i].x) : "v"(w[i].y), "v"(b[i]));
#define ADDDPP(i) asm volatile("v_add_f32_dpp %0, %1, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[i].x) : "v"(w[i].y));
#define EXP(i) asm volatile("v_exp_f32 %0, %1" : "=v"(a[i].x) : "v"(w[i].y));
#define RCP(i) asm volatile("v_rcp_f32 %0, %1" : "=v"(a[i].x) : "v"(w[i].y));
#define PKADD(i) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(a[i]) : "v"(w[i]));
#define NOP0(i) asm volatile("s_nop 0");
#define NOP1(i) asm volatile("s_nop 1");
#define DSRD(i) { float4 t; asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(8)" : "=v"(t) : "v"((unsigned)(i * 16))); acc4.x += t.x; }
      if constexpr (MODE == 0) { REP8(PK) }
      if constexpr (MODE == 1) { REP8(FMA) }
      if constexpr (MODE == 2) { REP8(ADD) }
      if constexpr (MODE == 3) { REP8(MOV) }
      if constexpr (MODE == 4) { REP8(FMACDPP) }
      if constexpr (MODE == 5) { REP8(ADDDPP) }
      if constexpr (MODE == 6) { REP8(EXP) }
      if constexpr (MODE == 7) { REP8(RCP) }
      if constexpr (MODE == 8) { REP8(PKADD) }
      if constexpr (MODE == 9) { REP8(NOP0) }
      if constexpr (MODE == 10) { REP8(NOP1) }
      if constexpr (MODE == 11) { REP8(DSRD) }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  float s = acc4.x;
  for (int i = 0; i < 8; ++i) s += a[i].x + a[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*Kern)(float*, int);
int main(int argc, char** argv) {
  const double ghz = argc > 1 ? atof(argv[1]) : 2.13;
  float* d;
  hipMalloc(&d, 1 << 26);
  hipMemset(d, 0, 1 << 26);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 2000;
  Kern ks[12] = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>, k<9>, k<10>, k<11>};
  const char* names[12] = {"v_pk_fma_f32", "v_fma_f32", "v_add_f32", "v_mov_b32", "v_fmac_f32_dpp", "v_add_f32_dpp",
                           "v_exp_f32", "v_rcp_f32", "v_pk_add_f32", "s_nop 0", "s_nop 1", "ds_read_b128 (bcast)"};
  printf("%-22s %28s %28s %28s\n", "instruction", "1 wave/SIMD ns (cyc)", "2 waves/SIMD ns (cyc)", "4 waves/SIMD ns (cyc)");
  for (int mode = 0; mode < 12; ++mode) {
    printf("%-22s", names[mode]);
    for (int wps : {1, 2, 4}) {
      const int blocks = 256 * wps;  // 256-thread blocks: 4 waves -> one per SIMD
      hipLaunchKernelGGL(ks[mode], dim3(blocks), dim3(256), 0, 0, d, iters);
      hipEventRecord(e0);
      hipLaunchKernelGGL(ks[mode], dim3(blocks), dim3(256), 0, 0, d, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double ns = ms * 1e6 / ((double)iters * 64 * wps);
      printf("   %12.3f (%6.2f cyc)   ", ns, ns * ghz);
    }
    printf("\n");
  }
  return 0;
}
