// Probe: issue cost of the f16 MFMA shapes on gfx950, one wave alone on its SIMD, back-to-back independent
// accumulators (4 chains).  Prints shader clocks (s_memtime) per MFMA for each shape.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_rate_probe.hip -o tools/probes/mfma_rate_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kIters = 512;

template <int SHAPE>
__global__ void k(float* out, long long* clk, float seed) {
  const int lane = threadIdx.x;
  h8 a8, b8;
  for (int j = 0; j < 8; ++j) { a8[j] = (_Float16)(seed * (lane + j)); b8[j] = (_Float16)(seed * (lane - j)); }
  const h4 a4 = h4{a8[0], a8[1], a8[2], a8[3]}, b4 = h4{b8[0], b8[1], b8[2], b8[3]};
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  f32x16 d0 = {}, d1 = {}, d2 = {}, d3 = {};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
    if constexpr (SHAPE == 0) {  // v_mfma_f32_16x16x32_f16
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c3, 0, 0, 0);
    } else if constexpr (SHAPE == 1) {  // v_mfma_f32_16x16x16_f16
      c0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c3, 0, 0, 0);
    } else if constexpr (SHAPE == 2) {  // v_mfma_f32_32x32x16_f16
      d0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, d3, 0, 0, 0);
    } else {  // v_mfma_f32_32x32x8_f16
      d0 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, d3, 0, 0, 0);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int j = 0; j < 4; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
  for (int j = 0; j < 16; ++j) s += d0[j] + d1[j] + d2[j] + d3[j];
  out[lane] = s;
  if (lane == 0) clk[0] = t1 - t0;
}

int main() {
  float* out;
  long long* clk;
  hipMalloc(&out, 64 * sizeof(float));
  hipMalloc(&clk, sizeof(long long));
  const char* names[4] = {"v_mfma_f32_16x16x32_f16", "v_mfma_f32_16x16x16_f16", "v_mfma_f32_32x32x16_f16",
                          "v_mfma_f32_32x32x8_f16"};
  const double flop[4] = {16 * 16 * 32 * 2, 16 * 16 * 16 * 2, 32 * 32 * 16 * 2, 32 * 32 * 8 * 2};
  for (int rep = 0; rep < 2; ++rep)
    for (int s = 0; s < 4; ++s) {
      if (s == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, out, clk, 1e-3f);
      if (s == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, out, clk, 1e-3f);
      if (s == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, out, clk, 1e-3f);
      if (s == 3) hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, out, clk, 1e-3f);
      long long c = 0;
      hipMemcpy(&c, clk, sizeof(c), hipMemcpyDeviceToHost);
      const double per = (double)c / (4.0 * kIters);
      if (rep == 1) printf("%-26s %6.2f clocks per MFMA  %7.1f FLOP/clock/SIMD\n", names[s], per, flop[s] / per);
    }
  return 0;
}
