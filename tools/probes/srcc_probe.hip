// Probe: chaining v_mfma_f32_16x16x16_f16 (K = 16) onto the accumulator of
// v_mfma_f32_16x16x32_f16 (K = 32) through SrcC -- the form the fp16 conv's tap-8 remainder avoided after it gave
// wrong sums.  D = A1 B1 (K = 32) + A2 B2 (K = 16) per 16 x 16 tile, four forms against a CPU reference:
//   chained      acc = mfma16(a2, b2, mfma32(a1, b1, 0))        (SrcC = the K = 32 result, back to back)
//   chained_nop  the same with s_nop 7 x 2 pinned between the two MFMAs (sched_barrier)
//   separate     mfma32(a1, b1, 0) + mfma16(a2, b2, 0) added by VALU (the conv's current form)
//   chained_rev  acc = mfma32(a1, b1, mfma16(a2, b2, 0))        (the other order)
//   asm_b2b      the chained pair hand-issued in one asm block with no wait states between
//   asm_nop      the same with 2 x s_nop 7 between
// Each form runs over 256 tiles with independent random data; the host reports the max error of each.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/srcc_probe.hip -o tools/probes/srcc_probe
// ISA:   hipcc --offload-arch=gfx950 -O3 -S --offload-device-only tools/probes/srcc_probe.hip -o /tmp/srcc.s
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// A1 [16][32], B1 [32][16], A2 [16][16], B2 [16][16] per tile; lane (o = lane & 15, g = lane >> 4)
template <int FORM>
__global__ void k(const _Float16* A1, const _Float16* B1, const _Float16* A2, const _Float16* B2, float* D) {
  const int tile = blockIdx.x, lane = threadIdx.x, g = lane >> 4, o = lane & 15;
  const _Float16* a1 = A1 + tile * 512;
  const _Float16* b1 = B1 + tile * 512;
  const _Float16* a2 = A2 + tile * 256;
  const _Float16* b2 = B2 + tile * 256;
  h8 fa1, fb1;
  for (int j = 0; j < 8; ++j) {
    fa1[j] = a1[o * 32 + 8 * g + j];   // A row o, k = 8g + j
    fb1[j] = b1[(8 * g + j) * 16 + o]; // B column o
  }
  h4 fa2, fb2;
  for (int j = 0; j < 4; ++j) {
    fa2[j] = a2[o * 16 + 4 * g + j];
    fb2[j] = b2[(4 * g + j) * 16 + o];
  }
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 acc;
  // every operand in registers before the first MFMA: the pair below issues with nothing between (r06's probe let
  // the K = 16 operands' global loads complete between the two MFMAs -- hundreds of cycles -- so it never
  // exercised the back-to-back SrcC dependency)
  asm volatile("" : "+v"(fa1), "+v"(fb1), "+v"(fa2), "+v"(fb2));  // forces every load's wait here
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (FORM == 4) {  // hand-issued back to back, no wait states (hazard recognizer bypassed)
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0\n\tv_mfma_f32_16x16x16_f16 %0, %3, %4, %0\n\ts_nop 7\n\ts_nop 7"
                 : "=&v"(acc) : "v"(fa1), "v"(fb1), "v"(fa2), "v"(fb2));
  } else if constexpr (FORM == 5) {  // hand-issued with 2 x s_nop 7 between
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0\n\ts_nop 7\n\ts_nop 7\n\tv_mfma_f32_16x16x16_f16 %0, %3, %4, %0\n\ts_nop 7\n\ts_nop 7"
                 : "=&v"(acc) : "v"(fa1), "v"(fb1), "v"(fa2), "v"(fb2));
  } else if constexpr (FORM >= 10) {  // hand-issued with s_nop (FORM - 10) between: FORM - 9 wait states
#define SRCC_PAIR(N)                                                                                                 \
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0\n\ts_nop " #N "\n\tv_mfma_f32_16x16x16_f16 %0, %3, %4, %0\n\ts_nop 7\n\ts_nop 7" \
               : "=&v"(acc) : "v"(fa1), "v"(fb1), "v"(fa2), "v"(fb2))
    if constexpr (FORM == 10) SRCC_PAIR(0);
    if constexpr (FORM == 11) SRCC_PAIR(1);
    if constexpr (FORM == 12) SRCC_PAIR(2);
    if constexpr (FORM == 13) SRCC_PAIR(3);
    if constexpr (FORM == 14) SRCC_PAIR(4);
    if constexpr (FORM == 15) SRCC_PAIR(5);
    if constexpr (FORM == 16) SRCC_PAIR(6);
    if constexpr (FORM == 17) SRCC_PAIR(7);
#undef SRCC_PAIR
  } else if constexpr (FORM == 0) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa1, fb1, z, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x16f16(fa2, fb2, acc, 0, 0, 0);
  } else if constexpr (FORM == 1) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa1, fb1, z, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    acc = __builtin_amdgcn_mfma_f32_16x16x16f16(fa2, fb2, acc, 0, 0, 0);
  } else if constexpr (FORM == 2) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa1, fb1, z, 0, 0, 0);
    acc += __builtin_amdgcn_mfma_f32_16x16x16f16(fa2, fb2, z, 0, 0, 0);
  } else {
    acc = __builtin_amdgcn_mfma_f32_16x16x16f16(fa2, fb2, z, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa1, fb1, acc, 0, 0, 0);
  }
  for (int j = 0; j < 4; ++j) D[tile * 256 + (4 * g + j) * 16 + o] = acc[j];  // D[row 4g + j][col o]
}

int main() {
  const int NT = 256;
  _Float16 *hA1 = new _Float16[NT * 512], *hB1 = new _Float16[NT * 512], *hA2 = new _Float16[NT * 256],
           *hB2 = new _Float16[NT * 256];
  srand(7);
  auto rnd = []() { return (_Float16)((rand() % 2001) / 1000.f - 1.f); };
  for (int i = 0; i < NT * 512; ++i) { hA1[i] = rnd(); hB1[i] = rnd(); }
  for (int i = 0; i < NT * 256; ++i) { hA2[i] = rnd(); hB2[i] = rnd(); }
  double* ref = new double[NT * 256];
  for (int t = 0; t < NT; ++t)
    for (int r = 0; r < 16; ++r)
      for (int c = 0; c < 16; ++c) {
        double s = 0;
        for (int kk = 0; kk < 32; ++kk) s += (double)(float)hA1[t * 512 + r * 32 + kk] * (double)(float)hB1[t * 512 + kk * 16 + c];
        for (int kk = 0; kk < 16; ++kk) s += (double)(float)hA2[t * 256 + r * 16 + kk] * (double)(float)hB2[t * 256 + kk * 16 + c];
        ref[t * 256 + r * 16 + c] = s;
      }
  _Float16 *dA1, *dB1, *dA2, *dB2;
  float* dD;
  (void)hipMalloc(&dA1, NT * 1024); hipMalloc(&dB1, NT * 1024); hipMalloc(&dA2, NT * 512); hipMalloc(&dB2, NT * 512);
  hipMalloc(&dD, NT * 1024);
  hipMemcpy(dA1, hA1, NT * 1024, hipMemcpyHostToDevice); hipMemcpy(dB1, hB1, NT * 1024, hipMemcpyHostToDevice);
  hipMemcpy(dA2, hA2, NT * 512, hipMemcpyHostToDevice); hipMemcpy(dB2, hB2, NT * 512, hipMemcpyHostToDevice);
  float* D = new float[NT * 256];
  const char* names[14] = {"chained (compiler wait states)", "chained + s_nop 7 x2", "separate + VALU add",
                           "chained, K=16 first", "asm back to back, 0 nops", "asm + s_nop 7 x2",
                           "asm + s_nop 0 (1 wait state)", "asm + s_nop 1 (2)", "asm + s_nop 2 (3)", "asm + s_nop 3 (4)",
                           "asm + s_nop 4 (5)", "asm + s_nop 5 (6)", "asm + s_nop 6 (7)", "asm + s_nop 7 (8)"};
  for (int f = 0; f < 14; ++f) {
    hipMemset(dD, 0, NT * 1024);
    if (f == 0) hipLaunchKernelGGL(k<0>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 1) hipLaunchKernelGGL(k<1>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 2) hipLaunchKernelGGL(k<2>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 3) hipLaunchKernelGGL(k<3>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 4) hipLaunchKernelGGL(k<4>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 5) hipLaunchKernelGGL(k<5>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 6) hipLaunchKernelGGL(k<10>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 7) hipLaunchKernelGGL(k<11>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 8) hipLaunchKernelGGL(k<12>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 9) hipLaunchKernelGGL(k<13>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 10) hipLaunchKernelGGL(k<14>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 11) hipLaunchKernelGGL(k<15>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 12) hipLaunchKernelGGL(k<16>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    if (f == 13) hipLaunchKernelGGL(k<17>, dim3(NT), dim3(64), 0, 0, dA1, dB1, dA2, dB2, dD);
    hipMemcpy(D, dD, NT * 1024, hipMemcpyDeviceToHost);
    double e = 0;
    int bad = 0;
    for (int i = 0; i < NT * 256; ++i) {
      const double d = fabs(D[i] - ref[i]);
      e = fmax(e, d);
      bad += d > 1e-3;
    }
    printf("%-32s max |err| %.3g  elements off by > 1e-3: %d / %d\n", names[f], e, bad, NT * 256);
  }
  return 0;
}
