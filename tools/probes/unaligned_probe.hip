// Probe: 16-B global loads (h8) at 2-byte-aligned addresses -- values and read rate against aligned loads.
// One pass: every wave sweeps its own 2 MiB slice of a 64 MiB f16 buffer (the core kernel's stream shape),
// starting at element offset `shift` (0 = aligned, 1..7 = misaligned).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/unaligned_probe.hip -o tools/probes/unaligned_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr int kSlice = 1 << 20;  // halves per workgroup slice (2 MiB)

__global__ __launch_bounds__(256) void sweep(const _Float16* __restrict__ src, float* out, int shift, int n_slices) {
  const _Float16* s = src + (size_t)(blockIdx.x % n_slices) * (kSlice / 2) + shift;  // slices overlap by half
  float acc = 0.f;
  for (int i = threadIdx.x; i < kSlice / 8 - 1; i += 256) {
    const h8 v = *reinterpret_cast<const h8*>(s + (size_t)i * 8);
    acc += (float)v[0] + (float)v[7];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ void check(const _Float16* src, _Float16* dst, int shift) {
  const h8 v = *reinterpret_cast<const h8*>(src + shift + 8 * threadIdx.x);
  for (int j = 0; j < 8; ++j) dst[8 * threadIdx.x + j] = v[j];
}

int main() {
  const size_t n = 64ull << 20;  // halves
  std::vector<_Float16> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (_Float16)(float)(i % 1021);
  _Float16 *d, *o;
  float* out;
  hipMalloc(&d, n * 2 + 64);
  hipMalloc(&o, 64 * 8 * 2);
  hipMalloc(&out, 1024 * 256 * 4);
  hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice);
  for (int shift = 0; shift < 8; ++shift) {
    hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, d, o, shift);
    std::vector<_Float16> r(512);
    hipMemcpy(r.data(), o, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 512; ++i) bad += (float)r[i] != (float)h[shift + i];
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int nsl = 48;  // 48 slices of 2 MiB overlapping by half: a 49 MiB working set
    hipLaunchKernelGGL(sweep, dim3(512), dim3(256), 0, 0, d, out, shift, nsl);
    hipEventRecord(e0);
    for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(sweep, dim3(512), dim3(256), 0, 0, d, out, shift, nsl);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double bytes = 512.0 * (kSlice / 8 - 1) * 16;
    printf("shift %d: %d / 512 wrong values; %.1f us per sweep, %.2f TB/s\n", shift, bad, ms * 100.f,
           bytes / (ms / 10 * 1e-3) / 1e12);
  }
  return 0;
}
