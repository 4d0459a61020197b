// Shared device helpers for the FD engine kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fdr.h"

namespace fdr {

constexpr int kWave = 64;
constexpr int kHidden = 64;  // policies/discrete.py:35-36, policies/mujoco.py:33-34

// ---------------------------------------------------------------------------------------------
// Counter random stream (oracle/rng.py restates it for the checker; DESIGN.md "Random streams")
// ---------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t hash_ctr(uint64_t key, uint64_t lane, uint64_t t, uint64_t k) {
  const uint64_t c = (lane << 32) | (t << 4) | k;
  return mix64(key + c * 0x9E3779B97F4A7C15ull);
}
constexpr uint64_t kJiggleT = (1ull << 28) - 1;

__device__ __forceinline__ float uniform24(uint64_t h) {
  return (float)(uint32_t)(h >> 40) * 0x1p-24f;
}
// Box-Muller on the hardware transcendental units: v_log_f32 is log2, v_cos_f32 takes revolutions,
// so cos(2*pi*u2) needs no range reduction.  Agrees with oracle/rng.py to a few ulp.
__device__ __forceinline__ float normal_bm(uint64_t h) {
  const float u1 = (float)((uint32_t)(h >> 40) + 1u) * 0x1p-24f;
  const float u2 = (float)((uint32_t)(h >> 16) & 0xFFFFFFu) * 0x1p-24f;
  const float r = __builtin_sqrtf(-1.38629436111989061f * __builtin_amdgcn_logf(u1));  // -2 ln u1
  return r * __builtin_amdgcn_cosf(u2);
}

// tanh(x) = 1 - 2 / (1 + e^{2x}) on v_exp_f32 / v_rcp_f32 (abs error ~3e-7; saturates to +-1)
constexpr float kTanhScale = 2.88539008177792681f;  // 2 * log2(e)
__device__ __forceinline__ float tanh_pre(float t) {  // tanh(x) for t = kTanhScale * x
  const float e = __builtin_amdgcn_exp2f(t);
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + e);
}
__device__ __forceinline__ float tanh_fast(float x) { return tanh_pre(x * kTanhScale); }
template <bool kPre>  // kPre: the argument is already x kTanhScale
__device__ __forceinline__ float tanh_act(float z) {
  if constexpr (kPre) return tanh_pre(z);
  else return tanh_fast(z);
}

// ---------------------------------------------------------------------------------------------
// Wave-scope LDS ordering: LDS ops of one wave complete in order, so a wave that only talks to
// itself through LDS needs a compiler fence, not an s_barrier (no cross-wave hand-off here).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
  return v;
}

// theta'[p] = fl32(base[p] +/- fl32(sigma * eps[p]))  -- no contraction (bit-exact with numpy).
// Branch-free: eps is always a readable address (the lane's base when it is not perturbed -- its value is then
// discarded by the select), so every element's two loads are unconditional and the compiler batches them.  (r12: a
// per-element `if (sgn != 0)` around the eps load put each load behind its own exec branch and wait -- ~200 serialised
// HBM round trips per thread in the MLP rollouts' prologue.)
struct ParamSrc {
  const float* base;
  const float* eps;  // table + idx, or base (unperturbed lane: loaded, not used)
  float sigma;
  int sgn;           // +1 / -1 / 0
  double n2;         // running sum of fl32(sigma*eps)^2 over the elements this thread loaded

  __device__ __forceinline__ float get(int64_t p) {
#pragma clang fp contract(off)
    const float t = base[p];
    const float st = sigma * eps[p];
    const double d = (double)st;
    n2 += sgn != 0 ? d * d : 0.0;
    return sgn > 0 ? t + st : (sgn < 0 ? t - st : t);
  }
  // get(p) counted in n2 only when `use` (an element read unconditionally from a clamped index whose value the caller
  // discards otherwise: no load behind a branch)
  __device__ __forceinline__ float get_if(int64_t p, bool use) {
#pragma clang fp contract(off)
    const float t = base[p];
    const float st = sigma * eps[p];
    const double d = (double)st;
    n2 += (use && sgn != 0) ? d * d : 0.0;
    return sgn > 0 ? t + st : (sgn < 0 ? t - st : t);
  }
  // same value, but not counted in n2 (an element several threads replicate)
  __device__ __forceinline__ float get_nocount(int64_t p) const {
#pragma clang fp contract(off)
    const float t = base[p];
    const float st = sigma * eps[p];
    return sgn > 0 ? t + st : (sgn < 0 ? t - st : t);
  }
};

}  // namespace fdr
