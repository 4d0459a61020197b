// Cross-lane primitives for the one-wave-per-lane MLP (gfx950, wave64 = 4 rows x 16 lanes).
//
// Measured on MI355X (tools/probes/dpp_probe.hip):
//   * DPP row_newbcast:k broadcasts lane k of each 16-lane row to the whole row, and can be an
//     operand modifier of v_fmac_f32 -> an FMA whose input vector element comes from another lane
//     costs ONE VALU instruction and no LDS traffic.
//   * v_permlane32_swap / v_permlane16_swap exchange halves / odd-even rows between two VGPRs.
//     The ROCm 7.2 builtins return a wrong second result, so they are used through inline asm.
// Hazards (hipcc does not pad inline asm): a VALU write of a DPP / permlane source needs 2 wait
// states, a VALU write of EXEC needs 5 before a DPP op -> each asm block starts with s_nop.
#pragma once
#include <hip/hip_runtime.h>

namespace fdr {

__device__ __forceinline__ void permlane32_swap(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void permlane16_swap(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}

// All-gather of a 64-element vector x (x[k] in lane k) into NQ row-replicated registers:
// X[q] in lane (r, c) = x[16 q + c] for every row r.
template <int NQ>
__device__ __forceinline__ void row_allgather(float x, float (&X)[NQ]) {
  static_assert(NQ >= 1 && NQ <= 4, "NQ in 1..4");
  float a = x, b = x;
  permlane32_swap(a, b);  // a = [x0 x1 x0 x1], b = [x2 x3 x2 x3]   (rows of 16)
  float c = a, d = a;
  permlane16_swap(c, d);  // c = [x0 x0 x0 x0], d = [x1 x1 x1 x1]
  X[0] = c;
  if constexpr (NQ > 1) X[1] = d;
  if constexpr (NQ > 2) {
    float e = b, f = b;
    permlane16_swap(e, f);  // e = [x2 ...], f = [x3 ...]
    X[2] = e;
    if constexpr (NQ > 3) X[3] = f;
  }
}

// Sum over the 4 rows (lane (r, c) ends with sum_r' v(r', c)); order: (r0+r2) + (r1+r3).
__device__ __forceinline__ float row_allreduce_sum(float v) {
  float a = v, b = v;
  permlane32_swap(a, b);  // a = [v0 v1 v0 v1], b = [v2 v3 v2 v3]
  float s = a + b;        // [v0+v2, v1+v3, v0+v2, v1+v3]
  float c = s, d = s;
  permlane16_swap(c, d);  // c = [s0 s0 s0 s0], d = [s1 s1 s1 s1]
  return c + d;
}

#define FDR_DPP_LINE(I, K) \
  "v_fmac_f32_dpp %0, %1, %" #I " row_newbcast:" #K " row_mask:0xf bank_mask:0xf\n\t"

// acc += sum_{c=0}^{15} w[c] * X(row lane c)   -- 16 FMAs, X broadcast by DPP
__device__ __forceinline__ void fmac_bcast16(float& acc, float X, const float* w) {
  asm volatile("s_nop 4\n\t"
      FDR_DPP_LINE(2, 0) FDR_DPP_LINE(3, 1) FDR_DPP_LINE(4, 2) FDR_DPP_LINE(5, 3)
      FDR_DPP_LINE(6, 4) FDR_DPP_LINE(7, 5) FDR_DPP_LINE(8, 6) FDR_DPP_LINE(9, 7)
      FDR_DPP_LINE(10, 8) FDR_DPP_LINE(11, 9) FDR_DPP_LINE(12, 10) FDR_DPP_LINE(13, 11)
      FDR_DPP_LINE(14, 12) FDR_DPP_LINE(15, 13) FDR_DPP_LINE(16, 14) FDR_DPP_LINE(17, 15)
      : "+v"(acc)
      : "v"(X), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]),
        "v"(w[7]), "v"(w[8]), "v"(w[9]), "v"(w[10]), "v"(w[11]), "v"(w[12]), "v"(w[13]),
        "v"(w[14]), "v"(w[15]));
}

// acc += w * X(row lane K)   -- one FMA (own hazard pad)
template <int K>
__device__ __forceinline__ void fmac_bcast1(float& acc, float X, float w) {
  asm volatile("s_nop 4\n\tv_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc)
               : "v"(X), "v"(w), "i"(K));
}

template <int K0, int N>
__device__ __forceinline__ void fmac_bcast_tail(float& acc, float X, const float* w) {
  if constexpr (N > 0) {
    fmac_bcast1<K0>(acc, X, w[0]);
    fmac_bcast_tail<K0 + 1, N - 1>(acc, X, w + 1);
  }
}

// acc += sum_{k<N} w[k] * x[k], with x given as its row all-gather X (x[k] = X[k/16](lane k%16)).
template <int N, int NQ>
__device__ __forceinline__ void fmac_vec(float& acc, const float (&X)[NQ], const float* w) {
  static_assert((N + 15) / 16 <= NQ, "not enough gathered rows");
#pragma unroll
  for (int q = 0; q < N / 16; ++q) fmac_bcast16(acc, X[q], w + 16 * q);
  if constexpr (N % 16 != 0) fmac_bcast_tail<0, N % 16>(acc, X[N / 16], w + N / 16 * 16);
}

// DPP moves within a row (bound_ctrl -> 0 outside the row)
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
constexpr int kDppQuadXor1 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int kDppQuadXor2 = 0x4E;   // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;
constexpr int kDppMirror = 0x140;
constexpr int kDppRowShl = 0x100;    // + n : lane i <- lane i + n (same row)

// all-reduce within each 16-lane row
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_mov<kDppQuadXor1>(v));
  v = fmaxf(v, dpp_mov<kDppQuadXor2>(v));
  v = fmaxf(v, dpp_mov<kDppHalfMirror>(v));
  v = fmaxf(v, dpp_mov<kDppMirror>(v));
  return v;
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<kDppQuadXor1>(v);
  v += dpp_mov<kDppQuadXor2>(v);
  v += dpp_mov<kDppHalfMirror>(v);
  v += dpp_mov<kDppMirror>(v);
  return v;
}

__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

}  // namespace fdr
