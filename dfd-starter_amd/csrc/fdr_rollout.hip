// fdr_rollout.hip -- whole-episode batched rollouts and batched policy forwards for the FD engine.
//
// Design (DESIGN.md "Rollout kernel"):
//   * ONE WAVE PER LANE (lane = one perturbation x env).  Hidden width 64 == wave width: wave lane
//     j owns hidden unit j of both layers and keeps its weight rows in VGPRs for the whole episode
//     (W1 row j, W2 row j, a 16-input slice of W3) -- theta' is read from HBM once per episode,
//     never per step.  The kernel is fp32-VALU-bound, not HBM-bound.
//   * theta'_l is built on the fly from theta + sign_l * fl32(sigma * table[idx_l + p])
//     (bit-exact with worker/worker.py:28) while loading those registers; the same pass
//     accumulates ||lambda_l||^2 for the learner (learner/finite_differences.py:107).
//   * Activations cross lanes through a 1 KiB per-wave LDS scratch (one ds_write_b32 per lane,
//     broadcast ds_read_b128 back) feeding packed f32 FMAs, or through DPP row_newbcast where the
//     input already sits in the caller's 16-lane row (the head, K a).
//   * The env (synthetic linear-tanh system or the trap gridworld) runs inside the same loop.
//   * 4 lanes (waves) per 256-thread workgroup, <= 128 VGPRs -> 16 waves/CU: 4096 lanes fill
//     all 256 CUs in one wave of workgroups.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <utility>

#include "fdr_common.h"
#include "fdr_internal.h"
#include "fdr_wave.h"

namespace fdr {

constexpr int kLanesPerBlock = 4;

#ifdef FDR_PHASE_STAMPS
// diagnostics build only (make stamps): s_memtime cycles per step phase of wave 0 of block 0
// -- policy L1, L2, head, action, env -- summed over the episode (tools/rollout_phases.py)
__device__ unsigned long long g_phase_stamps[5];
#endif

__host__ __device__ constexpr int round4(int x) { return (x + 3) / 4 * 4; }

// Flat parameter layout = nn.Module.parameters() order (policies/policy.py:36-42).
template <int NIN, int NA, bool DISC>
struct Layout {
  static constexpr int H = kHidden;
  static constexpr int NOUT = DISC ? NA : 2 * NA;
  // discrete: bn0.w bn0.b l1.w l1.b bn1.w bn1.b l2.w l2.b bn2.w bn2.b l3.w l3.b
  // mujoco:   l1.w l1.b l2.w l2.b l3.w l3.b
  static constexpr int64_t BN0W = 0;
  static constexpr int64_t BN0B = NIN;
  static constexpr int64_t L1W = DISC ? 2 * NIN : 0;
  static constexpr int64_t L1B = L1W + H * NIN;
  static constexpr int64_t BN1W = L1B + H;
  static constexpr int64_t BN1B = BN1W + H;
  static constexpr int64_t L2W = DISC ? BN1B + H : L1B + H;
  static constexpr int64_t L2B = L2W + H * H;
  static constexpr int64_t BN2W = L2B + H;
  static constexpr int64_t BN2B = BN2W + H;
  static constexpr int64_t L3W = DISC ? BN2B + H : L2B + H;
  static constexpr int64_t L3B = L3W + NOUT * H;
  static constexpr int64_t P = L3B + NOUT;
  static_assert(NOUT <= 16, "policy head wider than 16 outputs not compiled");
  static_assert(NIN <= 64, "observation wider than 64 not supported");
};

// trap-env observation (environment.py:59-61): python f64 division, cast to f32 by the policy
__device__ __forceinline__ float trap_obs(int j, int col, int row) {
  return j == 0 ? (float)((double)(col * 7) / 1918.0) : (float)((double)(row * 7) / 1071.0);
}

// torch: two separately rounded tensor ops (utils/torch_helpers.py:25, Normal.sample).
__device__ __forceinline__ float std_from_tanh(float t) {
#pragma clang fp contract(off)
  return 0.55f + 0.45f * t;
}
__device__ __forceinline__ float gauss_action(float mean, float std, float z) {
#pragma clang fp contract(off)
  return mean + std * z;
}
// eval BatchNorm as torch CPU computes it: alpha = w * invstd, beta = b - mean * alpha
__device__ __forceinline__ void bn_fold(float w, float b, float rm, float rv, float& a, float& c) {
#pragma clang fp contract(off)
  const float invstd = 1.0f / sqrtf(rv + 1e-5f);
  a = invstd * w;
  c = b - rm * a;
}

// Categorical entropy term p_n log2 p_n of a discrete action (p_n = p / tot, torch normalises probs;
// the ln 2 scale is applied once in the epilogue).  Fast reciprocal and log2: the entropy is a reported
// statistic (parity 1e-5), not an input to the trajectory; terms below 1e-30 contribute nothing.
__device__ __forceinline__ float disc_entropy_term(float p, float tot) {
  const float pn = p * __builtin_amdgcn_rcpf(tot);
  return pn > 1e-30f ? pn * __builtin_amdgcn_logf(pn) : 0.f;
}

// ---------------------------------------------------------------------------------------------
// One lane's policy, register resident.
//
// Matvecs run on packed f32 FMAs (v_pk_fma_f32, two MACs per instruction) over operands that sit
// in the lane's own registers -- DPP-operand FMAs issue at ~4.7 cycles per wave-instruction on
// gfx950 (tools/probes/valu_probe.hip) and were the rollout's bottleneck.  Activations cross lanes
// through a 1 KiB per-wave LDS scratch: one ds_write_b32 per lane, broadcast ds_read_b128 back.
//
//   L1 (NIN -> 64)  broadcast input (LDS), lane j: row j of W1 (VGPR pairs, or the per-wave LDS
//                   tile when NIN > 8; bias folded into the padding column); output j in lane j.
//   env (M s + K a) M s in the same pass as L1 over the broadcast input chunks (lane j < NIN: row j
//                   of M from the block's LDS copy); K a by DPP row_newbcast FMAs once the action
//                   (lanes 0 .. NA-1 of every row) is known.
//   L2 (64 -> 64)   8 x 8 lane blocks: lane (r = j/8, c = j%8) holds W2[8r + pi_c(i)][8c + k]
//                   (i, k < 8; 64 VGPRs), reads x[8c .. 8c + 7] (two b128), accumulates 8
//                   partial outputs in 4 packed pairs, then a 3-level reduce-scatter over the 8
//                   lanes of its half-row (DPP half_mirror, quad xor 2, quad xor 1: 7 adds)
//                   leaves output 8r + c = j in lane j.  pi_c(i) = c ^ sigma(i),
//                   sigma = (0 1 2 3 7 6 5 4), is the register order that makes every level send
//                   the partner exactly the outputs it keeps.
//   head (64 -> NOUT <= 16)  lane (q = j/16, o = j%16): W3[o][16q .. 16q + 15] against h2[16q + i],
//                   which sits in lane i of the lane's own row q (DPP row_newbcast FMAs, no LDS round
//                   trip), then the 4-row all-reduce (two permlane swaps).
// ---------------------------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
// c + a * (b.x, b.x) / c + a * (b.y, b.y): one element of a register pair broadcast by op_sel (hipcc 7.2 moves an
// odd element of a b128 load to an even register first: a v_mov per broadcast operand otherwise)
__device__ __forceinline__ f2 pk_fma_blo(f2 a, f2 b, f2 c) {
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(c) : "v"(a), "v"(b));
  return c;
}
__device__ __forceinline__ f2 pk_fma_bhi(f2 a, f2 b, f2 c) {
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(c) : "v"(a), "v"(b));
  return c;
}

// a * (b.x, b.x) / a * (b.y, b.y): the first term of an op_sel chain (no zeroed accumulator to move in)
__device__ __forceinline__ f2 pk_mul_blo(f2 a, f2 b) {
  f2 c;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(c) : "v"(a), "v"(b));
  return c;
}
__device__ __forceinline__ f2 pk_mul_bhi(f2 a, f2 b) {
  f2 c;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(c) : "v"(a), "v"(b));
  return c;
}

__host__ __device__ constexpr int l2_sigma(int i) { return i < 4 ? i : 11 - i; }

// per-wave LDS scratch for the cross-lane hand-offs of one step (16-B aligned slots).  LDS ops of
// one wave complete in order: a slot is rewritten only after the reads of its previous contents.
struct alignas(16) WaveScratch {
  float h1[kHidden];  // layer-1 output (L2 input); the env state when it differs from the policy input
  float x[kWave];     // policy input (+ the 1 of the folded bias column), written by every lane
};

template <int N>
__device__ __forceinline__ void lds_bcast(const float* v, float (&x)[N]) {  // N % 4 == 0
  const float4* v4 = reinterpret_cast<const float4*>(v);
#pragma unroll
  for (int q = 0; q < N / 4; ++q) {
    const float4 t = v4[q];
    x[4 * q] = t.x;
    x[4 * q + 1] = t.y;
    x[4 * q + 2] = t.z;
    x[4 * q + 3] = t.w;
  }
}

// sum_k w[k] x[k] over a 16-B aligned LDS row (N % 4 == 0), two packed partial sums
template <int N>
__device__ __forceinline__ float dot_lds_row(const float* w, const float (&x)[N], float init) {
  const float4* w4 = reinterpret_cast<const float4*>(w);
  f2 acc = {init, 0.f};
#pragma unroll
  for (int q = 0; q < N / 4; ++q) {
    const float4 t = w4[q];
    acc = pk_fma(f2{t.x, t.y}, f2{x[4 * q], x[4 * q + 1]}, acc);
    acc = pk_fma(f2{t.z, t.w}, f2{x[4 * q + 2], x[4 * q + 3]}, acc);
  }
  return acc.x + acc.y;
}

template <int NIN, int NA, bool DISC>
struct MlpLane {
  using L = Layout<NIN, NA, DISC>;
  using Scratch = WaveScratch;
  static constexpr int NOUT = L::NOUT;
  static constexpr int NX = round4(NIN);
  static constexpr bool kBiasCol = NIN < NX;  // b1 sits in W1 column NIN (input NIN == 1)
  // Per-wave LDS tile of lane-private weights, float4 chunks laid out [chunk][lane] (conflict-free
  // b128): W1 row j when NIN > 8 (bias folded into column NIN), then W3[o][16q .. 16q + 15].
  // Keeping them out of VGPRs leaves room for whole-row loads in flight (<= 128 VGPRs, 4 waves/SIMD);
  // the W3 chunks are read in the same LDS round trip as the head's input.
  static constexpr bool kW1Lds = NIN > 8;
  static constexpr int kW1Chunks = kW1Lds ? NX / 4 : 0;
  static constexpr int kTileF4 = (kW1Chunks + 4) * kWave;  // float4 per wave
  f2 w1[kW1Lds ? 1 : NX / 2];
  float b1;
  const float4* tile;  // this lane's column of the tile (chunk m at tile[m * kWave])
  f2 w2[32];           // w2[p * 8 + k] = (W2[8r + pi_c(2p)][8c + k], W2[8r + pi_c(2p + 1)][8c + k])
  float b2;
  float b3;
  float a0, c0, a1, c1, a2, c2;  // discrete: folded BN for input j / hidden unit j

  __device__ __forceinline__ void load(ParamSrc& src, int j, const float* bn_mean,
                                       const float* bn_var, float4* lds_tile) {
    const int r = j >> 3, c = j & 7, o = j & 15, q = j >> 4;
    tile = lds_tile + j;
    float4* my = lds_tile + j;
    auto w1v = [&](int k) {
      return k < NIN ? src.get(L::L1W + (int64_t)j * NIN + k) : (k == NIN ? src.get(L::L1B + j) : 0.f);
    };
    if constexpr (kW1Lds) {
#pragma unroll
      for (int m = 0; m < kW1Chunks; ++m) {
        const float e0 = w1v(4 * m), e1 = w1v(4 * m + 1), e2 = w1v(4 * m + 2), e3 = w1v(4 * m + 3);
        my[m * kWave] = float4{e0, e1, e2, e3};
      }
    } else {
#pragma unroll
      for (int p = 0; p < NX / 2; ++p) {
        const float e0 = w1v(2 * p), e1 = w1v(2 * p + 1);
        w1[p] = f2{e0, e1};
      }
    }
    b1 = kBiasCol ? 0.f : src.get(L::L1B + j);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row0 = 8 * r + (c ^ l2_sigma(2 * p)), row1 = 8 * r + (c ^ l2_sigma(2 * p + 1));
#pragma unroll
      for (int k = 0; k < 8; ++k)
        w2[p * 8 + k] = f2{src.get(L::L2W + (int64_t)row0 * kHidden + 8 * c + k),
                           src.get(L::L2W + (int64_t)row1 * kHidden + 8 * c + k)};
      // the group's weights and norm terms are final here (MlpPair::load: no deferred selects held in scratch)
#pragma unroll
      for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(w2[p * 8 + k]));
      asm volatile("" : "+v"(src.n2));
      __builtin_amdgcn_sched_barrier(0);
    }
    b2 = src.get(L::L2B + j);
    // Branch-free from here (r12): a load behind a condition ends its block with a vmcnt(0) wait.  The head rows
    // and the input BN are read from clamped indices by every lane, counted and kept only where they exist; the
    // running stats from a valid address whether or not they were given.
    {
      const bool has_o = o < NOUT;
      const int oc = has_o ? o : 0;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int64_t base = L::L3W + (int64_t)oc * kHidden + 16 * q + 4 * m;
        const float e0 = src.get_if(base, has_o), e1 = src.get_if(base + 1, has_o), e2 = src.get_if(base + 2, has_o),
                    e3 = src.get_if(base + 3, has_o);
        my[(kW1Chunks + m) * kWave] = has_o ? float4{e0, e1, e2, e3} : float4{0.f, 0.f, 0.f, 0.f};
      }
      const float b3v = src.get_if(L::L3B + oc, has_o && q == 0);
      b3 = has_o ? b3v : 0.f;
    }
    wave_lds_sync();
    a0 = c0 = a1 = c1 = a2 = c2 = 0.f;
    if constexpr (DISC) {
      const float* bm = bn_mean ? bn_mean : src.base;  // a readable address either way
      const float* bv = bn_var ? bn_var : src.base;
      auto stat = [&](int k, float& rm, float& rv) {
        const float m = bm[k], v = bv[k];
        rm = bn_mean ? m : 0.f;
        rv = bn_var ? v : 1.f;
      };
      {
        const bool in = j < NIN;
        const int jc = in ? j : 0;
        const float w = src.get_if(L::BN0W + jc, in), b = src.get_if(L::BN0B + jc, in);
        float rm, rv, a, c;
        stat(jc, rm, rv);
        bn_fold(w, b, rm, rv, a, c);
        a0 = in ? a : 0.f;
        c0 = in ? c : 0.f;
      }
      {
        const float w = src.get(L::BN1W + j), b = src.get(L::BN1B + j);
        float rm, rv;
        stat(NIN + j, rm, rv);
        bn_fold(w, b, rm, rv, a1, c1);
      }
      {
        const float w = src.get(L::BN2W + j), b = src.get(L::BN2B + j);
        float rm, rv;
        stat(NIN + kHidden + j, rm, rv);
        bn_fold(w, b, rm, rv, a2, c2);
      }
    }
  }

  // policy input for lane j < NIN from the (already obs-normalised) observation value
  __device__ __forceinline__ float input_transform(float x) const {
    if constexpr (DISC) {
      return fmaf(x, a0, c0);  // BatchNorm1d(n_in), eval mode
    } else {
      return x;
    }
  }

  // First hidden layer of unit j against the broadcast input xs (xs[NIN] == 1 picks up the folded
  // bias).
  __device__ __forceinline__ float layer1(const float (&xs)[NX]) const {
    f2 acc = {b1, 0.f};
    if constexpr (kW1Lds) {
#pragma unroll
      for (int q = 0; q < NX / 4; ++q) {
        const float4 w = tile[q * kWave];
        acc = pk_fma(f2{w.x, w.y}, f2{xs[4 * q], xs[4 * q + 1]}, acc);
        acc = pk_fma(f2{w.z, w.w}, f2{xs[4 * q + 2], xs[4 * q + 3]}, acc);
      }
    } else {
#pragma unroll
      for (int p = 0; p < NX / 2; ++p) acc = pk_fma(w1[p], f2{xs[2 * p], xs[2 * p + 1]}, acc);
    }
    const float z = acc.x + acc.y;
    if constexpr (DISC) {
      return fmaf(fmaxf(z, 0.f), a1, c1);
    } else {
      return tanh_fast(z);
    }
  }

  // First hidden layer and the env's M s in one pass over the broadcast input chunks (LDS):
  // returns unit j's activation, sets env = M[j] . x.  Chunks are consumed as they arrive so at most
  // two are live (VGPR budget: W2 holds 64 of the 128).
  // ss: the env state's broadcast copy when it differs from the policy input (nullptr: same)
  template <bool kSameInput>
  __device__ __forceinline__ float layer1_env_pk(const float* xs, const float* ss, const float* mrow,
                                                 float& env) const {
    const float4* x4 = reinterpret_cast<const float4*>(xs);
    const float4* s4 = reinterpret_cast<const float4*>(ss);
    const float4* m4 = reinterpret_cast<const float4*>(mrow);
    // four independent chains: back-to-back dependent packed FMAs cost an s_nop each
    f2 acc0 = {b1, 0.f}, acc1 = {0.f, 0.f}, accm0 = {0.f, 0.f}, accm1 = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NX / 4; ++q) {
      const float4 xv = x4[q], mv = m4[q];
      const float4 sv = kSameInput ? xv : s4[q];
      float4 w;
      if constexpr (kW1Lds) {
        w = tile[q * kWave];
      } else {
        w = float4{w1[2 * q].x, w1[2 * q].y, w1[2 * q + 1].x, w1[2 * q + 1].y};
      }
      acc0 = pk_fma(f2{w.x, w.y}, f2{xv.x, xv.y}, acc0);
      accm0 = pk_fma(f2{mv.x, mv.y}, f2{sv.x, sv.y}, accm0);
      acc1 = pk_fma(f2{w.z, w.w}, f2{xv.z, xv.w}, acc1);
      accm1 = pk_fma(f2{mv.z, mv.w}, f2{sv.z, sv.w}, accm1);
    }
    const f2 am = accm0 + accm1, ah = acc0 + acc1;
    env = am.x + am.y;
    const float z = ah.x + ah.y;
    if constexpr (DISC) {
      return fmaf(fmaxf(z, 0.f), a1, c1);
    } else {
      return tanh_fast(z);
    }
  }

  // Layer 1 and the env's M s from register-resident operands (rollout_kernel<WIDE>): the broadcast
  // input arrives through v_readlane (wave-uniform values), M row j is loop-invariant in VGPRs.
  __device__ __forceinline__ float layer1_env_reg(const float (&xv)[NX], const float (&sv)[NX],
                                                  const float (&mv)[NX], float& env) const {
    static_assert(!kW1Lds, "register-input layer 1 needs W1 in VGPRs");
    f2 acc0 = {b1, 0.f}, acc1 = {0.f, 0.f}, accm0 = {0.f, 0.f}, accm1 = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NX / 4; ++q) {
      acc0 = pk_fma(w1[2 * q], f2{xv[4 * q], xv[4 * q + 1]}, acc0);
      accm0 = pk_fma(f2{mv[4 * q], mv[4 * q + 1]}, f2{sv[4 * q], sv[4 * q + 1]}, accm0);
      acc1 = pk_fma(w1[2 * q + 1], f2{xv[4 * q + 2], xv[4 * q + 3]}, acc1);
      accm1 = pk_fma(f2{mv[4 * q + 2], mv[4 * q + 3]}, f2{sv[4 * q + 2], sv[4 * q + 3]}, accm1);
    }
    const f2 am = accm0 + accm1, ah = acc0 + acc1;
    env = am.x + am.y;
    const float z = ah.x + ah.y;
    if constexpr (DISC) {
      return fmaf(fmaxf(z, 0.f), a1, c1);
    } else {
      return tanh_fast(z);
    }
  }

  // this lane's W3 slice (the head's loop-invariant LDS tile chunks) into registers
  __device__ __forceinline__ void head_weights(float (&w3)[16]) const {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const float4 w = tile[(kW1Chunks + m) * kWave];
      w3[4 * m] = w.x;
      w3[4 * m + 1] = w.y;
      w3[4 * m + 2] = w.z;
      w3[4 * m + 3] = w.w;
    }
  }

  // second hidden layer and the head: h = layer-1 output of unit j; returns the head
  // pre-activation for output o = j & 15 (identical in the 4 rows).  w3r: the head's W3 slice when the
  // caller keeps it in registers (nullptr: read from the LDS tile each step).
  template <class Mark>
  __device__ __forceinline__ float layers23(float h, Scratch* sc, int j, Mark&& mark,
                                            const float* w3r = nullptr) const {
    const float h2 = layer2(h, sc, j);
    mark(1, h2);
    // h2[16q + i] sits in lane i of row q: DPP row_newbcast FMAs, no LDS round trip
    float w3[16];
    if (w3r) {
#pragma unroll
      for (int i = 0; i < 16; ++i) w3[i] = w3r[i];
    } else {
      head_weights(w3);
    }
    const float out = row_allreduce_sum(dot_row16(h2, w3)) + b3;
    mark(2, out);
    return out;
  }

  // Two-output head (discrete NA == 2, rollout_kernel<WIDE>): lane j multiplies its own unit h2[j] by
  // w3c = (W3[0][j], W3[1][j]), keeps the product of output o = j & 1 and hands the other to its quad
  // partner, then sums over the 32 lanes of its parity (row_ror 4, row_ror 8, quad xor 2, the 4-row
  // permlane all-reduce): output o in every lane of parity o, 9 VALU instead of the 16-DPP-FMA dot.
  // kKeepFirst: w3c already holds (W3[o][j], W3[1 - o][j]) (the WIDE kernel), so no selects
  template <bool kKeepFirst = false>
  __device__ __forceinline__ float head2(float h2, f2 w3c, float b3p, int j) const {
    const f2 m = w3c * f2{h2, h2};
    const bool odd = !kKeepFirst && (j & 1) != 0;
    const float keep = odd ? m.y : m.x, give = odd ? m.x : m.y;
    float v = keep + dpp_mov<kDppQuadXor1>(give);
    v += dpp_mov<kDppRowRor + 4>(v);
    v += dpp_mov<kDppRowRor + 8>(v);
    v += dpp_mov<kDppQuadXor2>(v);
    return row_allreduce_sum(v) + b3p;
  }

  // second hidden layer: h = layer-1 output of unit j; returns unit j's activation.  kAsm (the 256-VGPR WIDE
  // kernel only: in the 128-VGPR instances the asm block's live range spills): op_sel block, b2 in the own slot
  template <bool kAsm = false>
  __device__ __forceinline__ float layer2(float h, Scratch* sc, int j) const {
    const int c = j & 7;
    sc->h1[j] = h;
    wave_lds_sync();
    float x[8];
    lds_bcast<8>(sc->h1 + 8 * c, x);
    f2 acc[4];
    float kB2;
    if constexpr (kAsm) {
    // k = 0 starts the lane's own slot (acc[0].x, the reduce-scatter's non-DPP operand all the way down) from b2;
    // k = 1 .. 7 as op_sel broadcasts of the pairs (x[2j], x[2j + 1]) in one asm statement (no moves of odd
    // elements; operands %0-%3 acc, %(4 + 4 (k - 1) + p) = w2[8 p + k], %32-%35 the pairs)
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[p] = pk_fma(w2[p * 8], f2{x[0], x[0]}, f2{p == 0 ? b2 : 0.f, 0.f});
    {
      const f2 x01 = {x[0], x[1]}, x23 = {x[2], x[3]}, x45 = {x[4], x[5]}, x67 = {x[6], x[7]};
#define FDR_L2_HI "op_sel:[0,1,0] op_sel_hi:[1,1,1]"
#define FDR_L2_LO "op_sel_hi:[1,0,1]"
      asm(
          "v_pk_fma_f32 %0, %4, %32, %0 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %1, %5, %32, %1 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %2, %6, %32, %2 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %3, %7, %32, %3 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %0, %8, %33, %0 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %1, %9, %33, %1 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %2, %10, %33, %2 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %3, %11, %33, %3 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %0, %12, %33, %0 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %1, %13, %33, %1 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %2, %14, %33, %2 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %3, %15, %33, %3 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %0, %16, %34, %0 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %1, %17, %34, %1 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %2, %18, %34, %2 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %3, %19, %34, %3 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %0, %20, %34, %0 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %1, %21, %34, %1 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %2, %22, %34, %2 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %3, %23, %34, %3 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %0, %24, %35, %0 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %1, %25, %35, %1 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %2, %26, %35, %2 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %3, %27, %35, %3 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %0, %28, %35, %0 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %1, %29, %35, %1 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %2, %30, %35, %2 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %3, %31, %35, %3 " FDR_L2_HI "\n"
          : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])
          : "v"(w2[1]), "v"(w2[9]), "v"(w2[17]), "v"(w2[25]),
            "v"(w2[2]), "v"(w2[10]), "v"(w2[18]), "v"(w2[26]),
            "v"(w2[3]), "v"(w2[11]), "v"(w2[19]), "v"(w2[27]),
            "v"(w2[4]), "v"(w2[12]), "v"(w2[20]), "v"(w2[28]),
            "v"(w2[5]), "v"(w2[13]), "v"(w2[21]), "v"(w2[29]),
            "v"(w2[6]), "v"(w2[14]), "v"(w2[22]), "v"(w2[30]),
            "v"(w2[7]), "v"(w2[15]), "v"(w2[23]), "v"(w2[31]),
            "v"(x01), "v"(x23), "v"(x45), "v"(x67));
#undef FDR_L2_LO
#undef FDR_L2_HI
    }
    kB2 = 0.f;
    } else {
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[p] = f2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int p = 0; p < 4; ++p) acc[p] = pk_fma(w2[p * 8 + k], f2{x[k], x[k]}, acc[p]);
    kB2 = b2;
    }
    // reduce-scatter over the 8 lanes of the half-row: slot i = acc[i / 2][i % 2]
    const float q0 = acc[0].x + dpp_mov<kDppHalfMirror>(acc[2].x);
    const float q1 = acc[0].y + dpp_mov<kDppHalfMirror>(acc[2].y);
    const float q2 = acc[1].x + dpp_mov<kDppHalfMirror>(acc[3].x);
    const float q3 = acc[1].y + dpp_mov<kDppHalfMirror>(acc[3].y);
    const float r0 = q0 + dpp_mov<kDppQuadXor2>(q2);
    const float r1 = q1 + dpp_mov<kDppQuadXor2>(q3);
    const float z = kAsm ? r0 + dpp_mov<kDppQuadXor1>(r1) : (r0 + dpp_mov<kDppQuadXor1>(r1)) + kB2;
    if constexpr (DISC) {
      return fmaf(fmaxf(z, 0.f), a2, c2);
    } else {
      return tanh_fast(z);
    }
  }

  // Discrete: softmax across the row (o = j & 15 < NA); returns p_o, 0 for o >= NA.  kAll: every lane
  // holds a logit (head2: output j & 1).  kFast (sampled lanes): exp as v_exp_f32 of x log2 e and
  // the normalisation as a v_rcp_f32 product -- 4 VALU instead of libm expf (13) + the IEEE division (11); the
  // probabilities move by ~1e-7 relative (inside the 1e-5 forward tolerance), so a sampled action can differ
  // from the exact form's only where u * sum p lies within that of a partition boundary.  Deterministic lanes
  // (argmax, the trap env's integer-exact episodes) keep the exact form.
  template <bool kAll = false, bool kFast = false>
  __device__ __forceinline__ float softmax(float logit, int j) const {
    const bool valid = kAll || (j & 15) < NOUT;
    const float v = valid ? logit : -FLT_MAX;
    const float mx = row16_max_n<NOUT>(v);
    if constexpr (kFast) {
      const float e = valid ? __builtin_amdgcn_exp2f((v - mx) * 1.44269504088896341f) : 0.f;
      return e * __builtin_amdgcn_rcpf(row16_sum_n<NOUT>(e));
    } else {
      const float e = valid ? expf(v - mx) : 0.f;
      return e / row16_sum_n<NOUT>(e);
    }
  }
};

// ---------------------------------------------------------------------------------------------
// Batched single-step forward: fdr_policy_forward
// ---------------------------------------------------------------------------------------------
template <int NIN, int NA, bool DISC>
__global__ __launch_bounds__(64 * kLanesPerBlock) void policy_forward_kernel(
    LanesArgs lanes, int n_lanes, const float* __restrict__ bn_mean,
    const float* __restrict__ bn_var, const float* __restrict__ x, float* __restrict__ out0,
    float* __restrict__ out1) {
  using Lane = MlpLane<NIN, NA, DISC>;
  __shared__ float4 wtile[kLanesPerBlock * Lane::kTileF4];
  __shared__ typename Lane::Scratch scratch[kLanesPerBlock];
  const int j = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int lane = blockIdx.x * kLanesPerBlock + wv;
  if (lane >= n_lanes) return;
  ParamSrc src = lanes.src(lane);
  Lane pl;
  pl.load(src, j, bn_mean, bn_var, wtile + wv * Lane::kTileF4);
  auto* sc = &scratch[wv];
  sc->x[j] = j < NIN ? pl.input_transform(x[(int64_t)lane * NIN + j]) : (j == NIN ? 1.f : 0.f);
  wave_lds_sync();
  float xb[Lane::NX];
  lds_bcast<Lane::NX>(sc->x, xb);
  const float y = pl.layers23(pl.layer1(xb), sc, j, [](int, float) {});
  if constexpr (DISC) {
    const float p = pl.softmax(y, j);
    if (j < NA) out0[(int64_t)lane * NA + j] = p;
  } else {
    const float t = tanh_fast(y);
    const float ts = dpp_mov<kDppRowShl + NA>(t);  // lane o <- lane o + NA: the std half
    if (j < NA) {
      out0[(int64_t)lane * NA + j] = t;
      out1[(int64_t)lane * NA + j] = std_from_tanh(ts);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Whole-episode rollout: fdr_rollout
// ---------------------------------------------------------------------------------------------
// FEAT bit 0: record visited observations (fdr_rollout_states); bit 1: Welford obs statistics;
// bit 2: observation normalisation (obs_mean / obs_std given); bit 3: host-injected draws (u_inject);
// bit 4: terminating synthetic env (fdr_env_desc.done_threshold): the lane's episode ends after the step whose
// next state has |s'[done_dim]| > done_threshold (worker/agent.py:50-52: done -> break), or at T
// (one lane per wave: the wave leaves its loop -- only these instances carry the test)
// WIDE (synthetic env, few lanes: <= 2 waves per SIMD): a 256-VGPR budget instead of 128, so the
// step's loop invariants (M / K rows, the head's W3 slice) stay in registers; the policy input and env
// state cross lanes by v_readlane instead of an LDS round trip (NIN <= 8); a discrete env's candidate
// next states tanh(M s + K[:, a]) are formed for every action while the policy runs, so the action
// only selects one.
template <int NIN, int NA, bool DISC, int ENV, int FEAT, bool WIDE>
__global__ __launch_bounds__(64 * kLanesPerBlock, WIDE ? 2 : 4) void rollout_kernel(RolloutArgs a) {
  using Lane = MlpLane<NIN, NA, DISC>;
  constexpr int NX = Lane::NX;
  constexpr bool kRegIn = WIDE && ENV == FDR_ENV_SYNTH && !Lane::kW1Lds;
  constexpr bool kCand = kRegIn && DISC && NA <= 4;
  constexpr bool kHead2 = WIDE && DISC && NA == 2;
  // env rows [M[i] (NX) | K[i] (one column per action)], stride MKS (b128 rows)
  constexpr int NMK = NX + round4(NA);
  constexpr int MKS = NMK % 8 == 0 ? NMK + 4 : NMK;
  __shared__ float4 env4[(ENV == FDR_ENV_SYNTH) ? NIN * MKS / 4 : 1];
  __shared__ float4 wtile[kLanesPerBlock * Lane::kTileF4];
  __shared__ typename Lane::Scratch scratch[kLanesPerBlock];
  float* envMK = reinterpret_cast<float*>(env4);

  // wv through readfirstlane: the compiler then treats the lane index (and det) as wave-uniform (SGPRs,
  // scalar branches) instead of masking EXEC around the sampled / deterministic action paths
  const int j = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = blockIdx.x * kLanesPerBlock + wv;
  if constexpr (ENV == FDR_ENV_SYNTH) {
    for (int e = threadIdx.x; e < NIN * MKS; e += blockDim.x) {  // padding columns zero (b128 row reads)
      const int i = e / MKS, k = e % MKS;
      envMK[e] = (k < NIN ? a.M[i * NIN + k] : (k >= NX && k < NX + NA ? a.K[i * NA + k - NX] : 0.f));
    }
    __syncthreads();  // the only cross-wave hand-off: shared env matrices
  }
  if (lane >= a.n_lanes) return;

  ParamSrc src = a.lanes.src(lane);
  const bool det = a.lanes.deterministic ? a.lanes.deterministic[lane] != 0 : false;
  Lane pl;
  pl.load(src, j, a.bn_mean, a.bn_var, wtile + wv * Lane::kTileF4);
  {  // written now: a double live across the T-step loop would be spilled (and the asm keeps the compiler from
     // sinking the norm past the loop with every element's sigma * eps in scratch)
    double n2 = wave_sum(src.n2);
    asm volatile("" : "+v"(n2));
    if (j == 0 && a.norm2) a.norm2[lane] = n2;
  }

  const int ji = j < NIN ? j : NIN - 1;
  constexpr bool norm_obs = (FEAT & 4) != 0;
  const float om = norm_obs ? a.obs_mean[ji] : 0.f;
  const float osd = norm_obs ? a.obs_std[ji] : 1.f;
  auto policy_input = [&](float s) {
    float x = s;
    if (norm_obs) x = fminf(fmaxf((s - om) / osd, -10.f), 10.f);  // agent.py:40-41
    return pl.input_transform(x);
  };

  int col = 0, row = 0;  // trap env state (wave-uniform)
  float s = 0.f;         // synthetic env state element j (j < NIN)
  if constexpr (ENV == FDR_ENV_SYNTH) {
    s = a.s0[ji];
  } else {
    col = a.trap_start_col;
    row = a.trap_start_row;
    s = trap_obs(j, col, row);
  }
  const int T = a.T;
  const uint64_t key = a.key;
  const uint64_t ulane = (uint64_t)(a.lanes.lane_offset + lane);  // global lane id
  constexpr bool kTerm = (FEAT & 16) != 0;
  int nsteps = T;  // env.step calls of the episode (agent.py:47)
  double racc = 0.0;
  float eacc = 0.f;  // per-lane entropy sum (f32: T terms of O(1), rel. error ~1e-7 * sqrt(T))
  const int o = j & 15;
  // Random draws are made in batches: one counter hash per lane covers up to 64 future draws
  // (discrete: lane i holds the uniform of step t0 + i; continuous: lane i holds the normal of
  // step t0 + i / NA, dim i % NA).  Same (lane, t, k) counters as drawing them one at a time.
  constexpr int kDrawsPerStep = DISC ? 1 : NA;
  constexpr int kStepsPerBatch = 64 / kDrawsPerStep;
  float rbuf = 0.f;
  uint64_t os_mask = 0;  // obs-stat coins of the current 64-step batch (wave-uniform)
  int os_n = 0;
  float os_mean = 0.f, os_m2 = 0.f;

#ifdef FDR_PHASE_STAMPS
  uint64_t ph_acc[5] = {0, 0, 0, 0, 0};
  uint64_t ph_last = 0;
  auto mark = [&](int k, float dep) {
    uint64_t now;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(now) : "v"(dep));
    if (k >= 0) ph_acc[k] += now - ph_last;
    ph_last = now;
  };
#else
  auto mark = [](int, float) {};
#endif
  // Draw batch starting at step t (lane-parallel), and the normal of step t for action dim o.
  auto draw = [&](int t) {
    const int ds = j / kDrawsPerStep, dk = j % kDrawsPerStep;
    if constexpr ((FEAT & 8) != 0) {  // host-injected draws (u_inject), same batch layout
      const int tt = t + ds;
      rbuf = tt < T ? a.u_inject[((int64_t)lane * T + tt) * kDrawsPerStep + dk] : 0.f;
    } else {
      const uint64_t h = hash_ctr(key, ulane, (uint64_t)(t + ds), (uint64_t)dk);
      rbuf = DISC ? uniform24(h) : normal_bm(h);
    }
  };
  // WIDE: loop invariants in registers (M row ji, K row ji, the head's W3 slice)
  float mreg[kRegIn ? NX : 1], kreg[WIDE ? NA : 1], w3reg[WIDE ? 16 : 1];
  if constexpr (WIDE) {
    if constexpr (ENV == FDR_ENV_SYNTH) {
      const float* mr = envMK + ji * MKS;
#pragma unroll
      for (int k = 0; k < NA; ++k) kreg[k] = mr[NX + k];
      if constexpr (kRegIn) {
#pragma unroll
        for (int k = 0; k < NX; ++k) mreg[k] = mr[k];
      }
    }
    pl.head_weights(w3reg);
  }
  f2 w3c = {0.f, 0.f};  // head2: (W3[0][j], W3[1][j]) from lane (j >> 4, o) of the tile
  float b3p = 0.f;
  if constexpr (kHead2) {
    const float* t0 = reinterpret_cast<const float*>(pl.tile - j + (Lane::kW1Chunks + ((j & 15) >> 2)) * kWave +
                                                     (j >> 4) * 16);
    w3c = f2{t0[j & 3], t0[4 + (j & 3)]};
    if (WIDE && (j & 1)) w3c = f2{w3c.y, w3c.x};  // output j & 1 first (head2<true>)
    const float b30 = readlane_f(pl.b3, 0), b31 = readlane_f(pl.b3, 1);
    b3p = (j & 1) ? b31 : b30;
  }
  const int zbase = 4 * (o < NA ? o : 0);  // ds_bpermute byte address of dim o in step 0 of a batch
  auto fetch_z = [&](int t) {
    if constexpr (DISC) return 0.f;
    const int addr = zbase + 4 * NA * (t % kStepsPerBatch);
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(addr, __builtin_bit_cast(int, rbuf)));
  };
  // The deterministic / sampled choice is fixed for the episode (wave-uniform): one specialised loop each, and the
  // draw batches as an outer loop, so the per-step body carries neither branch.
  auto episode = [&](auto det_tag) {
    constexpr bool kDet = decltype(det_tag)::value;
    for (int t0 = 0; t0 < T; t0 += kStepsPerBatch) {
      if constexpr (!kDet) draw(t0);
      const int nb = T - t0 < kStepsPerBatch ? T - t0 : kStepsPerBatch;
      for (int tb = 0; tb < nb; ++tb) {
        const int t = t0 + tb;
        // The W1 / M / K rows are loop-invariant LDS data; hoisting their loads out of the loop would
        // pin ~46 more VGPRs (and spill W2).  Keep them per-step reads.
        asm volatile("" ::: "memory");
        mark(-1, s);
        const float zt = fetch_z(t);  // this step's normal for action dim o (continuous)
        if constexpr (FEAT & 1) {  // visited (raw) observations, worker/agent.py:36 / 58-59 (save_states)
          if (j < NIN) a.states[((int64_t)lane * T + t) * NIN + j] = s;
        }
        if constexpr (FEAT & 2) {
          // worker/agent.py:37-39: with probability obs_stats_update_chance the raw obs enters the lane's
          // WelfordRunningStat (utils/math_helpers.py:29-38, f32, same operation order, no contraction).
          // Coins come 64 steps at a time: lane i draws step t + i (counter k = 14), one ballot.
          if ((t & 63) == 0) {
            const float u = uniform24(hash_ctr(key, ulane, (uint64_t)(t + j), 14));
            os_mask = __ballot(u < a.os_chance);
          }
          if ((os_mask >> (t & 63)) & 1ull) {
    #pragma clang fp contract(off)
            const int cc = os_n;
            os_n += 1;
            const float delta = s - os_mean;
            const float delta_n = delta / (float)os_n;
            os_mean += delta_n;
            os_m2 += (delta * delta_n) * (float)cc;
          }
        }
        auto* sc = &scratch[wv];
        constexpr bool kSame = !DISC && !norm_obs;  // mujoco: policy input == env state
        const float* mrow = envMK + ji * MKS;
        float pre = 0.f;
        float h1;
        float cand[kCand ? NA : 1];  // discrete WIDE: next state for each action
        if constexpr (kRegIn) {
          // policy input and env state of lanes 0 .. NIN-1, wave-uniform through v_readlane
          const float xin = j < NIN ? policy_input(s) : 0.f;
          float xv[NX], sv[NX];
    #pragma unroll
          for (int k = 0; k < NX; ++k) {
            xv[k] = k < NIN ? readlane_f(xin, k) : (k == NIN ? 1.f : 0.f);
            sv[k] = k < NIN ? (kSame ? xv[k] : readlane_f(s, k)) : 0.f;
          }
          h1 = pl.layer1_env_reg(xv, sv, mreg, pre);
          if constexpr (kCand) {
    #pragma unroll
            for (int i = 0; i < NA; ++i) cand[i] = tanh_fast(pre + kreg[i]);
          }
        } else {
        // policy input (and env state) broadcast through the wave's LDS scratch, then packed FMAs
        // against the lane's W1 row and M row (two MACs per instruction instead of one DPP FMA)
        sc->x[j] = j < NIN ? policy_input(s) : (j == NIN ? 1.f : 0.f);
        if constexpr (ENV == FDR_ENV_SYNTH && !kSame) sc->h1[j] = j < NIN ? s : 0.f;
        wave_lds_sync();
        if constexpr (ENV == FDR_ENV_SYNTH) {
          // one pass over the input chunks: W1 row j against x, M row j against s (M's padding
          // columns are 0, so the bias column's 1 drops out of M s)
          h1 = pl.template layer1_env_pk<kSame>(sc->x, sc->h1, mrow, pre);
        } else {
          float xb[NX];
          lds_bcast<NX>(sc->x, xb);
          h1 = pl.layer1(xb);
        }
        }
        mark(0, h1);
        float y;
        if constexpr (kHead2) {
          const float h2 = pl.template layer2<WIDE>(h1, sc, j);
          mark(1, h2);
          y = pl.template head2<WIDE>(h2, w3c, b3p, j);
          mark(2, y);
        } else {
          y = pl.layers23(h1, sc, j, mark, WIDE ? w3reg : nullptr);
        }
        int act_d = 0;
        float act_c = 0.f;
        if constexpr (DISC) {
          float p;
          p = pl.template softmax<kHead2, !kDet>(y, j);
          if constexpr (kHead2 && !kDet) {
            // two outputs, sampled: everything in VALU, no readlane round trip -- lane parity o holds p_o;
            // tot = p0 + p1 (the oracle's 0 + p0 + p1, exactly), p0 to every lane by one DPP move, and the
            // inverse CDF of two outputs is (p0 <= u tot); no contraction of p's product into the sum
    #pragma clang fp contract(off)
            const float tot = p + dpp_mov<kDppQuadXor1>(p);
            const float p0 = dpp_mov<0xA0>(p);  // quad_perm [0,0,2,2]
            act_d = p0 <= readlane_f(rbuf, tb) * tot ? 1 : 0;
            eacc -= (j < NA) ? disc_entropy_term(p, tot) : 0.f;
          } else {
          float pv[NA];
    #pragma unroll
          for (int i = 0; i < NA; ++i) pv[i] = readlane_f(p, i);
          float tot = pv[0];  // sequential f32 cumsum, the oracle's order (0 + p0 == p0)
    #pragma unroll
          for (int i = 1; i < NA; ++i) tot += pv[i];
          // Branch-free selection (selects, no data-dependent control flow):
          //   argmax = first maximal index; inverse CDF = first i with cumsum_i > target, i.e. the
          //   number of (monotone) partial sums <= target, capped at NA - 1.
          if constexpr (kDet) {
            float best = pv[0];
    #pragma unroll
            for (int i = 1; i < NA; ++i) {
              act_d = pv[i] > best ? i : act_d;
              best = fmaxf(best, pv[i]);
            }
          } else {
            const float target = readlane_f(rbuf, tb) * tot;
            float c = 0.f;
    #pragma unroll
            for (int i = 0; i < NA - 1; ++i) {
              c += pv[i];
              act_d += c <= target ? 1 : 0;
            }
          }
          // Categorical(probs) entropy: probs normalised, log clamped (torch semantics)
          eacc -= (j < NA) ? disc_entropy_term(p, tot) : 0.f;
          }
        } else {
          const float th = tanh_fast(y);
          const float sd = std_from_tanh(dpp_mov<kDppRowShl + NA>(th));
          eacc += __builtin_amdgcn_logf(sd);  // log2; lanes >= NA and the ln 2 scale: epilogue
          act_c = kDet ? th : gauss_action(th, sd, zt);
        }

        mark(3, DISC ? (float)act_d : act_c);
        // ---- env step ----
        if constexpr (ENV == FDR_ENV_SYNTH) {
          if constexpr (kCand) {
            s = cand[0];
    #pragma unroll
            for (int i = 1; i < NA; ++i) s = act_d == i ? cand[i] : s;
          } else {
            if constexpr (DISC) {
              pre += mrow[NX + act_d];
            } else {
              float kr[NA];
    #pragma unroll
              for (int m = 0; m < NA; ++m) kr[m] = WIDE ? kreg[m] : mrow[NX + m];
              dpp_tail<NA>(pre, act_c, kr);  // a[m] sits in lane m of every row
            }
            s = tanh_fast(pre);
          }
          racc += (double)s;  // lane 0 holds the reward s'[0]; other lanes' sums are discarded
          if constexpr (kTerm) {  // done after this step: the reward and entropy of step t count (agent.py:46-52)
            if (fabsf(readlane_f(s, a.done_dim)) > a.done_thr) {
              nsteps = t + 1;
              return;
            }
          }
        } else {
          // custom_envs/simple_trap_env: node.py:9-14, tile_map.py:11-23, environment.py:33-48
          const int prev_x = col * 7;
          const int tc = col + act_d / 3 - 1, tr = row + act_d % 3 - 1;
          if (tc >= 0 && tc < a.map_w && tr >= 0 && tr < a.map_h && a.walkable[tr * a.map_w + tc]) {
            col = tc;
            row = tr;
          }
          racc += (double)(col * 7 - prev_x);
          s = trap_obs(j, col, row);
        }
        mark(4, s);
      }
    }
  };
  if (det)
    episode(std::true_type{});
  else
    episode(std::false_type{});
#ifdef FDR_PHASE_STAMPS
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int k = 0; k < 5; ++k) g_phase_stamps[k] = ph_acc[k];
#endif

  // ---- epilogue ----
  eacc *= 0.693147180559945309f;  // log2 -> ln (both kinds)
  const double esum = wave_sum((j < NA) ? (double)eacc : 0.0);
  if (j == 0) {
    double r = racc;
    if (a.jiggle) r += (hash_ctr(key, ulane, kJiggleT, 15) & 1ull) ? 1e-12 : -1e-12;
    a.ret[lane] = r;
    double e = esum / (double)nsteps;  // mean over the visited states (agent.py:60-65)
    if constexpr (!DISC) e += (double)NA * 1.4189385332046727;  // 0.5 + 0.5*ln(2*pi) per dim
    a.ent[lane] = e;
    a.steps[lane] = nsteps;
  }
  if constexpr (FEAT & 2) {
    if (j < NIN) {
      a.os_mean[(int64_t)lane * NIN + j] = os_mean;
      a.os_m2[(int64_t)lane * NIN + j] = os_m2;
    }
    if (j == 0) a.os_count[lane] = os_n;
  }
}

// ---------------------------------------------------------------------------------------------
// Two lanes per wave: rollout_pair_kernel (synthetic env)
//
// The wave's halves (threads 0-31 / 32-63, two DPP rows each) run one lane each; thread t of a
// half owns hidden units 2t, 2t+1 of layer 1 and units 16r + c, 16r + 8 + c (r = t/8, c = t%8) of
// layer 2.  Per lane the MAC instructions are those of the one-lane-per-wave kernel, but the
// per-lane scalar work (action, sampling, env tail, reward, loop control) is shared by the two
// lanes of a wave, and each wave carries two independent dependency chains:
//   L1 + M s   broadcast input of the half (LDS); W1 rows 2t, 2t+1 (per-wave tile) and M row t.
//   L2         thread (r, c) holds W2[16r + 8e + (c ^ sigma(p))][8c + k] (p < 8, e < 2, k < 8:
//              128 VGPRs) against h1[8c .. 8c + 7] (two b128), 16 partial outputs, then the
//              3-level reduce-scatter of the one-lane kernel over 16 slots (8 + 4 + 2 DPP adds).
//   head       thread (rho = t/16, o = t%16) sums W3[o][.] over the 32 units its own DPP row
//              holds (32 row_newbcast FMAs), then the two rows of the half (one permlane16 swap).
// ---------------------------------------------------------------------------------------------
constexpr int kPairWaves = 2;  // waves per workgroup (4 lanes): 4 workgroups, 8 waves per CU

// tanh_fast on a register pair: packed mul / add / fma around the two exp and two rcp
__device__ __forceinline__ f2 tanh2_pre(f2 t) {  // t = 2 log2(e) x
  const f2 d = f2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + f2{1.f, 1.f};
  return pk_fma(f2{-2.f, -2.f}, f2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)}, f2{1.f, 1.f});
}
__device__ __forceinline__ f2 tanh2_fast(f2 x) {
  return tanh2_pre(x * f2{kTanhScale, kTanhScale});
}
// Every weight and bias feeding a tanh is stored times kTanhScale (after its norm2 count), so the activation
// starts at the exp2 -- one multiply fewer per tanh (L1, L2, head, env: 4 per step)
constexpr float kPreScale = kTanhScale;
template <bool kPre>
__device__ __forceinline__ f2 tanh2_act(f2 z) {
  if constexpr (kPre) return tanh2_pre(z);
  else return tanh2_fast(z);
}

template <int NIN, int NA, bool DISC>
struct MlpPair {
  using L = Layout<NIN, NA, DISC>;
  static constexpr int NOUT = L::NOUT;
  static constexpr int NX = round4(NIN);
  static_assert(NX <= 32, "pair kernel: policy input wider than 32");
  static constexpr bool kBiasCol = NIN < NX;
  static constexpr bool kW1Lds = NIN > 8;
  static constexpr bool kPre = !DISC;  // tanh layers' weights stored x kTanhScale
  static constexpr float kWS = kPre ? kTanhScale : 1.f;
  static constexpr int kW1Chunks = kW1Lds ? NX / 4 : 0;     // per W1 row
  static constexpr int kTileF4 = (2 * kW1Chunks + 8) * kWave;  // float4 per wave: W1 rows, W3 slice
  f2 w1a[kW1Lds ? 1 : NX / 2], w1b[kW1Lds ? 1 : NX / 2];
  float b1a, b1b;
  const float4* tile;  // this thread's column of the wave tile (chunk m at tile[m * kWave])
  f2 w2[64];           // w2[p * 8 + k] = (W2[16r + (c ^ sigma(p))][8c + k], W2[16r + 8 + (c ^ sigma(p))][8c + k])
  float b2a, b2b, b3;
  float a0, c0, a1a, c1a, a1b, c1b, a2a, c2a, a2b, c2b;  // discrete: folded BN

  // unit of layer 2 that row-thread k's value e (0: z.x, 1: z.y) holds, within the row's 32 units
  __host__ __device__ static constexpr int head_unit(int rho, int k, int e) {
    return 32 * rho + 8 * (k >> 2) + 4 * e + (k & 3);  // thread 4q + c holds units 8q + c, 8q + 4 + c
  }

  __device__ __forceinline__ void load(ParamSrc& src, int t, int tid, const float* bn_mean, const float* bn_var,
                                       float4* wave_tile) {
    const int rho = t >> 4, o = t & 15;
    const int ua = 2 * t, ub = 2 * t + 1;
    float4* my = wave_tile + tid;
    tile = my;
    auto w1v = [&](int u, int k) {
      return kWS * (k < NIN ? src.get(L::L1W + (int64_t)u * NIN + k) : (k == NIN ? src.get(L::L1B + u) : 0.f));
    };
    if constexpr (kPk) {
#pragma unroll
      for (int j = 0; j < 2 * kW1Chunks; ++j) {
        const float e0 = w1v(ua, 2 * j), f0 = w1v(ub, 2 * j), e1 = w1v(ua, 2 * j + 1), f1 = w1v(ub, 2 * j + 1);
        my[j * kWave] = float4{e0, f0, e1, f1};
      }
    } else if constexpr (kW1Lds) {
#pragma unroll
      for (int m = 0; m < kW1Chunks; ++m) {
        const float e0 = w1v(ua, 4 * m), e1 = w1v(ua, 4 * m + 1), e2 = w1v(ua, 4 * m + 2), e3 = w1v(ua, 4 * m + 3);
        my[m * kWave] = float4{e0, e1, e2, e3};
        const float f0 = w1v(ub, 4 * m), f1 = w1v(ub, 4 * m + 1), f2_ = w1v(ub, 4 * m + 2), f3 = w1v(ub, 4 * m + 3);
        my[(kW1Chunks + m) * kWave] = float4{f0, f1, f2_, f3};
      }
    } else {
#pragma unroll
      for (int p = 0; p < NX / 2; ++p) {
        const float e0 = w1v(ua, 2 * p), e1 = w1v(ua, 2 * p + 1);
        w1a[p] = f2{e0, e1};
        const float f0 = w1v(ub, 2 * p), f1 = w1v(ub, 2 * p + 1);
        w1b[p] = f2{f0, f1};
      }
    }
    b1a = kBiasCol ? 0.f : kWS * src.get(L::L1B + ua);
    b1b = kBiasCol ? 0.f : kWS * src.get(L::L1B + ub);
    // (load groups: each group's loads are issued together, the next group's after it -- hoisting every load of the
    // prologue to its top spilled ~140 values to scratch)
    __builtin_amdgcn_sched_barrier(0);
    // quad q = t / 4 owns units 8q .. 8q + 7; thread c = t % 4 of it takes inputs 16c .. 16c + 15 and pair p the
    // units (8q + (c ^ p), 8q + 4 + (c ^ p)): the quad's reduce-scatter (partners c ^ 2, c ^ 1) leaves pair 0
    const int q4 = t >> 2, c4 = t & 3;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row0 = 8 * q4 + (c4 ^ p), row1 = row0 + 4;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float e0 = src.get(L::L2W + (int64_t)row0 * kHidden + 16 * c4 + k);
        const float e1 = src.get(L::L2W + (int64_t)row1 * kHidden + 16 * c4 + k);
        w2[p * 16 + k] = f2{kWS * e0, kWS * e1};
      }
      // the group's weights and its norm terms are final here (else the compiler defers the selects past the other
      // groups' loads and keeps every sigma * eps in scratch meanwhile)
#pragma unroll
      for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(w2[p * 16 + k]));
      asm volatile("" : "+v"(src.n2));
      __builtin_amdgcn_sched_barrier(0);
    }
    const int u2a = 8 * q4 + c4, u2b = 8 * q4 + 4 + c4;  // this thread's layer-2 units
    b2a = kWS * src.get(L::L2B + u2a);
    b2b = kWS * src.get(L::L2B + u2b);
    // branch-free (MlpLane::load): clamped indices, counted and kept only where the element exists
    {
      const bool has_o = o < NOUT;
      const int oc = has_o ? o : 0;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        float e[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int w = 4 * m + i;
          // w < 16: value z.x of row-thread w; else z.y of row-thread w - 16
          e[i] = src.get_if(L::L3W + (int64_t)oc * kHidden + head_unit(rho, w & 15, w >> 4), has_o);
        }
        my[(2 * kW1Chunks + m) * kWave] =
            has_o ? float4{kWS * e[0], kWS * e[1], kWS * e[2], kWS * e[3]} : float4{0.f, 0.f, 0.f, 0.f};
      }
      const float b3v = src.get_if(L::L3B + oc, has_o && rho == 0);
      b3 = has_o ? kWS * b3v : 0.f;
    }
    wave_lds_sync();
    a0 = c0 = a1a = c1a = a1b = c1b = a2a = c2a = a2b = c2b = 0.f;
    if constexpr (DISC) {
      const float* bm = bn_mean ? bn_mean : src.base;  // a readable address either way
      const float* bv = bn_var ? bn_var : src.base;
      auto stat = [&](int k, float& rm, float& rv) {
        const float m = bm[k], v = bv[k];
        rm = bn_mean ? m : 0.f;
        rv = bn_var ? v : 1.f;
      };
      {
        const bool in = t < NIN;
        const int tc = in ? t : 0;
        const float w = src.get_if(L::BN0W + tc, in), b = src.get_if(L::BN0B + tc, in);
        float rm, rv, a, c;
        stat(tc, rm, rv);
        bn_fold(w, b, rm, rv, a, c);
        a0 = in ? a : 0.f;
        c0 = in ? c : 0.f;
      }
      auto fold = [&](int64_t wofs, int64_t bofs, int st, int u, float& av, float& cv) {
        const float w = src.get(wofs + u), b = src.get(bofs + u);
        float rm, rv;
        stat(st + u, rm, rv);
        bn_fold(w, b, rm, rv, av, cv);
      };
      fold(L::BN1W, L::BN1B, NIN, ua, a1a, c1a);
      fold(L::BN1W, L::BN1B, NIN, ub, a1b, c1b);
      fold(L::BN2W, L::BN2B, NIN + kHidden, u2a, a2a, c2a);
      fold(L::BN2W, L::BN2B, NIN + kHidden, u2b, a2b, c2b);
    }
  }

  __device__ __forceinline__ float input_transform(float x) const {
    if constexpr (DISC) {
      return fmaf(x, a0, c0);
    } else {
      return x;
    }
  }

  __device__ __forceinline__ float act1(float z, float av, float cv) const {
    if constexpr (DISC) {
      return fmaf(fmaxf(z, 0.f), av, cv);
    } else {
      return tanh_act<kPre>(z);
    }
  }

  // Loop-invariant LDS rows of layer 1 (W1 rows 2t, 2t+1 when kW1Lds) and the env's M row t, loaded
  // a phase ahead of their use (after the head of the previous step), off the step's dependency chain.
  // NIN = 4k + 1 with the folded bias (HalfCheetah's 17): the last input chunk is [x_{NIN-1}, 1, 0, 0] and the
  // W1 / M chunks [w, b, 0, 0] / [m, 0, 0, 0] -- taken as one scalar input (a ds_read_b32 of x, a float2 of
  // W1, a float of M) and 3 FMAs instead of a fifth b128 chunk and 6 packed FMAs
  static constexpr bool kTail = kW1Lds && kBiasCol && NX - NIN == 3;
  static constexpr int NQ = kTail ? NX / 4 - 1 : NX / 4;  // full input chunks
  // W1 rows 2t, 2t+1 interleaved in the tile, [w_a(2j), w_b(2j), w_a(2j+1), w_b(2j+1)] per
  // float4, so each input k is ONE packed FMA over the two units into an (a, b) accumulator -- the layer's
  // output pair needs no horizontal adds / register shuffles before the packed tanh, and the folded bias
  // column is an add, not a multiply by 1
  static constexpr bool kPk = kW1Lds && kBiasCol;
  static constexpr int kPkPairs = (NIN + 2) / 2;  // float4 pairs of inputs 0 .. NIN (the bias column)
  struct L1Rows {
    float4 wa[kW1Lds && !kPk ? NQ : 1], wb[kW1Lds && !kPk ? NQ : 1], m[NQ];
    float2 ta, tb;  // kTail: (w, b) of the last chunk
    float tm;
    float4 wp[kPk ? kPkPairs : 1];
  };
  __device__ __forceinline__ void l1_prefetch(L1Rows& r, const float* mrow) const {
    const float4* m4 = reinterpret_cast<const float4*>(mrow);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if constexpr (kW1Lds && !kPk) {
        r.wa[q] = tile[q * kWave];
        r.wb[q] = tile[(kW1Chunks + q) * kWave];
      }
      r.m[q] = m4[q];
    }
    if constexpr (kPk) {
#pragma unroll
      for (int j = 0; j < kPkPairs; ++j) r.wp[j] = tile[j * kWave];
      if constexpr (kTail) r.tm = mrow[4 * NQ];
    } else if constexpr (kTail) {
      r.ta = *reinterpret_cast<const float2*>(&tile[NQ * kWave]);
      r.tb = *reinterpret_cast<const float2*>(&tile[(kW1Chunks + NQ) * kWave]);
      r.tm = mrow[4 * NQ];
    }
  }

  // Layer 1 (units 2t, 2t+1) and the env's M[t] . s in one pass over the broadcast input chunks.
  template <bool kSameInput>
  __device__ __forceinline__ f2 layer1_env(const float* xs, const float* ss, const L1Rows& rows, float& env) const {
    const float4* x4 = reinterpret_cast<const float4*>(xs);
    const float4* s4 = reinterpret_cast<const float4*>(ss);
    return layer1_env_q<kSameInput>([&](int q) { return x4[q]; }, [&](int q) { return s4[q]; }, rows, env,
                                    kTail ? xs[4 * NQ] : 0.f, kTail ? ss[4 * NQ] : 0.f);
  }
  template <bool kSameInput, class XQ, class SQ>
  __device__ __forceinline__ f2 layer1_env_q(XQ&& xq, SQ&& sq, const L1Rows& rows, float& env, float xt,
                                             float st) const {
    f2 aa0 = {b1a, 0.f}, aa1 = {0.f, 0.f}, ab0 = {b1b, 0.f}, ab1 = {0.f, 0.f};
    f2 am0 = {0.f, 0.f}, am1 = {0.f, 0.f};
    if constexpr (kPk) {
      // units (a, b) packed: acc[k % NC] += (w_a(k), w_b(k)) * x_k; the bias column (k = NIN) is added.
      // NC = 2 chains of ~9 dependent packed FMAs
      constexpr int NC = 2;
      f2 acc[NC];
#pragma unroll
      for (int q = 0; q < NC; ++q) acc[q] = f2{0.f, 0.f};
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const float4 xv = xq(q), mv = rows.m[q];
        const float4 sv = kSameInput ? xv : sq(q);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 4 * q + i;
          if (k < NIN) {
            const float4 w = rows.wp[k >> 1];
            const f2 xp = (i < 2) ? f2{xv.x, xv.y} : f2{xv.z, xv.w};
            if (kPre && k == NIN % NC) {  // the chain that takes the bias column starts from it
              const float4 wb = rows.wp[NIN >> 1];
              const f2 bias = (NIN & 1) ? f2{wb.z, wb.w} : f2{wb.x, wb.y};
              acc[k % NC] = (k & 1) ? pk_fma_bhi(f2{w.z, w.w}, xp, bias) : pk_fma_blo(f2{w.x, w.y}, xp, bias);
            } else if (k < NC)
              acc[k % NC] = (k & 1) ? pk_mul_bhi(f2{w.z, w.w}, xp) : pk_mul_blo(f2{w.x, w.y}, xp);
            else
              acc[k % NC] = (k & 1) ? pk_fma_bhi(f2{w.z, w.w}, xp, acc[k % NC]) : pk_fma_blo(f2{w.x, w.y}, xp, acc[k % NC]);
          }
        }
        am0 = pk_fma(f2{mv.x, mv.y}, f2{sv.x, sv.y}, am0);
        am1 = pk_fma(f2{mv.z, mv.w}, f2{sv.z, sv.w}, am1);
      }
      if constexpr (kTail) {  // input 4 NQ = NIN - 1, then the bias
        const float4 w = rows.wp[(NIN - 1) >> 1];
        acc[(NIN - 1) % NC] = pk_fma(((NIN - 1) & 1) ? f2{w.z, w.w} : f2{w.x, w.y}, f2{xt, xt}, acc[(NIN - 1) % NC]);
        am1.x = fmaf(rows.tm, kSameInput ? xt : st, am1.x);
      }
      if constexpr (!kPre || NIN % NC >= NIN) {
        const float4 w = rows.wp[NIN >> 1];
        acc[NIN % NC] = acc[NIN % NC] + ((NIN & 1) ? f2{w.z, w.w} : f2{w.x, w.y});
      }
      const f2 h = acc[0] + acc[1];
      const f2 am = am0 + am1;
      env = am.x + am.y;
      if constexpr (DISC) {
        return f2{act1(h.x, a1a, c1a), act1(h.y, a1b, c1b)};
      } else {
        return tanh2_act<kPre>(h);
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const float4 xv = xq(q), mv = rows.m[q];
      const float4 sv = kSameInput ? xv : sq(q);
      float4 wa, wb;
      if constexpr (kW1Lds) {
        wa = rows.wa[q];
        wb = rows.wb[q];
      } else {
        wa = float4{w1a[2 * q].x, w1a[2 * q].y, w1a[2 * q + 1].x, w1a[2 * q + 1].y};
        wb = float4{w1b[2 * q].x, w1b[2 * q].y, w1b[2 * q + 1].x, w1b[2 * q + 1].y};
      }
      aa0 = pk_fma(f2{wa.x, wa.y}, f2{xv.x, xv.y}, aa0);
      ab0 = pk_fma(f2{wb.x, wb.y}, f2{xv.x, xv.y}, ab0);
      am0 = pk_fma(f2{mv.x, mv.y}, f2{sv.x, sv.y}, am0);
      aa1 = pk_fma(f2{wa.z, wa.w}, f2{xv.z, xv.w}, aa1);
      ab1 = pk_fma(f2{wb.z, wb.w}, f2{xv.z, xv.w}, ab1);
      am1 = pk_fma(f2{mv.z, mv.w}, f2{sv.z, sv.w}, am1);
    }
    if constexpr (kTail) {  // w x + b of the last chunk, and m s
      aa1 = pk_fma(f2{rows.ta.x, rows.ta.y}, f2{xt, 1.f}, aa1);
      ab1 = pk_fma(f2{rows.tb.x, rows.tb.y}, f2{xt, 1.f}, ab1);
      am1.x = fmaf(rows.tm, kSameInput ? xt : st, am1.x);
    }
    const f2 am = am0 + am1, ha = aa0 + aa1, hb = ab0 + ab1;
    env = am.x + am.y;
    if constexpr (DISC) {
      return f2{act1(ha.x + ha.y, a1a, c1a), act1(hb.x + hb.y, a1b, c1b)};
    } else {
      return tanh2_act<kPre>(f2{ha.x + ha.y, hb.x + hb.y});
    }
  }

  // Layer 2 and the head: h1 = this thread's layer-1 units (2t, 2t+1); h1s = the half's scratch.
  // Returns the head pre-activation for output o = t & 15 (identical in both rows of the half).
  template <class Mark>
  __device__ __forceinline__ float layers23(f2 h1, float* h1s, int t, Mark&& mark) const {
    const int c4 = t & 3;
    float x[16];
    reinterpret_cast<f2*>(h1s)[t] = h1;
    wave_lds_sync();
    lds_bcast<16>(h1s + 16 * c4, x);
    float w3[32];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const float4 w = tile[(2 * kW1Chunks + m) * kWave];
      w3[4 * m] = w.x;
      w3[4 * m + 1] = w.y;
      w3[4 * m + 2] = w.z;
      w3[4 * m + 3] = w.w;
    }
    f2 acc[4];
#pragma unroll
    for (int p = 0; p < 4; ++p)  // k = 0; kPre: the own pair (p = 0) starts from the biases
      acc[p] = pk_fma(w2[p * 16], f2{x[0], x[0]}, (kPre && p == 0) ? f2{b2a, b2b} : f2{0.f, 0.f});
    {
      // k = 1 .. 15 by op_sel broadcasts of the pairs xp[j] = (x[2j], x[2j + 1]) in one asm statement (operands:
      // %0-%3 acc, %(4 + 4 (k - 1) + p) = w2[16 p + k], %64-%71 the pairs); k = 15 writes acc[3], acc[2] first,
      // the reduce-scatter's first DPP sources
      f2 xp[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) xp[j] = f2{x[2 * j], x[2 * j + 1]};
#define FDR_L2_HI "op_sel:[0,1,0] op_sel_hi:[1,1,1]"
#define FDR_L2_LO "op_sel_hi:[1,0,1]"
      asm(
          "v_pk_fma_f32 %0, %4, %64, %0 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %1, %5, %64, %1 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %2, %6, %64, %2 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %3, %7, %64, %3 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %0, %8, %65, %0 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %1, %9, %65, %1 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %2, %10, %65, %2 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %3, %11, %65, %3 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %0, %12, %65, %0 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %1, %13, %65, %1 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %2, %14, %65, %2 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %3, %15, %65, %3 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %0, %16, %66, %0 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %1, %17, %66, %1 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %2, %18, %66, %2 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %3, %19, %66, %3 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %0, %20, %66, %0 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %1, %21, %66, %1 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %2, %22, %66, %2 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %3, %23, %66, %3 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %0, %24, %67, %0 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %1, %25, %67, %1 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %2, %26, %67, %2 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %3, %27, %67, %3 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %0, %28, %67, %0 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %1, %29, %67, %1 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %2, %30, %67, %2 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %3, %31, %67, %3 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %0, %32, %68, %0 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %1, %33, %68, %1 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %2, %34, %68, %2 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %3, %35, %68, %3 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %0, %36, %68, %0 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %1, %37, %68, %1 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %2, %38, %68, %2 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %3, %39, %68, %3 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %0, %40, %69, %0 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %1, %41, %69, %1 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %2, %42, %69, %2 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %3, %43, %69, %3 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %0, %44, %69, %0 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %1, %45, %69, %1 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %2, %46, %69, %2 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %3, %47, %69, %3 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %0, %48, %70, %0 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %1, %49, %70, %1 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %2, %50, %70, %2 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %3, %51, %70, %3 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %0, %52, %70, %0 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %1, %53, %70, %1 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %2, %54, %70, %2 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %3, %55, %70, %3 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %0, %56, %71, %0 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %1, %57, %71, %1 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %2, %58, %71, %2 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %3, %59, %71, %3 " FDR_L2_LO "\n"
          "v_pk_fma_f32 %3, %63, %71, %3 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %2, %62, %71, %2 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %0, %60, %71, %0 " FDR_L2_HI "\n"
          "v_pk_fma_f32 %1, %61, %71, %1 " FDR_L2_HI "\n"
          : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])
          : "v"(w2[1]), "v"(w2[17]), "v"(w2[33]), "v"(w2[49]),
            "v"(w2[2]), "v"(w2[18]), "v"(w2[34]), "v"(w2[50]),
            "v"(w2[3]), "v"(w2[19]), "v"(w2[35]), "v"(w2[51]),
            "v"(w2[4]), "v"(w2[20]), "v"(w2[36]), "v"(w2[52]),
            "v"(w2[5]), "v"(w2[21]), "v"(w2[37]), "v"(w2[53]),
            "v"(w2[6]), "v"(w2[22]), "v"(w2[38]), "v"(w2[54]),
            "v"(w2[7]), "v"(w2[23]), "v"(w2[39]), "v"(w2[55]),
            "v"(w2[8]), "v"(w2[24]), "v"(w2[40]), "v"(w2[56]),
            "v"(w2[9]), "v"(w2[25]), "v"(w2[41]), "v"(w2[57]),
            "v"(w2[10]), "v"(w2[26]), "v"(w2[42]), "v"(w2[58]),
            "v"(w2[11]), "v"(w2[27]), "v"(w2[43]), "v"(w2[59]),
            "v"(w2[12]), "v"(w2[28]), "v"(w2[44]), "v"(w2[60]),
            "v"(w2[13]), "v"(w2[29]), "v"(w2[45]), "v"(w2[61]),
            "v"(w2[14]), "v"(w2[30]), "v"(w2[46]), "v"(w2[62]),
            "v"(w2[15]), "v"(w2[31]), "v"(w2[47]), "v"(w2[63]),
            "v"(xp[0]), "v"(xp[1]), "v"(xp[2]), "v"(xp[3]), "v"(xp[4]), "v"(xp[5]), "v"(xp[6]), "v"(xp[7]));
#undef FDR_L2_LO
#undef FDR_L2_HI
    }
    // reduce-scatter over the quad: slot i = acc[i / 2][i % 2]; level 1 o_i = v_i + partner(c ^ 2).v_{i + 4} in
    // the order o2, o3, o0, o1, level 2 o_i += partner(c ^ 1).o_{i + 2} -- every DPP source >= 3 instructions old
    f2 zs;
    {
      float o0, o1, o2, o3;
      asm volatile(
          "v_add_f32_dpp %2, %10, %6 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_add_f32_dpp %3, %11, %7 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_add_f32_dpp %0, %8, %4 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_add_f32_dpp %1, %9, %5 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_add_f32_dpp %0, %2, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_add_f32_dpp %1, %3, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          : "=&v"(o0), "=&v"(o1), "=&v"(o2), "=&v"(o3)
          : "v"(acc[0].x), "v"(acc[0].y), "v"(acc[1].x), "v"(acc[1].y), "v"(acc[2].x), "v"(acc[2].y), "v"(acc[3].x),
            "v"(acc[3].y));
      zs = f2{o0, o1};
    }
    const float za = kPre ? zs.x : zs.x + b2a;  // unit 8q + c
    const float zb = kPre ? zs.y : zs.y + b2b;  // unit 8q + 4 + c
    mark(1, za);
    float h2a, h2b;
    if constexpr (DISC) {
      h2a = fmaf(fmaxf(za, 0.f), a2a, c2a);
      h2b = fmaf(fmaxf(zb, 0.f), a2b, c2b);
    } else {
      const f2 h2 = tanh2_act<kPre>(f2{za, zb});
      h2a = h2.x;
      h2b = h2.y;
    }
    float u;
    dpp_dot_32x1(u, h2a, h2b, w3);  // one chain of 32 (the accumulator is no DPP source: no wait states)
    float v = u;
    permlane16_swap(u, v);  // u = row 2h's partial, v = row 2h+1's, in both rows of half h
    const float out = (u + v) + b3;
    mark(2, out);
    return out;
  }

  template <bool kAll = false, bool kFast = false>  // as MlpLane::softmax
  __device__ __forceinline__ float softmax(float logit, int t) const {
    const bool valid = (t & 15) < NOUT;
    const float v = valid ? logit : -FLT_MAX;
    const float mx = row16_max_n<NOUT>(v);
    if constexpr (kFast) {
      const float e = valid ? __builtin_amdgcn_exp2f((v - mx) * 1.44269504088896341f) : 0.f;
      return e * __builtin_amdgcn_rcpf(row16_sum_n<NOUT>(e));
    } else {
      const float e = valid ? expf(v - mx) : 0.f;
      return e / row16_sum_n<NOUT>(e);
    }
  }
};

struct alignas(16) PairScratch {
  float h1[2][kHidden];  // per half: layer-1 output; the env state when it differs from the input
  float x[2][32];        // per half: policy input (+ the 1 of the folded bias column)
};

template <int K>
__device__ __forceinline__ float row_bcast(float v) {  // lane K of the caller's 16-lane row
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x150 + K, 0xF, 0xF, false));
}

template <int N, int... I>
__device__ __forceinline__ void row_bcast_all(float v, float (&out)[N], std::integer_sequence<int, I...>) {
  ((out[I] = row_bcast<I>(v)), ...);
}

// FEAT bit 0: record visited observations; bit 2: observation normalisation (bit 1, the Welford
// statistics, runs on rollout_kernel); bit 4: terminating synthetic env -- each half keeps a done flag (wave-uniform
// scalars alive0 / alive1): a finished half's steps still execute in lockstep with its partner but add nothing to
// its reward, entropy or step count, and the wave leaves the loop when both halves are done
template <int NIN, int NA, bool DISC, int FEAT>
__global__ __launch_bounds__(64 * kPairWaves, 2) void rollout_pair_kernel(RolloutArgs a) {
  using Lane = MlpPair<NIN, NA, DISC>;
  constexpr int NX = Lane::NX;
  constexpr int NMK = NX + round4(NA);
  constexpr int MKS = NMK % 8 == 0 ? NMK + 4 : NMK;
  __shared__ float4 env4[NIN * MKS / 4];
  __shared__ float4 wtile[kPairWaves * Lane::kTileF4];
  __shared__ PairScratch scratch[kPairWaves];
  float* envMK = reinterpret_cast<float*>(env4);
  for (int e = threadIdx.x; e < NIN * MKS; e += blockDim.x) {
    const int i = e / MKS, k = e % MKS;
    envMK[e] = kPreScale * (k < NIN ? a.M[i * NIN + k] : (k >= NX && k < NX + NA ? a.K[i * NA + k - NX] : 0.f));
  }
  __syncthreads();

  const int tid = threadIdx.x & 63, wv = threadIdx.x >> 6, hh = tid >> 5, t = tid & 31;
  const int lane0 = a.lane_base + (blockIdx.x * kPairWaves + wv) * 2;
  if (lane0 >= a.n_lanes) return;  // whole wave idle
  const bool active = lane0 + hh < a.n_lanes;
  const int lane = active ? lane0 + hh : lane0;  // an idle half shadows its partner, writes nothing

  ParamSrc src = a.lanes.src(lane);
  const bool det = a.lanes.deterministic ? a.lanes.deterministic[lane] != 0 : false;
  Lane pl;
  pl.load(src, t, tid, a.bn_mean, a.bn_var, wtile + wv * Lane::kTileF4);
  {
    double n2 = src.n2;
#pragma unroll
    for (int m = 16; m >= 1; m >>= 1) n2 += __shfl_xor(n2, m, kWave);
    // formed here: otherwise the compiler sinks the norm (and its store) past the step loop and keeps every
    // element's sigma * eps in scratch across it
    asm volatile("" : "+v"(n2));
    if (t == 0 && active && a.norm2) a.norm2[lane] = n2;
  }

  const int ji = t < NIN ? t : NIN - 1;
  constexpr bool norm_obs = (FEAT & 4) != 0;
  const float om = norm_obs ? a.obs_mean[ji] : 0.f;
  const float osd = norm_obs ? a.obs_std[ji] : 1.f;
  auto policy_input = [&](float s) {
    float x = s;
    if (norm_obs) x = fminf(fmaxf((s - om) / osd, -10.f), 10.f);  // agent.py:40-41
    return pl.input_transform(x);
  };
  float s = a.s0[ji];
  const int T = a.T;
  const uint64_t key = a.key;
  const uint64_t ulane = (uint64_t)(a.lanes.lane_offset + lane);
  double racc = 0.0;
  float eacc = 0.f;
  const int o = t & 15;
  constexpr int kDrawsPerStep = DISC ? 1 : NA;
  constexpr int kStepsPerBatch = 32 / kDrawsPerStep;
  constexpr bool kTerm = (FEAT & 16) != 0;
  bool alive0 = true, alive1 = true;  // wave-uniform: half 0 / half 1 still stepping (kTerm)
  int n0 = T, n1 = T;                 // their env.step counts
  auto alive_me = [&]() { return hh ? alive1 : alive0; };
  float rbuf = 0.f;
  const int zbase = 4 * (32 * hh + (DISC ? 0 : (o < NA ? o : 0)));
  auto* sc = &scratch[wv];
  [[maybe_unused]] float* xs = sc->x[hh];
  float* h1s = sc->h1[hh];
  const float* mrow = envMK + ji * MKS;
  constexpr bool kSame = !DISC && !norm_obs;
  typename Lane::L1Rows l1rows;
  pl.l1_prefetch(l1rows, mrow);
  float kr[DISC ? 1 : NA];  // K row t: loop-invariant, kept in VGPRs
#pragma unroll
  for (int m = 0; m < (DISC ? 1 : NA); ++m) kr[m] = mrow[NX + m];
  int tb = 0;
#ifdef FDR_PHASE_STAMPS
  uint64_t ph_acc[5] = {0, 0, 0, 0, 0};
  uint64_t ph_last = 0;
  auto mark = [&](int k, float dep) {
    uint64_t now;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(now) : "v"(dep));
    if (k >= 0) ph_acc[k] += now - ph_last;
    ph_last = now;
  };
#else
  auto mark = [](int, float) {};
#endif
  // draw batch starting at step st: thread t holds the draw of (step st + t / k, dim t % k)
  auto draw = [&](int st) {
    const int ds = t / kDrawsPerStep, dk = t % kDrawsPerStep;
    const uint64_t hsh = hash_ctr(key, ulane, (uint64_t)(st + ds), (uint64_t)dk);
    rbuf = DISC ? uniform24(hsh) : normal_bm(hsh);
  };
  auto step = [&](int st, int tb) {
    // this step's draw: the uniform (discrete) or the normal of action dim o (continuous)
    const float zt = __builtin_bit_cast(
        float, __builtin_amdgcn_ds_bpermute(zbase + 4 * kDrawsPerStep * tb, __builtin_bit_cast(int, rbuf)));
    if constexpr (FEAT & 1) {
      if (t < NIN && active && (!kTerm || alive_me())) a.states[((int64_t)lane * T + st) * NIN + t] = s;
    }
    float pre = 0.f;
    xs[t] = t < NIN ? policy_input(s) : (t == NIN ? 1.f : 0.f);
    if constexpr (!kSame) h1s[t] = t < NIN ? s : 0.f;
    wave_lds_sync();
    const f2 h1 = pl.template layer1_env<kSame>(xs, h1s, l1rows, pre);

    mark(0, h1.x);
    const float y = pl.layers23(h1, h1s, t, mark);
    pl.l1_prefetch(l1rows, mrow);  // next step's rows, in flight during the action and env phases
    if constexpr (DISC) {
      const float p = det ? pl.softmax(y, t) : pl.template softmax<false, true>(y, t);
      float pv[NA];
      row_bcast_all(p, pv, std::make_integer_sequence<int, NA>{});  // pv[i] = p of output i
      float tot = 0.f;
#pragma unroll
      for (int i = 0; i < NA; ++i) tot += pv[i];
      int act_d = 0;
      if (det) {
        float best = pv[0];
#pragma unroll
        for (int i = 1; i < NA; ++i) {
          act_d = pv[i] > best ? i : act_d;
          best = fmaxf(best, pv[i]);
        }
      } else {
        const float target = zt * tot;
        float cs = 0.f;
#pragma unroll
        for (int i = 0; i < NA - 1; ++i) {
          cs += pv[i];
          act_d += cs <= target ? 1 : 0;
        }
      }
      eacc -= (o < NA && (!kTerm || alive_me())) ? disc_entropy_term(p, tot) : 0.f;
      pre += mrow[NX + act_d];
    } else {
      const float th = tanh_act<Lane::kPre>(y);
      const float sd = std_from_tanh(dpp_mov<kDppRowShl + NA>(th));
      if constexpr (kTerm)
        eacc += alive_me() ? __builtin_amdgcn_logf(sd) : 0.f;
      else
        eacc += __builtin_amdgcn_logf(sd);
      const float act_c = det ? th : gauss_action(th, sd, zt);
      mark(3, act_c);
      dpp_tail<NA>(pre, act_c, kr);  // a[m] sits in thread m of both rows of the half
    }
    s = tanh_pre(pre);  // M, K stored x kPreScale
    mark(4, s);
    if constexpr (kTerm) {
      racc += alive_me() ? (double)s : 0.0;  // thread 0 of the half holds the reward s'[0]
      // done after this step (agent.py:50-52): the half's state element done_dim sits in its thread done_dim
      const bool d0 = fabsf(readlane_f(s, a.done_dim)) > a.done_thr;
      const bool d1 = fabsf(readlane_f(s, 32 + a.done_dim)) > a.done_thr;
      if (alive0 && d0) {
        alive0 = false;
        n0 = st + 1;
      }
      if (alive1 && d1) {
        alive1 = false;
        n1 = st + 1;
      }
      return !alive0 && !alive1;
    } else {
      racc += (double)s;  // thread 0 of the half holds the reward s'[0]
      return false;
    }
  };
  if constexpr (!DISC) {
    [&] {
      // continuous: the loop unrolled by the draw batch (5 steps for 6 dims); the draw is issued
      // unconditionally at the top of the unrolled body (det lanes ignore it), so it schedules into the
      // first step's waits instead of sitting behind a branch
      int st = 0;
      for (; st + kStepsPerBatch <= T; st += kStepsPerBatch) {
        asm volatile("" ::: "memory");
        mark(-1, s);
        draw(st);
#pragma unroll
        for (int k = 0; k < kStepsPerBatch; ++k) {
          if (k) {
            asm volatile("" ::: "memory");
            mark(-1, s);
          }
          if (step(st + k, k)) return;  // kTerm: both halves done
        }
      }
      if (st < T) {
        draw(st);
        for (int k = 0; st + k < T; ++k) {
          asm volatile("" ::: "memory");
          mark(-1, s);
          if (step(st + k, k)) return;
        }
      }
    }();
  } else {
    for (int st = 0; st < T; ++st) {
      asm volatile("" ::: "memory");
      mark(-1, s);
      if (!det && tb == 0) draw(st);
      if (step(st, tb)) break;
      tb = tb + 1 == kStepsPerBatch ? 0 : tb + 1;
    }
  }

#ifdef FDR_PHASE_STAMPS
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int k = 0; k < 5; ++k) g_phase_stamps[k] = ph_acc[k];
#endif
  eacc *= 0.693147180559945309f;  // log2 -> ln (both kinds)
  double esum = (t < NA) ? (double)eacc : 0.0;  // row 0 of the half: one copy of each output
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) esum += __shfl_xor(esum, m, kWave);
  if (t == 0 && active) {
    double r = racc;
    if (a.jiggle) r += (hash_ctr(key, ulane, kJiggleT, 15) & 1ull) ? 1e-12 : -1e-12;
    a.ret[lane] = r;
    const int nsteps = hh ? n1 : n0;
    double e = esum / (double)nsteps;
    if constexpr (!DISC) e += (double)NA * 1.4189385332046727;
    a.ent[lane] = e;
    a.steps[lane] = nsteps;
  }
}

// ---------------------------------------------------------------------------------------------
// Dispatch tables (compiled shapes)
// ---------------------------------------------------------------------------------------------
#define FDR_SHAPES(X) \
  X(2, 9, true)       \
  X(4, 2, true)       \
  X(8, 4, true)       \
  X(17, 6, false)     \
  X(11, 3, false)     \
  X(8, 2, false)

int launch_policy_forward(const PolicyKey& k, const LanesArgs& lanes, int n_lanes,
                          const float* bn_mean, const float* bn_var, const float* x, float* out0,
                          float* out1, hipStream_t stream) {
  const dim3 grid((n_lanes + kLanesPerBlock - 1) / kLanesPerBlock), block(64 * kLanesPerBlock);
#define FDR_FWD(NIN, NA, DISC)                                                                  \
  if (k.n_in == NIN && k.n_act == NA && k.discrete == DISC) {                                   \
    if (Layout<NIN, NA, DISC>::P != k.n_params)                                                 \
      return set_error(FDR_ERR_INVALID, "n_params does not match the policy layout");           \
    hipLaunchKernelGGL((policy_forward_kernel<NIN, NA, DISC>), grid, block, 0, stream, lanes,   \
                       n_lanes, bn_mean, bn_var, x, out0, out1);                                \
    return check_launch("policy_forward_kernel");                                               \
  }
  FDR_SHAPES(FDR_FWD)
#undef FDR_FWD
  return set_error(FDR_ERR_UNSUPPORTED, "no compiled policy_forward for this (kind, n_in, n_act)");
}

template <int NIN, int NA, bool DISC, int ENV, bool WIDE = false>
static void launch_feat(const RolloutArgs& args, dim3 grid, dim3 block, hipStream_t stream) {
  const int feat = (args.states ? 1 : 0) | (args.os_mean ? 2 : 0) | (args.obs_mean ? 4 : 0);
#define FDR_FEAT_CASE(F) \
  case F: hipLaunchKernelGGL((rollout_kernel<NIN, NA, DISC, ENV, F, WIDE>), grid, block, 0, stream, args); break;
  // terminating env instances (bit 4) only for the synthetic env, so the fixed-length kernels stay as they are
  const int term = (ENV == FDR_ENV_SYNTH && args.done_thr > 0.f) ? 16 : 0;
  if constexpr (!WIDE) {
    if (args.u_inject) {  // injected draws (never with the Welford statistics: fdr_rollout_ex refuses it)
      switch (feat | 8 | term) {
        FDR_FEAT_CASE(8) FDR_FEAT_CASE(9) FDR_FEAT_CASE(12) FDR_FEAT_CASE(13)
        FDR_FEAT_CASE(24) FDR_FEAT_CASE(25) FDR_FEAT_CASE(28) FDR_FEAT_CASE(29)
      }
      return;
    }
  }
  switch (feat | term) {
    FDR_FEAT_CASE(0) FDR_FEAT_CASE(1) FDR_FEAT_CASE(2) FDR_FEAT_CASE(3)
    FDR_FEAT_CASE(4) FDR_FEAT_CASE(5) FDR_FEAT_CASE(6) FDR_FEAT_CASE(7)
    FDR_FEAT_CASE(16) FDR_FEAT_CASE(17) FDR_FEAT_CASE(18) FDR_FEAT_CASE(19)
    FDR_FEAT_CASE(20) FDR_FEAT_CASE(21) FDR_FEAT_CASE(22) FDR_FEAT_CASE(23)
  }
#undef FDR_FEAT_CASE
}

// More lanes than one resident round (2 waves per SIMD = 16 lanes per CU) go out as consecutive launches of
// equal rounds: one launch of two rounds lets early-finishing CUs start second-round workgroups while slow
// ones still run their first, and the last CUs' second round then runs alone at the end.
template <int NIN, int NA, bool DISC>
static void launch_pair(const RolloutArgs& args, int round_lanes, hipStream_t stream) {
  const int quantum = 2 * kPairWaves;
  const int n_rounds = round_lanes > 0 ? (args.n_lanes + round_lanes - 1) / round_lanes : 1;
  const int per = ((args.n_lanes + n_rounds - 1) / n_rounds + quantum - 1) / quantum * quantum;
  const int feat = (args.states ? 1 : 0) | (args.obs_mean ? 4 : 0) | (args.done_thr > 0.f ? 16 : 0);
  RolloutArgs r = args;
  for (int base = 0; base < args.n_lanes; base += per) {
    r.lane_base = base;
    const dim3 grid((std::min(per, args.n_lanes - base) + quantum - 1) / quantum), block(64 * kPairWaves);
#define FDR_PAIR_CASE(F) \
  case F: hipLaunchKernelGGL((rollout_pair_kernel<NIN, NA, DISC, F>), grid, block, 0, stream, r); break;
    switch (feat) {
      FDR_PAIR_CASE(0) FDR_PAIR_CASE(1) FDR_PAIR_CASE(4) FDR_PAIR_CASE(5)
      FDR_PAIR_CASE(16) FDR_PAIR_CASE(17) FDR_PAIR_CASE(20) FDR_PAIR_CASE(21)
    }
#undef FDR_PAIR_CASE
  }
}

static int pair_round_lanes(const Context& ctx) { return 16 * context_cus(ctx); }

// Synthetic-env rollouts: rollout_pair_kernel (two lanes per wave) or rollout_kernel (one lane per
// wave), by the context's rollout_impl: FDR_ROLLOUT_AUTO (default) takes the pair kernel once it puts
// >= 2 waves on every SIMD (n_lanes >= 4 x SIMDs; measured DESIGN.md 3.0: below that the one-lane kernel's
// extra waves win).  The Welford obs statistics and the trap env always use rollout_kernel.
static bool use_pair_kernel(const Context& ctx, int n_lanes) {
  if (ctx.rollout_impl != FDR_ROLLOUT_AUTO) return ctx.rollout_impl == FDR_ROLLOUT_PAIR;
  return n_lanes >= 4 * 4 * context_cus(ctx);  // 4 SIMDs per CU, 2 lanes x 2 waves per SIMD
}

// The register-rich one-lane kernel (rollout_kernel<WIDE>) when its 2-waves-per-SIMD occupancy holds
// every lane in one pass (n_lanes <= 8 x CUs): below that the step is a latency chain, and VGPR room
// buys a shorter one.
static bool use_wide_kernel(const Context& ctx, int n_lanes) {
  if (ctx.rollout_impl != FDR_ROLLOUT_AUTO) return ctx.rollout_impl == FDR_ROLLOUT_WIDE;
  return n_lanes <= 2 * 4 * context_cus(ctx);
}

int launch_rollout(const Context& ctx, const PolicyKey& k, int env_kind, const RolloutArgs& args, hipStream_t stream) {
  const dim3 grid((args.n_lanes + kLanesPerBlock - 1) / kLanesPerBlock), block(64 * kLanesPerBlock);
#define FDR_ROLL(NIN, NA, DISC)                                                                 \
  if (k.n_in == NIN && k.n_act == NA && k.discrete == DISC) {                                   \
    if (Layout<NIN, NA, DISC>::P != k.n_params)                                                 \
      return set_error(FDR_ERR_INVALID, "n_params does not match the policy layout");           \
    if (env_kind == FDR_ENV_SYNTH) {                                                            \
      if (use_pair_kernel(ctx, args.n_lanes) && !args.os_mean && !args.u_inject) {                         \
        launch_pair<NIN, NA, DISC>(args, pair_round_lanes(ctx), stream);                        \
        return check_launch("rollout_pair_kernel<synth>");                                      \
      }                                                                                         \
      if (use_wide_kernel(ctx, args.n_lanes) && !args.u_inject) {                               \
        launch_feat<NIN, NA, DISC, FDR_ENV_SYNTH, true>(args, grid, block, stream);             \
        return check_launch("rollout_kernel<synth, wide>");                                     \
      }                                                                                         \
      launch_feat<NIN, NA, DISC, FDR_ENV_SYNTH>(args, grid, block, stream);                     \
      return check_launch("rollout_kernel<synth>");                                             \
    }                                                                                           \
    if constexpr (NIN == 2 && NA == 9 && DISC) {                                                \
      if (env_kind == FDR_ENV_TRAP) {                                                           \
        launch_feat<NIN, NA, DISC, FDR_ENV_TRAP>(args, grid, block, stream);                    \
        return check_launch("rollout_kernel<trap>");                                            \
      }                                                                                         \
    }                                                                                           \
    return set_error(FDR_ERR_UNSUPPORTED, "env kind not compiled for this policy shape");       \
  }
  FDR_SHAPES(FDR_ROLL)
#undef FDR_ROLL
  return set_error(FDR_ERR_UNSUPPORTED, "no compiled rollout for this (kind, n_in, n_act)");
}

}  // namespace fdr

namespace fdr {

// ---------------------------------------------------------------------------------------------
// Welford merge (utils/math_helpers.py:68-87, increment_from_obs_stats_update): the lanes' partial
// statistics folded into the accumulator in lane order, f32, the reference's operation order.
// One thread per observation dimension; lanes with count 0 are skipped, as the reference.
// ---------------------------------------------------------------------------------------------
__global__ void obs_stats_merge_kernel(const float* __restrict__ mean, const float* __restrict__ m2,
                                       const int32_t* __restrict__ count, int n, int d, float* acc_mean,
                                       float* acc_m2, int64_t* acc_count) {
#pragma clang fp contract(off)
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  int64_t c = *acc_count;
  float m = j < d ? acc_mean[j] : 0.f, v = j < d ? acc_m2[j] : 0.f;
  for (int i = 0; i < n; ++i) {
    const int64_t oc = count[i];
    if (oc == 0) continue;
    const int64_t cnt = c + oc;
    if (j < d) {
      const float om = mean[(int64_t)i * d + j], ov = m2[(int64_t)i * d + j];
      const float md = om - m;
      const float mds = md * md;
      const float cm = ((float)c * m + (float)oc * om) / (float)cnt;
      v = (v + ov) + ((mds * (float)c) * (float)oc) / (float)cnt;
      m = cm;
    }
    c = cnt;
  }
  if (j < d) {
    acc_mean[j] = m;
    acc_m2[j] = v;
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) *acc_count = c;
}

int launch_obs_stats_merge(const float* mean, const float* m2, const int32_t* count, int n, int d, float* acc_mean,
                           float* acc_m2, int64_t* acc_count, hipStream_t stream) {
  if (d > 1024) return set_error(FDR_ERR_UNSUPPORTED, "obs_dim > 1024");
  hipLaunchKernelGGL(obs_stats_merge_kernel, dim3(1), dim3(1024), 0, stream, mean, m2, count, n, d, acc_mean, acc_m2,
                     acc_count);
  return check_launch("obs_stats_merge_kernel");
}

}  // namespace fdr

#ifdef FDR_PHASE_STAMPS
extern "C" int fdr_debug_phase_read(unsigned long long* out5) {
  return hipMemcpyFromSymbol(out5, HIP_SYMBOL(fdr::g_phase_stamps), 5 * sizeof(unsigned long long)) == hipSuccess
             ? 0 : -1;
}
#endif
