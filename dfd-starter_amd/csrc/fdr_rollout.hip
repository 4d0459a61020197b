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
//   * Activations cross lanes in registers: a 3-instruction permlane all-gather replicates the
//     64-vector in every 16-lane row, then every FMA reads its input element through DPP
//     row_newbcast (fdr_wave.h) -> one VALU op per MAC, no LDS traffic in the T-step loop except
//     the env matrix rows.
//   * The env (synthetic linear-tanh system or the trap gridworld) runs inside the same loop.
//   * 4 lanes (waves) per 256-thread workgroup, <= 128 VGPRs -> 16 waves/CU: 4096 lanes fill
//     all 256 CUs in one wave of workgroups.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "fdr_common.h"
#include "fdr_internal.h"
#include "fdr_wave.h"

namespace fdr {

constexpr int kLanesPerBlock = 4;

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

// ---------------------------------------------------------------------------------------------
// One lane's policy, register resident.  Wave lane j = 16 r + c.
// ---------------------------------------------------------------------------------------------
template <int NIN, int NA, bool DISC>
struct MlpLane {
  using L = Layout<NIN, NA, DISC>;
  static constexpr int NOUT = L::NOUT;
  static constexpr int NQI = (NIN + 15) / 16;  // gathered rows of the input vector
  // Wide inputs keep W1 in a per-wave LDS tile [k][64] (lane-contiguous, conflict-free
  // ds_read_b32) instead of NIN persistent VGPRs: keeps the rollout at <= 128 VGPRs.
  static constexpr bool kW1Lds = NIN > 8;
  static constexpr int kW1Regs = kW1Lds ? 1 : NIN;
  static constexpr int kLdsFloats = kW1Lds ? NIN * kWave : 0;
  float w1[kW1Regs], b1;
  float* w1s;  // LDS tile (kW1Lds)
  float w2[kHidden], b2;
  float w3[16], b3;  // W3[o = c][16 r .. 16 r + 15]
  float a0, c0, a1, c1, a2, c2;  // discrete: folded BN for input j / hidden unit j

  __device__ __forceinline__ void load(ParamSrc& src, int j, const float* bn_mean,
                                       const float* bn_var, float* lds_tile) {
    const int o = j & 15, r = j >> 4;
    w1s = lds_tile;
    if constexpr (kW1Lds) {
#pragma unroll
      for (int k = 0; k < NIN; ++k) w1s[k * kWave + j] = src.get(L::L1W + (int64_t)j * NIN + k);
      wave_lds_sync();
    } else {
#pragma unroll
      for (int k = 0; k < NIN; ++k) w1[k] = src.get(L::L1W + (int64_t)j * NIN + k);
    }
    b1 = src.get(L::L1B + j);
#pragma unroll
    for (int k = 0; k < kHidden; ++k) w2[k] = src.get(L::L2W + (int64_t)j * kHidden + k);
    b2 = src.get(L::L2B + j);
    if (o < NOUT) {
#pragma unroll
      for (int k = 0; k < 16; ++k) w3[k] = src.get(L::L3W + (int64_t)o * kHidden + 16 * r + k);
      b3 = r == 0 ? src.get(L::L3B + o) : src.get_nocount(L::L3B + o);
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) w3[k] = 0.f;
      b3 = 0.f;
    }
    a0 = c0 = a1 = c1 = a2 = c2 = 0.f;
    if constexpr (DISC) {
      if (j < NIN) {
        const float w = src.get(L::BN0W + j), b = src.get(L::BN0B + j);
        bn_fold(w, b, bn_mean ? bn_mean[j] : 0.f, bn_var ? bn_var[j] : 1.f, a0, c0);
      }
      {
        const float w = src.get(L::BN1W + j), b = src.get(L::BN1B + j);
        bn_fold(w, b, bn_mean ? bn_mean[NIN + j] : 0.f, bn_var ? bn_var[NIN + j] : 1.f, a1, c1);
      }
      {
        const float w = src.get(L::BN2W + j), b = src.get(L::BN2B + j);
        bn_fold(w, b, bn_mean ? bn_mean[NIN + kHidden + j] : 0.f,
                bn_var ? bn_var[NIN + kHidden + j] : 1.f, a2, c2);
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

  // Both hidden layers and the head: returns the head pre-activation for output o = j & 15
  // (identical in the 4 rows).  X = row all-gather of the policy input.
  __device__ __forceinline__ float forward(const float (&X)[NQI], int j) const {
    float z;
    if constexpr (kW1Lds) {
      float wt[NIN];
#pragma unroll
      for (int k = 0; k < NIN; ++k) wt[k] = w1s[k * kWave + j];
      z = dot_gathered<NIN>(X, wt, b1);
    } else {
      z = dot_gathered<NIN>(X, w1, b1);
    }
    float h;
    if constexpr (DISC) {
      h = fmaf(fmaxf(z, 0.f), a1, c1);
    } else {
      h = tanh_fast(z);
    }
    float Hq[4];
    row_allgather<4>(h, Hq);
    z = dot_gathered<kHidden>(Hq, w2, b2);
    if constexpr (DISC) {
      h = fmaf(fmaxf(z, 0.f), a2, c2);
    } else {
      h = tanh_fast(z);
    }
    const float y = dot_row16(h, w3, 0.f);  // row r: inputs 16 r .. 16 r + 15 are its own lanes
    return row_allreduce_sum(y) + b3;
  }

  // Discrete: softmax across the row (o = j & 15 < NA); returns p_o, 0 for o >= NA.
  __device__ __forceinline__ float softmax(float logit, int j) const {
    const bool valid = (j & 15) < NOUT;
    const float v = valid ? logit : -FLT_MAX;
    const float mx = row16_max(v);
    const float e = valid ? expf(v - mx) : 0.f;
    return e / row16_sum(e);
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
  __shared__ float w1tile[kLanesPerBlock * (Lane::kLdsFloats > 0 ? Lane::kLdsFloats : 1)];
  const int j = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int lane = blockIdx.x * kLanesPerBlock + wv;
  if (lane >= n_lanes) return;
  ParamSrc src = lanes.src(lane);
  Lane pl;
  pl.load(src, j, bn_mean, bn_var, w1tile + wv * Lane::kLdsFloats);
  const float xin = j < NIN ? pl.input_transform(x[(int64_t)lane * NIN + j]) : 0.f;
  float X[Lane::NQI];
  row_allgather<Lane::NQI>(xin, X);
  const float y = pl.forward(X, j);
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
// FEAT bit 0: record visited observations (fdr_rollout_states); bit 1: Welford obs statistics
template <int NIN, int NA, bool DISC, int ENV, int FEAT>
__global__ __launch_bounds__(64 * kLanesPerBlock, 4) void rollout_kernel(RolloutArgs a) {
  using Lane = MlpLane<NIN, NA, DISC>;
  constexpr int NQI = Lane::NQI;
  constexpr int MS = (round4(NIN) % 8 == 0) ? round4(NIN) + 4 : round4(NIN);  // M row stride
  constexpr int KS = round4(NA) + ((round4(NA) % 8 == 0) ? 4 : 0);             // K row stride
  __shared__ float4 env4[(ENV == FDR_ENV_SYNTH) ? (NIN * MS + NIN * KS + 3) / 4 : 1];
  __shared__ float w1tile[kLanesPerBlock * (Lane::kLdsFloats > 0 ? Lane::kLdsFloats : 1)];
  float* envM = reinterpret_cast<float*>(env4);
  float* envK = envM + NIN * MS;

  const int j = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int lane = blockIdx.x * kLanesPerBlock + wv;
  if constexpr (ENV == FDR_ENV_SYNTH) {
    for (int e = threadIdx.x; e < NIN * NIN; e += blockDim.x) envM[(e / NIN) * MS + e % NIN] = a.M[e];
    for (int e = threadIdx.x; e < NIN * NA; e += blockDim.x) envK[(e / NA) * KS + e % NA] = a.K[e];
    __syncthreads();  // the only cross-wave hand-off: shared env matrices
  }
  if (lane >= a.n_lanes) return;

  ParamSrc src = a.lanes.src(lane);
  const bool det = a.lanes.deterministic ? a.lanes.deterministic[lane] != 0 : false;
  Lane pl;
  pl.load(src, j, a.bn_mean, a.bn_var, w1tile + wv * Lane::kLdsFloats);
  const double n2 = wave_sum(src.n2);

  const int ji = j < NIN ? j : NIN - 1;
  const bool norm_obs = a.obs_mean != nullptr;
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

  for (int t = 0; t < T; ++t) {
    const int tb = t % kStepsPerBatch;
    if (!det && tb == 0) {
      const int ds = j / kDrawsPerStep, dk = j % kDrawsPerStep;
      const uint64_t h = hash_ctr(key, ulane, (uint64_t)(t + ds), (uint64_t)dk);
      rbuf = DISC ? uniform24(h) : normal_bm(h);
    }
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
    float X[NQI];
    row_allgather<NQI>(policy_input(s), X);
    const float y = pl.forward(X, j);
    int act_d = 0;
    float act_c = 0.f;
    if constexpr (DISC) {
      const float p = pl.softmax(y, j);
      float pv[NA];
#pragma unroll
      for (int i = 0; i < NA; ++i) pv[i] = readlane_f(p, i);
      float tot = 0.f;  // sequential f32 cumsum, the oracle's order
#pragma unroll
      for (int i = 0; i < NA; ++i) tot += pv[i];
      // Branch-free selection (selects, no data-dependent control flow):
      //   argmax = first maximal index; inverse CDF = first i with cumsum_i > target, i.e. the
      //   number of (monotone) partial sums <= target, capped at NA - 1.
      if (det) {
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
      const float pn = p / tot;
      const float lg = pn > 0.f ? logf(pn) : -FLT_MAX;
      eacc -= (j < NA) ? pn * lg : 0.f;
    } else {
      const float th = tanh_fast(y);
      const float sd = std_from_tanh(dpp_mov<kDppRowShl + NA>(th));
      eacc += (j < NA) ? __logf(sd) : 0.f;
      const float z = __shfl(rbuf, tb * NA + (o < NA ? o : 0), kWave);  // normal (t, o)
      act_c = det ? th : gauss_action(th, sd, z);
    }

    // ---- env step ----
    if constexpr (ENV == FDR_ENV_SYNTH) {
      float S[NQI];
      if (!DISC && !norm_obs) {
#pragma unroll
        for (int q = 0; q < NQI; ++q) S[q] = X[q];  // policy input == env state: reuse the gather
      } else {
        row_allgather<NQI>(s, S);
      }
      const float* mrow = envM + ji * MS;
      float mr[NIN];
#pragma unroll
      for (int k = 0; k < NIN; ++k) mr[k] = mrow[k];
      float pre = dot_gathered<NIN>(S, mr, 0.f);
      if constexpr (DISC) {
        pre += envK[ji * KS + act_d];
      } else {
        const float* krow = envK + ji * KS;
        float kr[NA];
#pragma unroll
        for (int m = 0; m < NA; ++m) kr[m] = krow[m];
        dpp_tail<NA>(pre, act_c, kr);  // a[m] sits in lane m of every row
      }
      s = tanh_fast(pre);
      racc += (double)s;  // lane 0 holds the reward s'[0]; other lanes' sums are discarded
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
  }

  // ---- epilogue ----
  const double esum = wave_sum((j < NA) ? (double)eacc : 0.0);
  if (j == 0) {
    double r = racc;
    if (a.jiggle) r += (hash_ctr(key, ulane, kJiggleT, 15) & 1ull) ? 1e-12 : -1e-12;
    a.ret[lane] = r;
    double e = esum / (double)T;
    if constexpr (!DISC) e += (double)NA * 1.4189385332046727;  // 0.5 + 0.5*ln(2*pi) per dim
    a.ent[lane] = e;
    a.steps[lane] = T;
    if (a.norm2) a.norm2[lane] = n2;
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

template <int NIN, int NA, bool DISC, int ENV>
static void launch_feat(const RolloutArgs& args, dim3 grid, dim3 block, hipStream_t stream) {
  const int feat = (args.states ? 1 : 0) | (args.os_mean ? 2 : 0);
  switch (feat) {
    case 0: hipLaunchKernelGGL((rollout_kernel<NIN, NA, DISC, ENV, 0>), grid, block, 0, stream, args); break;
    case 1: hipLaunchKernelGGL((rollout_kernel<NIN, NA, DISC, ENV, 1>), grid, block, 0, stream, args); break;
    case 2: hipLaunchKernelGGL((rollout_kernel<NIN, NA, DISC, ENV, 2>), grid, block, 0, stream, args); break;
    default: hipLaunchKernelGGL((rollout_kernel<NIN, NA, DISC, ENV, 3>), grid, block, 0, stream, args); break;
  }
}

int launch_rollout(const PolicyKey& k, int env_kind, const RolloutArgs& args, hipStream_t stream) {
  const dim3 grid((args.n_lanes + kLanesPerBlock - 1) / kLanesPerBlock), block(64 * kLanesPerBlock);
#define FDR_ROLL(NIN, NA, DISC)                                                                 \
  if (k.n_in == NIN && k.n_act == NA && k.discrete == DISC) {                                   \
    if (Layout<NIN, NA, DISC>::P != k.n_params)                                                 \
      return set_error(FDR_ERR_INVALID, "n_params does not match the policy layout");           \
    if (env_kind == FDR_ENV_SYNTH) {                                                            \
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
