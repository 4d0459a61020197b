// fdr_atari.hip -- AtariPolicy (policies/atari.py:7-51) rollouts on gfx950.
//
// Same pack / prep / finish machinery as the ImpalaPolicy path (fdr_impala.hip): theta'_l gathered
// once per rollout into a per-lane pack (conv weights as v_mfma_f32_16x16x4_f32 B-fragments with
// 8x8 / 4x4 taps, fc W^T), then per step:
//   atari_conv_kernel  one 512-thread workgroup per (lane, env): synthetic 4x84x84 stacked frame ->
//                      conv 8x8 s4 + BN + ReLU (LDS) -> conv 4x4 s2 + BN + ReLU -> 2592 features
//   atari_core_kernel  one workgroup per lane: fc 2592 -> 256 (float4 W^T streams), BN1d, ReLU, head,
//                      softmax, action, reward, per-step entropy
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>

#include "fdr_impala.h"

namespace fdr {
namespace atari {

using impala::Layout;
using impala::Section;
using impala::StepArgs;
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kC = 4, kH = 84, kW = 84, kPlane = kH * kW, kFramePix = kC * kPlane;
constexpr int kO1 = 20, kO2 = 9;         // conv output sides
constexpr int kFeat = 32 * kO2 * kO2;    // 2592 (policies/atari.py:47)
constexpr int kFc = 256;
constexpr int kThreads = 512;

struct Offsets {  // pack offsets (floats) beyond what Layout carries
  int32_t c1w, c1b, bn1, c2w, c2b, bn2, fcw, fcb, bn3, head_w, head_b;
};

static int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// Walk the reference parameters() order (atari.py:36-51) into pack sections.
bool make_layout(int n_act, Layout* L, Offsets* o) {
  if (n_act < 1 || n_act > impala::kMaxAct) return false;
  *L = Layout{};
  L->n_act = n_act;
  int32_t dst = 0, src = 0;
  auto add = [&](int32_t kind, int32_t len, int32_t a, int32_t b, int32_t src_len) {
    dst = (int32_t)round_up(dst, 16);
    Section& s = L->sec[L->n_sections++];
    s = Section{dst, len, src, kind, a, b};
    const int32_t at = dst;
    dst += len;
    src += src_len;
    return at;
  };
  o->c1w = add(impala::kConvFrag, 4 * 64 * 16, 4 | (64 << 8), 16, 16 * 4 * 64);
  o->c1b = add(impala::kCopy, 16, 0, 0, 16);
  o->bn1 = add(impala::kCopy, 32, 0, 0, 32);      // BatchNorm2d(16) weight, bias
  o->c2w = add(impala::kConvFrag, 16 * 16 * 32, 16 | (16 << 8), 32, 32 * 16 * 16);
  o->c2b = add(impala::kCopy, 32, 0, 0, 32);
  o->bn2 = add(impala::kCopy, 64, 0, 0, 64);      // BatchNorm2d(32)
  o->fcw = add(impala::kTranspose, kFeat * kFc, kFc, kFeat, kFeat * kFc);
  o->fcb = add(impala::kCopy, kFc, 0, 0, kFc);
  o->bn3 = add(impala::kCopy, 2 * kFc, 0, 0, 2 * kFc);  // BatchNorm1d(256)
  o->head_w = add(impala::kCopy, n_act * kFc + n_act, 0, 0, n_act * kFc + n_act);
  o->head_b = o->head_w + n_act * kFc;
  L->P = src;
  L->pack = round_up(dst, 64);
  L->n_bn_stats = 16 + 32 + kFc;
  return true;
}

struct Args {
  StepArgs s;
  Offsets o;
};

// acc[i] += A(tile) * B over K = CIN * KH * KW; output pixel m -> (m / OW, m % OW), input pixel
// (S*oy + ky, S*ox + kx) of the [CIN][IH][IW] image X (no padding); k-step = tap-major, 4 channels.
template <int CIN, int NT, int TPW, int MT, int NPIX, int OW, int S, int IW, int IPLANE, int KW, int KS>
__device__ __forceinline__ void conv_s(const float* X, const float (&bf)[KS], f32x4 (&acc)[TPW], int wave, int lane) {
  int base[TPW];
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    int mt = (wave + 8 * i) / NT;
    mt = mt < MT ? mt : MT - 1;
    int m = mt * 16 + (lane & 15);
    m = m < NPIX ? m : NPIX - 1;
    base[i] = g * IPLANE + S * (m / OW) * IW + S * (m % OW);
    acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int tap = s / (CIN / 4);
    const int off = 4 * (s % (CIN / 4)) * IPLANE + (tap / KW) * IW + (tap % KW);
#pragma unroll
    for (int i = 0; i < TPW; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(X[base[i] + off], bf[s], acc[i], 0, 0, 0);
  }
}

__global__ __launch_bounds__(kThreads) void atari_conv_kernel(Layout L, Args A) {
  const StepArgs& a = A.s;
  const Offsets& o = A.o;
  __shared__ float frame[kFramePix];
  __shared__ float h1[16 * kO1 * kO1];
  __shared__ float bnt[2 * (16 + 32)];
  const int b = blockIdx.x, xcd = b & 7, slot = b >> 3;
  const int lane = (slot / a.envs) * 8 + xcd, e = slot % a.envs;
  if (lane >= a.n_lanes) return;
  const int wave = threadIdx.x >> 6, ln = threadIdx.x & 63;
  const int64_t env = (int64_t)lane * a.envs + e;
  const float* pk = a.pack + (int64_t)lane * a.pack_stride;

  float bf1[64];
#pragma unroll
  for (int s = 0; s < 64; ++s) bf1[s] = pk[o.c1w + s * 64 + ln];
  if (threadIdx.x < 48) {  // BN2d(16), BN2d(32) folded (eval mode)
    const int c = threadIdx.x, first = c < 16;
    const int ch = first ? c : c - 16;
    const int st = first ? c : c;  // running stats: [16 | 32 | 256]
    const float rm = a.bn_mean ? a.bn_mean[st] : 0.f;
    const float rv = a.bn_var ? a.bn_var[st] : 1.f;
    const int w_off = first ? o.bn1 + ch : o.bn2 + ch;
    const int nch = first ? 16 : 32;
    const float sc = pk[w_off] * (1.f / sqrtf(rv + impala::kBnEps));
    bnt[2 * c] = sc;
    bnt[2 * c + 1] = pk[w_off + nch] - rm * sc;
  }
  if (a.frames) {  // shared_frames (strategies): every lane reads the probe frame e
    const float* fr = a.frames + (a.shared_frames ? (int64_t)e : env) * kFramePix;
    for (int p = threadIdx.x; p < kFramePix; p += kThreads) frame[p] = fr[p];
  } else {  // oracle/atari.py frames: byte (p & 7) of the counter hash of word p >> 3
    const uint64_t gid = (uint64_t)(a.lane_offset * a.envs + env);
    for (int w = threadIdx.x; w < kFramePix / 8; w += kThreads) {
      const uint64_t hb = mix64(a.fkey + ((gid << 32) | ((uint64_t)a.t << 11) | (uint64_t)w) * impala::kGolden);
#pragma unroll
      for (int j = 0; j < 8; ++j) frame[8 * w + j] = (float)((uint32_t)(hb >> (8 * j)) & 255u);
    }
  }
  __syncthreads();

  // conv1 4->16, 8x8 stride 4: 400 pixels = 25 tiles, K = 256 (64 k-steps = 64 taps x 4 channels)
  {
    f32x4 acc[4];
    conv_s<4, 1, 4, 25, 400, kO1, 4, kW, kPlane, 8, 64>(frame, bf1, acc, wave, ln);
    const int n = ln & 15;
    const float bias = pk[o.c1b + n], sc = bnt[2 * n], sh = bnt[2 * n + 1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int mt = wave + 8 * i;
      if (mt >= 25) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt * 16 + (ln >> 4) * 4 + r;
        h1[n * 400 + m] = impala::relu(fmaf(acc[i][r] + bias, sc, sh));
      }
    }
  }
  float bf2[64];
  {
    const int nt = wave & 1;
#pragma unroll
    for (int s = 0; s < 64; ++s) bf2[s] = pk[o.c2w + (s * 2 + nt) * 64 + ln];
  }
  __syncthreads();
  // conv2 16->32, 4x4 stride 2: 81 pixels = 6 tiles x 2 channel tiles, K = 256
  {
    f32x4 acc[2];
    conv_s<16, 2, 2, 6, 81, kO2, 2, kO1, 400, 4, 64>(h1, bf2, acc, wave, ln);
    const int n = (wave & 1) * 16 + (ln & 15);
    const float bias = pk[o.c2b + n], sc = bnt[2 * (16 + n)], sh = bnt[2 * (16 + n) + 1];
    float* out = a.feat + env * kFeat;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int mt = (wave + 8 * i) >> 1;
      if (mt >= 6) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt * 16 + (ln >> 4) * 4 + r;
        if (m < 81) out[n * 81 + m] = impala::relu(fmaf(acc[i][r] + bias, sc, sh));  // flatten (C,H,W)
      }
    }
  }
}

template <int E, int MODE>
__global__ __launch_bounds__(impala::kCoreThreads) void atari_core_kernel(Layout L, Args A) {
  const StepArgs& a = A.s;
  const Offsets& o = A.o;
  // xs (the conv features) -> fc partials -> BN'd hidden + logits, phases separated by barriers
  __shared__ float xs[kFeat * E];
  float* part = xs;
  float* hs = xs + 4 * kFc * E;
  float* logit = hs + kFc * E;
  static_assert((5 * kFc + impala::kMaxAct) * E <= kFeat * E, "atari core LDS aliasing");
  const int lane = blockIdx.x, j = threadIdx.x;
  // shared_frames (strategies, E = 1): block b is probe frame b % T of pack lane b / T
  const float* pk = a.pack + (int64_t)(a.shared_frames ? lane / a.T : lane) * a.pack_stride;
  const int64_t e0 = (int64_t)lane * E;
  for (int i = j; i < kFeat * E; i += impala::kCoreThreads) {
    const int e = i / kFeat, k = i - e * kFeat;
    xs[k * E + e] = a.feat[(e0 + e) * kFeat + k];
  }
  __syncthreads();
  // fc 2592 -> 256: wave wq streams rows [648 wq, 648 wq + 648) of W^T as float4
  const int c4 = j & 63, wq = j >> 6;
  float acc[4][E];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int e = 0; e < E; ++e) acc[c][e] = 0.f;
  const float4* w4 = reinterpret_cast<const float4*>(pk + o.fcw) + c4;
#pragma unroll 4
  for (int k = wq * (kFeat / 4); k < (wq + 1) * (kFeat / 4); ++k) {
    const float4 w = impala::ld_stream(w4 + (int64_t)k * (kFc / 4));
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float x = xs[k * E + e];
      acc[0][e] = fmaf(w.x, x, acc[0][e]);
      acc[1][e] = fmaf(w.y, x, acc[1][e]);
      acc[2][e] = fmaf(w.z, x, acc[2][e]);
      acc[3][e] = fmaf(w.w, x, acc[3][e]);
    }
  }
  __syncthreads();  // every read of xs is done before the partials overwrite it
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int e = 0; e < E; ++e) part[(wq * kFc + 4 * c4 + c) * E + e] = acc[c][e];
  __syncthreads();
  {  // fc bias, BatchNorm1d(256) (eval), ReLU
    const float rm = a.bn_mean ? a.bn_mean[48 + j] : 0.f;
    const float rv = a.bn_var ? a.bn_var[48 + j] : 1.f;
    const float sc = pk[o.bn3 + j] * (1.f / sqrtf(rv + impala::kBnEps));
    const float sh = pk[o.bn3 + kFc + j] - rm * sc;
    const float bj = pk[o.fcb + j];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float y = ((part[j * E + e] + part[(kFc + j) * E + e]) + part[(2 * kFc + j) * E + e]) +
                      part[(3 * kFc + j) * E + e];
      hs[j * E + e] = impala::relu(fmaf(y + bj, sc, sh));
    }
  }
  __syncthreads();
  const int NA = a.n_act;
  if (j < NA * E) {
    const int ai = j / E, e = j - ai * E;
    const float* w = pk + o.head_w + ai * kFc;
    float s = 0.f;
    for (int k = 0; k < kFc; ++k) s = fmaf(w[k], hs[k * E + e], s);
    logit[e * impala::kMaxAct + ai] = s + pk[o.head_b + ai];
  }
  __syncthreads();
  if (j < E) impala::core_finish<E, MODE>(a, logit, lane, j, MODE == impala::kRollout);
}

template <int E>
static int launch_steps(const Layout& L, const Args& A0, hipStream_t stream) {
  Args A = A0;
  const int conv_grid = (A.s.n_lanes + 7) / 8 * 8 * A.s.envs;
  for (int t = 0; t < A.s.T; ++t) {
    A.s.t = t;
    hipLaunchKernelGGL(atari_conv_kernel, dim3(conv_grid), dim3(kThreads), 0, stream, L, A);
    hipLaunchKernelGGL((atari_core_kernel<E, impala::kRollout>), dim3(A.s.n_lanes), dim3(impala::kCoreThreads), 0,
                       stream, L, A);
  }
  return check_launch("atari step kernels");
}

struct Plan {
  int64_t pack, feat, n2, total;
  int nblk;
};
static Plan plan(const Layout& L, int n_lanes, int envs) {
  Plan p{};
  int64_t off = 0;
  auto take = [&](int64_t bytes) { const int64_t at = off; off += round_up(std::max<int64_t>(bytes, 0), 256); return at; };
  p.nblk = impala::prep_blocks(L);
  p.pack = take((int64_t)n_lanes * L.pack * 4);
  p.feat = take((int64_t)n_lanes * envs * kFeat * 4);
  p.n2 = take((int64_t)n_lanes * p.nblk * 8);
  p.total = off;
  return p;
}

int64_t workspace_bytes(int n_act, int n_lanes, int envs) {
  Layout L;
  Offsets o;
  if (!make_layout(n_act, &L, &o)) return -1;
  return plan(L, n_lanes, envs).total;
}

int64_t num_params(int n_act) {
  Layout L;
  Offsets o;
  return make_layout(n_act, &L, &o) ? L.P : -1;
}

constexpr uint64_t kFrameSalt = 0x4652414D45533031ull, kRewardSalt = 0x5245574152443031ull;

int launch_rollout(int n_act, int envs, int T, uint64_t env_seed, const LanesArgs& lanes, int n_lanes, uint64_t seed,
                   int jiggle, const float* bn_mean, const float* bn_var, double* ret, double* ent, int32_t* steps,
                   double* norm2, int32_t* actions, float* probs, void* ws, int64_t ws_bytes, hipStream_t stream) {
  Layout L;
  Args A{};
  if (!make_layout(n_act, &L, &A.o)) return set_error(FDR_ERR_UNSUPPORTED, "n_act must be in 1..32");
  const Plan p = plan(L, n_lanes, envs);
  if (!ws || ws_bytes < p.total) return set_error(FDR_ERR_WORKSPACE, "atari workspace too small");
  if (n_lanes == 0) return FDR_OK;
  char* w = static_cast<char*>(ws);
  StepArgs& a = A.s;
  a.pack = reinterpret_cast<float*>(w + p.pack);
  a.pack_stride = L.pack;
  a.bn_mean = bn_mean;
  a.bn_var = bn_var;
  a.n_lanes = n_lanes;
  a.envs = envs;
  a.n_act = n_act;
  a.T = T;
  a.lane_offset = lanes.lane_offset;
  a.fkey = mix64(env_seed ^ kFrameSalt);
  a.rkey = mix64(env_seed ^ kRewardSalt);
  a.akey = mix64(seed);
  a.feat = reinterpret_cast<float*>(w + p.feat);
  a.ret = ret;
  a.ent = ent;
  a.actions = actions;
  a.probs = probs;
  a.deterministic = lanes.deterministic;
  double* n2 = reinterpret_cast<double*>(w + p.n2);
  int rc = impala::launch_prep(L, lanes, const_cast<float*>(a.pack), n2, n_lanes, stream);
  if (rc) return rc;
  const int64_t ne = (int64_t)n_lanes * envs;
  hipLaunchKernelGGL(impala::init_kernel, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, stream, ne,
                     (float*)nullptr, (float*)nullptr, (float*)nullptr, ret, ent);
  switch (envs) {
    case 1: rc = launch_steps<1>(L, A, stream); break;
    case 2: rc = launch_steps<2>(L, A, stream); break;
    case 4: rc = launch_steps<4>(L, A, stream); break;
    default: return set_error(FDR_ERR_UNSUPPORTED, "envs_per_lane must be 1, 2 or 4");
  }
  if (rc) return rc;
  const int64_t nmax = std::max<int64_t>(ne, n_lanes);
  hipLaunchKernelGGL(impala::finish_kernel, dim3((unsigned)((nmax + 255) / 256)), dim3(256), 0, stream, n_lanes, envs,
                     T, 1, jiggle, a.akey, lanes.lane_offset, n2, p.nblk, ret, ent, steps, norm2);
  return check_launch("atari finish");
}

int64_t forward_workspace_bytes(int n_act, int n) {
  Layout L;
  Offsets o;
  if (!make_layout(n_act, &L, &o)) return -1;
  return plan(L, 1, n).total;
}

int launch_forward(int n_act, const float* theta, int n, const float* frames, const float* bn_mean,
                   const float* bn_var, float* probs, float* feat, void* ws, int64_t ws_bytes, hipStream_t stream) {
  Layout L;
  Args A{};
  if (!make_layout(n_act, &L, &A.o)) return set_error(FDR_ERR_UNSUPPORTED, "n_act must be in 1..32");
  const Plan p = plan(L, 1, n);
  if (!ws || ws_bytes < p.total) return set_error(FDR_ERR_WORKSPACE, "atari forward workspace too small");
  if (n == 0) return FDR_OK;
  char* w = static_cast<char*>(ws);
  LanesArgs lanes{};
  lanes.base = theta;
  StepArgs& a = A.s;
  a.pack = reinterpret_cast<float*>(w + p.pack);
  a.pack_stride = 0;
  a.bn_mean = bn_mean;
  a.bn_var = bn_var;
  a.n_lanes = n;
  a.envs = 1;
  a.n_act = n_act;
  a.frames = frames;
  a.feat = feat ? feat : reinterpret_cast<float*>(w + p.feat);
  a.probs = probs;
  int rc = impala::launch_prep(L, lanes, const_cast<float*>(a.pack), reinterpret_cast<double*>(w + p.n2), 1, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(atari_conv_kernel, dim3((n + 7) / 8 * 8), dim3(kThreads), 0, stream, L, A);
  hipLaunchKernelGGL((atari_core_kernel<1, impala::kForward>), dim3(n), dim3(impala::kCoreThreads), 0, stream, L, A);
  return check_launch("atari forward");
}

// AtariPolicy.get_strategy of every lane's theta'_l over Z shared probe frames (policies/atari.py:30-31, the lane
// novelty of worker.py:53 / strategy_handler.py:25-30): chunks of kStratLanes lanes, each chunk ONE prep, ONE conv
// launch over (lane, frame) and ONE core launch -- the per-lane forwards of the host loop, batched.
constexpr int kStratLanes = 256;

int64_t strategies_workspace_bytes(int n_act, int n_lanes, int Z) {
  Layout L;
  Offsets o;
  if (!make_layout(n_act, &L, &o) || n_lanes < 0 || Z < 0) return -1;
  const int c = std::min(n_lanes, kStratLanes);
  return plan(L, c, Z).total;
}

int launch_strategies(int n_act, const LanesArgs& lanes, int n_lanes, int Z, const float* frames, const float* bn_mean,
                      const float* bn_var, float* probs, void* ws, int64_t ws_bytes, hipStream_t stream) {
  Layout L;
  Args A{};
  if (!make_layout(n_act, &L, &A.o)) return set_error(FDR_ERR_UNSUPPORTED, "n_act must be in 1..32");
  const int chunk = std::min(n_lanes, kStratLanes);
  const Plan p = plan(L, chunk, Z);
  if (!ws || ws_bytes < p.total) return set_error(FDR_ERR_WORKSPACE, "atari strategies workspace too small");
  if (n_lanes == 0 || Z == 0) return FDR_OK;
  char* w = static_cast<char*>(ws);
  StepArgs& a = A.s;
  a.pack = reinterpret_cast<float*>(w + p.pack);
  a.pack_stride = L.pack;
  a.bn_mean = bn_mean;
  a.bn_var = bn_var;
  a.envs = Z;
  a.T = Z;
  a.n_act = n_act;
  a.frames = frames;
  a.shared_frames = 1;
  a.feat = reinterpret_cast<float*>(w + p.feat);
  double* n2 = reinterpret_cast<double*>(w + p.n2);
  for (int l0 = 0; l0 < n_lanes; l0 += chunk) {
    const int nl = std::min(chunk, n_lanes - l0);
    LanesArgs la = lanes;
    la.base = lanes.base + (int64_t)l0 * lanes.base_stride;
    if (la.idx) la.idx += l0;
    if (la.sign) la.sign += l0;
    if (la.deterministic) la.deterministic += l0;
    la.lane_offset += l0;
    int rc = impala::launch_prep(L, la, const_cast<float*>(a.pack), n2, nl, stream);
    if (rc) return rc;
    a.n_lanes = nl;
    a.probs = probs + (int64_t)l0 * Z * n_act;
    hipLaunchKernelGGL(atari_conv_kernel, dim3((nl + 7) / 8 * 8 * Z), dim3(kThreads), 0, stream, L, A);
    hipLaunchKernelGGL((atari_core_kernel<1, impala::kForward>), dim3(nl * Z), dim3(impala::kCoreThreads), 0, stream,
                       L, A);
  }
  return check_launch("atari strategies");
}

// The env's frames at steps t0 .. t0 + n - 1 of global env env_id (the atari_conv_kernel hash; they do not depend
// on the actions): one workgroup per step, 8 pixels (one hash word) per thread and iteration, two float4 stores.
__global__ __launch_bounds__(256) void env_frames_kernel(uint64_t fkey, uint64_t env_id, int t0, float* frames) {
  const int t = t0 + blockIdx.x;
  float4* fr = reinterpret_cast<float4*>(frames + (int64_t)blockIdx.x * kFramePix);
  for (int w = threadIdx.x; w < kFramePix / 8; w += 256) {
    const uint64_t hb = mix64(fkey + ((env_id << 32) | ((uint64_t)t << 11) | (uint64_t)w) * impala::kGolden);
    const uint32_t lo = (uint32_t)hb, hi = (uint32_t)(hb >> 32);
    fr[2 * w] = float4{(float)(lo & 255u), (float)((lo >> 8) & 255u), (float)((lo >> 16) & 255u), (float)(lo >> 24)};
    fr[2 * w + 1] = float4{(float)(hi & 255u), (float)((hi >> 8) & 255u), (float)((hi >> 16) & 255u), (float)(hi >> 24)};
  }
}

int launch_env_frames(uint64_t env_seed, uint64_t env_id, int t0, int n, float* frames, hipStream_t stream) {
  static_assert(kFramePix % 8 == 0, "whole hash words per frame");
  if (n == 0) return FDR_OK;
  hipLaunchKernelGGL(env_frames_kernel, dim3(n), dim3(256), 0, stream, mix64(env_seed ^ kFrameSalt), env_id, t0, frames);
  return check_launch("atari env_frames_kernel");
}

}  // namespace atari
}  // namespace fdr
