// Internal (non-ABI) declarations of the ImpalaPolicy path (fdr_impala.hip).
#pragma once
#include <cfloat>

#include "fdr_internal.h"

namespace fdr {
namespace impala {

constexpr int kConvs = 15;   // 3 stages x (entry conv + 2 residual blocks x 2 convs)
constexpr int kBns = 17;     // the 15 BatchNorm2d in front of them + fc BN1d + head BN1d
constexpr int kFeat = 2048;  // 32 x 8 x 8 (policies/impala.py:113)
constexpr int kHid = 256;    // fc width == LSTM hidden
constexpr int kGates = 1024;
constexpr int kCoreIn = 257; // fc output + clipped reward (policies/impala.py:116, 163-164)
#define FDR_CORE_UNROLL 4    // weight-stream loop unroll of the core kernels (loads in flight per thread)
#define FDR_CORE_UNROLL_H 2  // fp16 step kernel's fc / gate streams (A/B: 0.377 -> 0.360 ms per step vs 4)
// fp16 pair-form core step on MFMA (core_kernel_hpm2): fc W^T and [W_ih | W_hh]^T as v_mfma_f32_16x16x32_f16
// A-fragment images [k-step][16-column tile][64 lanes][8 halves] (lane l: W[16 nt + (l & 15)][32 ks + 8 (l >> 4) ..
// + 7]), one for theta and one per pair for sigma-eps; K of the gates (513) zero-padded to 17 k-steps.
constexpr int kFcKS = kFeat / 32, kFcNT = kHid / 16;
constexpr int kGateK = kCoreIn + kHid, kGateKS = (kGateK + 31) / 32, kGateNT = kGates / 16;
constexpr int64_t kFcImg = (int64_t)kFcKS * kFcNT * 512;      // halves
constexpr int64_t kGateImg = (int64_t)kGateKS * kGateNT * 512;
constexpr int64_t kMImg = kFcImg + kGateImg;                    // halves per image (2.2 MB)
constexpr int kReplayChunk = 64;  // entropy replay: steps per batched input-projection GEMM
constexpr int kMaxAct = 32;
constexpr int kMaxSections = 64;
constexpr int kFramePix = 3 * 64 * 64;

// One contiguous run of the per-lane parameter pack: pack[dst + u] = theta'[src + f(u)].
enum SectionKind : int32_t { kCopy = 0, kConvFrag = 1, kTranspose = 2, kConvFragH = 3 };
struct Section {
  int32_t dst, len, src, kind, a, b;  // conv frag: a = Cin, b = Cout; transpose: a = rows, b = cols of W
};

// Per-lane parameter pack: theta' gathered ONCE per rollout into the order the kernels read
// (conv weights as MFMA B-fragments, fc / LSTM weights transposed for coalesced row streaming).
struct Layout {
  int32_t n_act;
  int32_t n_sections;
  int64_t P;     // reference parameter count (policies/impala.py)
  int64_t pack;  // floats per lane (multiple of 64)
  int32_t conv_w[kConvs], conv_b[kConvs];
  int32_t bn_w[kBns], bn_b[kBns], bn_stat[kBns];
  int32_t fc_wt, fc_b, lstm_wt, lstm_bih, lstm_bhh, head_w, head_b;
  int32_t n_bn_stats;
  Section sec[kMaxSections];
  // fp16 mode (BASELINE config 5): a second, half-precision pack of the MFMA/streamed weights
  int64_t hpack;                  // halves per lane (multiple of 64)
  int32_t conv_h[kConvs];         // f16 MFMA A-fragments of each conv (v_mfma_f32_16x16x32_f16)
  int32_t fc_wt_h, lstm_wt_h;     // W^T of fc / [W_ih | W_hh] in f16
  int32_t n_hsections;
  Section hsec[24];
};

bool make_layout(int n_act, Layout* out);

struct StepArgs {
  const float* pack;
  int64_t pack_stride;  // floats between lanes' packs (0: every lane shares one pack)
  _Float16* hpack;      // fp16 mode: half pack (conv A-fragments, fc / LSTM W^T), or NULL
  int64_t hpack_stride;
  const float* bn_mean;
  const float* bn_var;
  int n_lanes, envs, n_act, t, T;
  int64_t lane_offset;
  uint64_t fkey, rkey, akey;
  const float* frames;     // external frames [lane*E+e][3][64][64] (forward API) or NULL
  int shared_frames;       // 1: every lane reads frames [e][3][64][64] (strategy probe set zeta)
  float* feat;             // [lane*E+e][2048]
  // core
  float* h;
  float* c;
  float* rprev;
  float* ci;               // [t][lane*E+e][257] (entropy replay) or NULL
  const float* gx;         // replay: x W_ih^T of steps [gx_t0, gx_t0 + kReplayChunk), [t - gx_t0][lane*E+e][1024], or NULL
  int gx_t0;
  double* ret;
  double* ent;
  int32_t* actions;        // [lane*E+e][T] or NULL
  float* probs;            // rollout: [lane*E+e][T][A]; forward: [lane*E+e][A]; or NULL
  const int8_t* deterministic;
  const float* reward_in;  // forward: reward carried by the obs
  const float* notdone;    // forward: done mask (policies/impala.py:170-176)
  uint64_t* dbg;           // diagnostics: phase clocks of conv workgroup 0 (fdr_impala_debug_clock) or NULL
  // pair form of the rollout core step (fdr_impala_desc.pairs): theta's (half) pack, the pairs' sigma-eps
  // (half) packs [n_lanes / 2][stride], the lanes' signs -- f16 operands in fp16 mode, f32 otherwise
  const _Float16* th;
  const _Float16* ep;
  const float* th32;
  const float* ep32;
  int64_t ep_stride;
  const int8_t* sign;
  // MFMA form (fp16 pairs): theta's image and the pairs' sigma-eps images [n_lanes / 2][kMImg]
  const _Float16* thm;
  const _Float16* epm;
  // fp16 conv: the lanes' folded BN / bias tables [lane][3][kBnTab] (scale | shift | conv bias), built once per rollout
  // by bn_table_kernel -- constant over the episode -- or NULL (each conv workgroup folds them itself)
  const float* bntab;
  // fp16 MFMA pair rollout with the replay GEMM: the core inputs as f16 rows of kCiPitch halves (zero beyond
  // kCoreIn) -- xproj_pair_kernel's B operand, rounded as it would round the f32 rows -- in place of ci, or NULL
  _Float16* ci16;
};
constexpr int kCiPitch = (kCoreIn + 31) / 32 * 32;

// phase clock of the first conv workgroup (s_memtime), for the phase breakdown in DESIGN.md -- a diagnostics build
// only (make STAMPS=1 -> -DFDR_CONV_STAMPS; tools/impala_phases_h2.py).  In the product the stamps compile away: even
// runtime-gated, each conditional store was a control-flow join at which the waitcnt pass drained every load in flight
// (vmcnt(0), CDNA4 counts stores too), including the next conv's weight-block prefetch.
#ifdef FDR_CONV_STAMPS
#define FDR_STAMP(a, k)                                                      \
  do {                                                                       \
    if ((a).dbg && blockIdx.x == 0 && threadIdx.x == 0) (a).dbg[k] = clock64(); \
  } while (0)
#else
#define FDR_STAMP(a, k) \
  do {                  \
  } while (0)
#endif

constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;
constexpr float kBnEps = 1e-5f;
// kStrategy: the replay's sequence form over a probe set (get_strategy), probabilities out
enum CoreMode { kRollout = 0, kReplay = 1, kForward = 2, kStrategy = 3 };
constexpr bool seq_mode(int m) { return m == kReplay || m == kStrategy; }
constexpr int kCoreThreads = 256;
constexpr int kBnTab = 15 * 32;

__device__ __forceinline__ float relu(float v) { return v > 0.f ? v : 0.f; }

// Streamed weights of the core kernels: each lane's W^T is read once per step and evicted before the
// next step needs it (GBs per step), so the loads are non-temporal (measured: f32 core 0.75 -> 0.68 ms,
// f16 0.41 -> 0.38 ms per step at 1024 lanes x 4 envs).
template <class T>
__device__ __forceinline__ T ld_stream(const T* p) {
  static_assert(sizeof(T) == 16 || sizeof(T) == 8, "8- or 16-byte streamed loads");
  typedef float fv __attribute__((ext_vector_type(sizeof(T) / 4)));
  const fv v = __builtin_nontemporal_load(reinterpret_cast<const fv*>(p));
  return __builtin_bit_cast(T, v);
}
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// Softmax, action (argmax / inverse CDF on the counter stream), synthetic reward and return, or the
// entropy term (replay), or the probabilities (forward), for env e of lane `lane` (thread e < E).
// ent_acc (kReplay, optional): accumulate the step's entropy into this register instead of a.ent (a kernel that runs
// many replay steps stores it once)
// t_step >= 0: the step in place of a.t (a kernel that runs many steps)
template <int E, int MODE>
__device__ __forceinline__ void core_finish(const StepArgs& a, const float* logit, int lane, int j,
                                            bool step_entropy = false, double* ent_acc = nullptr, int t_step = -1) {
  const int at_t = t_step >= 0 ? t_step : a.t;
  const int A = a.n_act;
  const int64_t e0 = (int64_t)lane * E;
    const int e = j;
    const float* lg = logit + e * kMaxAct;
    float mx = -FLT_MAX;
    for (int i = 0; i < A; ++i) mx = fmaxf(mx, lg[i]);
    float p[kMaxAct];
    float sum = 0.f;
    for (int i = 0; i < A; ++i) {
      p[i] = expf(lg[i] - mx);
      sum += p[i];
    }
    const float inv = 1.f / sum;
    for (int i = 0; i < A; ++i) p[i] *= inv;
    const int64_t ge = e0 + e;
    if constexpr (MODE == kForward) {
      if (a.probs)
        for (int i = 0; i < A; ++i) a.probs[ge * A + i] = p[i];
    } else if constexpr (MODE == kStrategy) {
      for (int i = 0; i < A; ++i) a.probs[(ge * a.T + at_t) * A + i] = p[i];
    } else if constexpr (MODE == kReplay) {
      // torch Categorical(probs).entropy(): normalise, log clamped at float min
      float tot = 0.f;
      for (int i = 0; i < A; ++i) tot += p[i];
      float h = 0.f;
      for (int i = 0; i < A; ++i) {
        const float pn = p[i] / tot;
        const float l = pn > 0.f ? logf(pn) : -FLT_MAX;
        h -= pn * l;
      }
      if (ent_acc)
        *ent_acc += (double)h;
      else
        a.ent[ge] += (double)h;
    } else {
      if (a.probs)
        for (int i = 0; i < A; ++i) a.probs[(ge * a.T + a.t) * A + i] = p[i];
      const uint64_t gid = (uint64_t)(a.lane_offset * E + ge);
      int act = 0;
      const bool det = a.deterministic && a.deterministic[lane];
      if (det) {
        float best = p[0];
        for (int i = 1; i < A; ++i)
          if (p[i] > best) { best = p[i]; act = i; }
      } else {  // inverse CDF, sequential f32 cumsum (oracle/policies.py categorical_inverse_cdf)
        float tot = 0.f;
        for (int i = 0; i < A; ++i) tot += p[i];
        const float u = uniform24(hash_ctr(a.akey, gid, (uint64_t)a.t, 0));
        const float target = u * tot;
        float cs = 0.f;
        for (int i = 0; i < A - 1; ++i) {
          cs += p[i];
          act += cs <= target ? 1 : 0;
        }
      }
      const uint64_t ctr = (gid << 32) | ((uint64_t)a.t << 11);
      const int tgt = (int)((mix64(a.rkey + ctr * kGolden) >> 40) % (uint64_t)A);
      const float r = act == tgt ? 1.f : (act == (tgt + 1) % A ? -1.f : 0.f);
      a.ret[ge] += (double)r;
      if (a.rprev) a.rprev[ge] = r;
      if (a.actions) a.actions[ge * a.T + a.t] = act;
      if (step_entropy) {  // stateless policies: the mean per-step entropy equals the batched one
        float tot = 0.f;
        for (int i = 0; i < A; ++i) tot += p[i];
        float hh = 0.f;
        for (int i = 0; i < A; ++i) {
          const float pn = p[i] / tot;
          const float l = pn > 0.f ? logf(pn) : -FLT_MAX;
          hh -= pn * l;
        }
        a.ent[ge] += (double)hh;
      }
    }
}

// shared launch helpers of the pack-based policies (defined in fdr_impala.hip)
int launch_prep(const Layout& L, const LanesArgs& lanes, float* pack, double* n2_part, int n_lanes,
                hipStream_t stream);
int prep_blocks(const Layout& L);
__global__ void init_kernel(int64_t n_env, float* h, float* c, float* rprev, double* ret, double* ent);
__global__ void finish_kernel(int n_lanes, int envs, int T, int entropy, int jiggle, uint64_t akey,
                              int64_t lane_offset, const double* n2_part, int nblk, double* ret,
                              double* ent, int32_t* steps, double* norm2);

// the fp16 conv stack's folded BN / bias tables of n lanes (one workgroup per lane): tab [lane][3 * kBnTab]
__global__ void bn_table_kernel(Layout L, StepArgs a, float* tab);
// fp16 mode kernels (fdr_impala_h.hip)
// the conv stack: one env per 8-wave workgroup (kHThreads), 80 KiB LDS, <= 128 VGPRs -- two workgroups per CU
template <int NTH>
__global__ void conv_kernel_h2(Layout L, StepArgs a);
template <int E, int MODE>
__global__ void core_kernel_h(Layout L, StepArgs a);   // per-lane form (non-pair batches, forward)
template <int E>
__global__ void core_kernel_p(Layout L, StepArgs a);   // f32 pair form (rollout mode, bit-exact), grid n_lanes / 2
template <int E>
__global__ void core_kernel_pr(Layout L, StepArgs a);  // f32 pair form of the replay (with a.gx)
// fp16 pair form on MFMA: theta x + s (E x) over fragment images, two antithetic pairs per workgroup (512 threads),
// grid n_lanes / 4 (n_lanes % 4 == 0)
template <int E, int MODE>
__global__ void core_kernel_hpm2(Layout L, StepArgs a);
// replay input projection of a chunk in the fp16 pair form on MFMA: grid xproj_grid(n_lanes) (XCD-aware, 1-D);
// H16: the core inputs from a.ci16 (the rollout), else from the f32 rows a.ci (lane strategies)
template <int E, bool H16>
__global__ void xproj_pair_kernel(Layout L, StepArgs a, int t0, int tc, float* gx);
inline dim3 xproj_grid(int n_lanes) { return dim3((unsigned)(((n_lanes / 2 + 7) / 8) * 8 * (kGateNT / 4))); }
// the entropy replay of one chunk (steps t0 .. t0 + tc - 1 on a.gx) in ONE launch: the W_hh step of the pair form
// for two pairs per workgroup in a loop, h / c / ent in registers, the next step's first W_hh fragments in flight
// under each epilogue
template <int E, int MODE>  // kReplay (entropy sums) or kStrategy (probabilities over a probe sequence)
__global__ void replay_chunk_hpm2(Layout L, StepArgs a, int t0, int tc);
// MFMA images (kMImg halves each) of n half packs: grid (kFcKS + 4 kGateKS, n)
__global__ void mfma_image_kernel(Layout L, const _Float16* src, int64_t src_stride, _Float16* dst);
constexpr int kHThreads = 512;

struct Plan {  // workspace carve-up (byte offsets)
  int64_t pack, hpack, feat, h, c, rprev, ci, gx, n2, zeros, thpack, epack, idxe, n2x, mimg, bntab, total;
  int nblk;    // prep blocks per lane
};
// pairs: the fp16 pair form (theta half pack, one sigma-eps half pack per pair, a zero base, pair offsets)
Plan plan(const Layout& L, int n_lanes, int envs, int T, bool entropy, bool fp16 = false, bool pairs = false);
bool pair_core_supported(int envs);

struct RolloutCall {
  const Context* ctx;
  const Layout* layout;
  LanesArgs lanes;
  int n_lanes, envs, T, entropy, jiggle, fp16, pairs;
  uint64_t seed, env_seed;
  const float* bn_mean;
  const float* bn_var;
  double* ret;
  double* ent;
  int32_t* steps;
  double* norm2;
  int32_t* actions;
  float* probs;
};
int launch_rollout(const RolloutCall& c, void* ws, int64_t ws_bytes, hipStream_t stream);

struct ForwardCall {
  const Layout* layout;
  int fp16;
  const float* theta;
  int n_envs;
  const float* frames;
  const float* reward;
  const float* notdone;
  float* h;
  float* c;
  float* probs;
  float* feat_out;
  const float* bn_mean;
  const float* bn_var;
};
int64_t forward_workspace_bytes(const Layout& L, int n_envs, bool fp16 = false);

// get_strategy over a probe set (policies/impala.py:24-27): Z shared frames, one LSTM sequence per lane
struct StrategiesCall {
  const Layout* layout;
  LanesArgs lanes;
  int n_lanes, n_states, fp16;
  int pairs;             // fdr_impala_desc.pairs: fp16 + n_lanes % 4 == 0 -> the pair form on MFMA
  const float* frames;   // [Z][3][64][64] f32 0..255
  const float* reward;   // [Z] or NULL
  float* h;              // [n_lanes][256] in/out initial state, or NULL (zero state)
  float* c;
  float* probs;          // [n_lanes][Z][A]
  const float* bn_mean;
  const float* bn_var;
};
int64_t strategies_workspace_bytes(const Layout& L, int n_lanes, int n_states, bool fp16, bool pairs = false);
int launch_strategies(const StrategiesCall& c, void* ws, int64_t ws_bytes, hipStream_t stream);
int launch_env_frames(uint64_t env_seed, int n_act, uint64_t env_id, int t0, int n, const int32_t* actions,
                      float* frames, float* reward, hipStream_t stream);
int set_profile(Context& ctx, int on);
int read_profile(Context& ctx, double* out3);
void destroy_profile(Profile* p);
int launch_forward(const ForwardCall& c, void* ws, int64_t ws_bytes, hipStream_t stream);

// ImpalaPolicy.compute_vbn (policies/impala.py:12-16): train-mode pass of an n-obs buffer (fdr_impala_vbn.hip)
struct VbnCall {
  const Layout* layout;
  const float* theta;
  int n;
  const float* frames;   // [n][3][64][64] f32 0..255
  const float* reward;   // [n] or NULL
  int first_done;        // the first obs' done flag: zero the carried state
  float* h;              // [256] in/out carried LSTM state, or NULL (zero, not written)
  float* c;
  float momentum;
  float* bn_mean;        // [fdr_impala_num_bn_stats] running stats, updated in place
  float* bn_var;
};
int64_t vbn_workspace_bytes(int n);
int launch_vbn(const VbnCall& c, void* ws, int64_t ws_bytes, hipStream_t stream);

}  // namespace impala
}  // namespace fdr
