// Internal (non-ABI) declarations of the ImpalaPolicy path (fdr_impala.hip).
#pragma once
#include "fdr_internal.h"

namespace fdr {
namespace impala {

constexpr int kConvs = 15;   // 3 stages x (entry conv + 2 residual blocks x 2 convs)
constexpr int kBns = 17;     // the 15 BatchNorm2d in front of them + fc BN1d + head BN1d
constexpr int kFeat = 2048;  // 32 x 8 x 8 (policies/impala.py:113)
constexpr int kHid = 256;    // fc width == LSTM hidden
constexpr int kGates = 1024;
constexpr int kCoreIn = 257; // fc output + clipped reward (policies/impala.py:116, 163-164)
constexpr int kMaxAct = 32;
constexpr int kMaxSections = 64;
constexpr int kFramePix = 3 * 64 * 64;

// One contiguous run of the per-lane parameter pack: pack[dst + u] = theta'[src + f(u)].
enum SectionKind : int32_t { kCopy = 0, kConvFrag = 1, kTranspose = 2 };
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
};

bool make_layout(int n_act, Layout* out);

struct Plan {  // workspace carve-up (byte offsets)
  int64_t pack, feat, h, c, rprev, ci, n2, total;
  int nblk;    // prep blocks per lane
};
Plan plan(const Layout& L, int n_lanes, int envs, int T, bool entropy);

struct RolloutCall {
  const Layout* layout;
  LanesArgs lanes;
  int n_lanes, envs, T, entropy, jiggle;
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
int64_t forward_workspace_bytes(const Layout& L, int n_envs);
void set_profile(int on);
void set_debug_clock(uint64_t* buf);
int read_profile(double* out3);
int launch_forward(const ForwardCall& c, void* ws, int64_t ws_bytes, hipStream_t stream);

}  // namespace impala
}  // namespace fdr
