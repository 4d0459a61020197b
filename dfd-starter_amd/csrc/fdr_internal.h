// Internal (non-ABI) declarations shared by the fdr translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fdr_common.h"

namespace fdr {

int set_error(int code, const char* msg);
int check_launch(const char* what);

// Per-device engine state behind an fdr_ctx (include/fdr.h): the settings that were process-wide
// globals before (rollout kernel selection, Impala phase profiling, replay GEMM switch, debug clocks).
// A NULL ctx at the ABI means default_context(), the process-wide one (FDR_ROLLOUT read at first use).
namespace impala {
struct Profile;
}
struct Context {
  int device = -1;      // -1: any (the default context follows the current device)
  int cus = 0;          // compute units of `device` (0: query the current device)
  int rollout_impl = 2; // FDR_ROLLOUT_AUTO
  int replay_gemm = 1;
  uint64_t* debug_clock = nullptr;
  impala::Profile* prof = nullptr;  // owned, created on first enable
};
Context& default_context();
int context_cus(const Context& c);

struct PolicyKey {
  int n_in, n_act;
  bool discrete;
  int64_t n_params;
};

// Device-side view of fdr_lanes_desc (passed by value as a kernel argument).
struct LanesArgs {
  const float* base;
  int64_t base_stride;
  const float* table;
  int64_t max_idx;  // table_size - n_params: largest legal offset
  const int64_t* idx;
  const int8_t* sign;
  float sigma;
  const int8_t* deterministic;
  int64_t lane_offset;

  // A lane whose table offset is out of range is never dereferenced: it runs unperturbed and
  // reports norm2 = NaN, which poisons the FD step visibly instead of faulting the GPU.
  __device__ __forceinline__ ParamSrc src(int lane) const {
    ParamSrc s;
    s.base = base + (int64_t)lane * base_stride;
    s.sigma = sigma;
    s.n2 = 0.0;
    s.sgn = 0;
    s.eps = s.base;  // unperturbed: a readable address whose value ParamSrc discards
    if (table != nullptr) {
      const int64_t off = idx[lane];
      const int sg = sign ? (int)sign[lane] : 1;
      if (off < 0 || off > max_idx) {
        s.n2 = __builtin_nan("");
      } else if (sg != 0) {
        s.sgn = sg > 0 ? 1 : -1;
        s.eps = table + off;
      }
    }
    return s;
  }
};

struct RolloutArgs {
  LanesArgs lanes;
  int n_lanes;
  int lane_base;  // first lane of this launch (rollout_pair_kernel launches lanes in rounds, launch_pair)
  int T;
  uint64_t key;
  int jiggle;
  const float* bn_mean;
  const float* bn_var;
  const float* obs_mean;
  const float* obs_std;
  // synthetic env
  const float* M;
  const float* K;
  const float* s0;
  float done_thr;  // > 0: terminating env, done when |s'[done_dim]| > done_thr (fdr_env_desc.done_threshold)
  int done_dim;
  // trap env
  const uint8_t* walkable;
  int map_w, map_h, trap_start_col, trap_start_row;
  // outputs
  double* ret;
  double* ent;
  int32_t* steps;
  double* norm2;
  float* states;  // NULL, or [n_lanes, T, n_in] visited raw observations (fdr_rollout_states)
  // NULL, or per-lane Welford obs statistics (fdr_rollout_obs_stats)
  float* os_mean;
  float* os_m2;
  int32_t* os_count;
  float os_chance;
  // NULL, or [n_lanes, T, k] host-injected draws replacing the counter stream (fdr_rollout_extras.u_inject)
  const float* u_inject;
};

int launch_policy_forward(const PolicyKey& k, const LanesArgs& lanes, int n_lanes,
                          const float* bn_mean, const float* bn_var, const float* x, float* out0,
                          float* out1, hipStream_t stream);
int launch_rollout(const Context& ctx, const PolicyKey& k, int env_kind, const RolloutArgs& args, hipStream_t stream);

// Delayed-return perturbation rows (fdr_fd_lambda_norms / fdr_fd_grad_lambda), by value to kernels.
int64_t bn_refresh_workspace_bytes(int n);
int launch_bn_refresh(int n_in, const float* theta, const float* x, int n, float momentum, float* rm, float* rv,
                      void* ws, int64_t ws_bytes, hipStream_t stream);

struct LambdaRow {
  const float* table;
  int64_t max_idx;
  const int64_t* idx;
  const int8_t* sign;
  const int32_t* slot;
  const float* drift;
  int n_slots;
  int64_t P;
  float sigma;

  // pointer to eps_i (row 0 if the offset is out of range: the caller poisons that row with NaN)
  __device__ __forceinline__ const float* eps(int i, bool& bad) const {
    const int64_t off = idx[i];
    bad = off < 0 || off > max_idx;
    return table + (bad ? 0 : off);
  }
  __device__ __forceinline__ const float* dr(int i) const {
    const int s = slot ? slot[i] : -1;
    return (s >= 0 && s < n_slots) ? drift + (int64_t)s * P : nullptr;
  }
  __device__ __forceinline__ float value(const float* e, const float* d, int sg, int64_t p) const {
#pragma clang fp contract(off)
    float v = sigma * e[p];
    v = sg < 0 ? -v : v;
    return d ? v + d[p] : v;
  }
};
int launch_lambda_norms(const LambdaRow& R, int n, double* n2, hipStream_t stream);
int launch_lambda_grad(const LambdaRow& R, const double* coef, int n, double* g, void* ws, int64_t ws_bytes,
                       hipStream_t stream);
int launch_obs_stats_merge(const float* mean, const float* m2, const int32_t* count, int n, int d, float* acc_mean,
                           float* acc_m2, int64_t* acc_count, hipStream_t stream);

}  // namespace fdr
