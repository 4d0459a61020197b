// fdr_api.hip -- the extern "C" boundary (include/fdr.h): argument validation, error state,
// descriptor translation, kernel dispatch.  No allocation, no host sync, no copies.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/fdr_diag.h"
#include "fdr_impala.h"
#include "fdr_internal.h"

namespace fdr {
namespace atari {
int64_t num_params(int n_act);
int64_t workspace_bytes(int n_act, int n_lanes, int envs);
int64_t forward_workspace_bytes(int n_act, int n);
int launch_rollout(int n_act, int envs, int T, uint64_t env_seed, const LanesArgs& lanes, int n_lanes, uint64_t seed,
                   int jiggle, const float* bn_mean, const float* bn_var, double* ret, double* ent, int32_t* steps,
                   double* norm2, int32_t* actions, float* probs, void* ws, int64_t ws_bytes, hipStream_t stream);
int launch_forward(int n_act, const float* theta, int n, const float* frames, const float* bn_mean,
                   const float* bn_var, float* probs, float* feat, void* ws, int64_t ws_bytes, hipStream_t stream);
int launch_env_frames(uint64_t env_seed, uint64_t env_id, int t0, int n, float* frames, hipStream_t stream);
int64_t strategies_workspace_bytes(int n_act, int n_lanes, int Z);
int launch_strategies(int n_act, const LanesArgs& lanes, int n_lanes, int Z, const float* frames, const float* bn_mean,
                      const float* bn_var, float* probs, void* ws, int64_t ws_bytes, hipStream_t stream);
int64_t vbn_workspace_bytes(int n);  // (fdr_impala_vbn.hip)
int launch_vbn(const float* theta, int n, const float* frames, float momentum, float* bn_mean, float* bn_var, void* ws,
               int64_t ws_bytes, hipStream_t stream);
}  // namespace atari
}  // namespace fdr

namespace fdr {

static thread_local std::string g_err;

int set_error(int code, const char* msg) {
  g_err = msg ? msg : "";
  return code;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return FDR_ERR_HIP;
  }
  return FDR_OK;
}

int launch_perturb(const float* theta, int64_t P, const float* table, int64_t table_size,
                   const int64_t* idx, const int8_t* sign, int n, float sigma, float* out,
                   hipStream_t stream);
int launch_fd_weights(const double* r_all, int n_all, double pr, int lo, int n_local,
                      const int8_t* sign, const double* n2, int lpd, float sigma, double* coef,
                      hipStream_t stream);
int64_t grad_workspace_bytes(int n_dirs, int64_t P);
int launch_fd_grad(const float* table, int64_t table_size, const int64_t* idx, const double* coef,
                   int n_dirs, int64_t P, double* g, void* ws, int64_t ws_bytes, hipStream_t stream);
int64_t dsgd_workspace_bytes(int64_t P);
int launch_strategy_dist(const float* S, int n, const float* B, int H, int Z, int D, int kind, double* dists,
                         double* min_d, int32_t* arg, hipStream_t stream);
int launch_dsgd(float* theta, const double* g, int64_t P, double lr, double lr_scale, double* out,
                void* ws, int64_t ws_bytes, hipStream_t stream);
int launch_dsgd_ex(float* theta, const double* src, int mom, int64_t P, double lr, double lr_scale, double* g_out,
                   double* out, void* ws, int64_t ws_bytes, hipStream_t stream);
int64_t fused_workspace_bytes(int n_dirs, int n_local, int64_t P, int mode);
int64_t fused_counter_bytes(int n_dirs, int64_t P);
int launch_fd_grad_fused(const float* table, int64_t table_size, const int64_t* idx, int n_dirs, int64_t P,
                         const double* r_all, int n_all, double pr, int lo, const int8_t* sign, const double* n2,
                         int lpd, float sigma, int mode, double* out, float* theta, double lr, double lr_scale,
                         float* hist, double* dsgd_out, void* ws, int64_t ws_bytes, hipStream_t stream);
int launch_rank_weights(const double* r_all, int n_all, int lo, int n_local, double* w, hipStream_t stream);

static int policy_key(const fdr_policy_desc* p, PolicyKey* k) {
  if (!p) return set_error(FDR_ERR_INVALID, "policy desc is NULL");
  if (p->hidden != kHidden) return set_error(FDR_ERR_UNSUPPORTED, "hidden width must be 64");
  if (p->kind != FDR_POLICY_DISCRETE && p->kind != FDR_POLICY_MUJOCO)
    return set_error(FDR_ERR_INVALID, "unknown policy kind");
  k->n_in = p->n_in;
  k->n_act = p->n_act;
  k->discrete = p->kind == FDR_POLICY_DISCRETE;
  k->n_params = p->n_params;
  return FDR_OK;
}

static int lanes_args(const fdr_lanes_desc* l, int n_lanes, int64_t P, LanesArgs* out) {
  if (!l || !l->base) return set_error(FDR_ERR_INVALID, "lanes desc / base is NULL");
  if (n_lanes < 0) return set_error(FDR_ERR_INVALID, "n_lanes < 0");
  if (l->table) {
    if (!l->idx) return set_error(FDR_ERR_INVALID, "table given without idx");
    if (l->table_size < P) return set_error(FDR_ERR_INVALID, "table smaller than n_params");
  }
  out->base = l->base;
  out->base_stride = l->base_stride;
  out->table = l->table;
  out->max_idx = l->table ? l->table_size - P : 0;
  out->idx = l->idx;
  out->sign = l->sign;
  out->sigma = l->sigma;
  out->deterministic = l->deterministic;
  out->lane_offset = l->lane_offset;
  return FDR_OK;
}

}  // namespace fdr

using namespace fdr;

// fdr_ctx: one engine context per device (fdr::Context: rollout kernel selection, Impala phase profiling, replay
// GEMM switch, debug clocks).  NULL = the process-wide default context.
struct fdr_ctx {
  fdr::Context c;
};

namespace fdr {
Context& default_context() {
  static Context* d = [] {
    Context* c = new Context();
    const char* e = getenv("FDR_ROLLOUT");
    c->rollout_impl = !e ? FDR_ROLLOUT_AUTO
                         : strcmp(e, "single") == 0 ? FDR_ROLLOUT_SINGLE
                         : strcmp(e, "wide") == 0   ? FDR_ROLLOUT_WIDE
                                                    : strcmp(e, "pair") == 0 ? FDR_ROLLOUT_PAIR : FDR_ROLLOUT_AUTO;
    return c;
  }();
  return *d;
}

int context_cus(const Context& c) {
  if (c.cus > 0) return c.cus;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  return cus;
}
}  // namespace fdr

// The context of a call: ctx, or the default one; a ctx is bound to its device (the caller's current device
// must be that device -- its stream belongs to it).
static int resolve(fdr_ctx* ctx, Context** out) {
  if (!ctx) {
    *out = &default_context();
    return FDR_OK;
  }
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return set_error(FDR_ERR_HIP, "hipGetDevice failed");
  if (dev != ctx->c.device) {
    char msg[96];
    snprintf(msg, sizeof(msg), "fdr_ctx belongs to device %d, the current device is %d", ctx->c.device, dev);
    return set_error(FDR_ERR_INVALID, msg);
  }
  *out = &ctx->c;
  return FDR_OK;
}

#define FDR_CTX(ctx, C)          \
  Context* C = nullptr;          \
  {                              \
    const int rc_ = resolve(ctx, &C); \
    if (rc_) return rc_;         \
  }                              \
  (void)C

extern "C" {

const char* fdr_version(void) { return "fdr 0.5 gfx950"; }
const char* fdr_last_error(void) { return g_err.c_str(); }

static int set_impl(Context& c, int32_t impl) {
  if (impl != FDR_ROLLOUT_PAIR && impl != FDR_ROLLOUT_SINGLE && impl != FDR_ROLLOUT_AUTO && impl != FDR_ROLLOUT_WIDE)
    return set_error(FDR_ERR_INVALID, "unknown rollout impl");
  c.rollout_impl = impl;
  return FDR_OK;
}
int fdr_rollout_set_impl(int32_t impl) { return set_impl(default_context(), impl); }
int fdr_ctx_set_rollout_impl(fdr_ctx* ctx, int32_t impl) { return set_impl(ctx ? ctx->c : default_context(), impl); }
int fdr_ctx_set_replay_gemm(fdr_ctx* ctx, int32_t on) {
  (ctx ? ctx->c : default_context()).replay_gemm = on != 0;
  return FDR_OK;
}
int fdr_ctx_impala_profile(fdr_ctx* ctx, int32_t enable) { return impala::set_profile(ctx ? ctx->c : default_context(), enable); }
int fdr_ctx_impala_profile_read(fdr_ctx* ctx, double* ms) {
  if (!ms) return set_error(FDR_ERR_INVALID, "NULL pointer");
  return impala::read_profile(ctx ? ctx->c : default_context(), ms);
}
int fdr_ctx_impala_debug_clock(fdr_ctx* ctx, uint64_t* buf) {
  (ctx ? ctx->c : default_context()).debug_clock = buf;
  return FDR_OK;
}

int fdr_ctx_create(int device, fdr_ctx** out) {
  if (!out) return set_error(FDR_ERR_INVALID, "out is NULL");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
    return set_error(FDR_ERR_HIP, "no such HIP device");
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return set_error(FDR_ERR_HIP, "hipDeviceGetAttribute failed");
  fdr_ctx* c = new fdr_ctx();
  c->c.device = device;
  c->c.cus = cus;
  c->c.rollout_impl = default_context().rollout_impl;  // FDR_ROLLOUT applies to new contexts too
  *out = c;
  return FDR_OK;
}

int fdr_ctx_destroy(fdr_ctx* ctx) {
  if (ctx) impala::destroy_profile(ctx->c.prof);
  delete ctx;
  return FDR_OK;
}

int fdr_ctx_device(const fdr_ctx* ctx) { return ctx ? ctx->c.device : -1; }

int fdr_perturb(fdr_ctx* ctx, const float* theta, int64_t n_params, const float* table,
                int64_t table_size, const int64_t* idx, const int8_t* sign, int32_t n_lanes,
                float sigma, float* out, fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (!theta || !table || !idx || !out) return set_error(FDR_ERR_INVALID, "NULL pointer");
  if (n_params <= 0 || table_size < n_params || n_lanes < 0)
    return set_error(FDR_ERR_INVALID, "bad sizes");
  if (n_lanes == 0) return FDR_OK;
  return launch_perturb(theta, n_params, table, table_size, idx, sign, n_lanes, sigma, out,
                        (hipStream_t)stream);
}

int fdr_policy_forward(fdr_ctx* ctx, const fdr_policy_desc* policy, const fdr_lanes_desc* lanes,
                       int32_t n_lanes, const float* x, float* out0, float* out1,
                       fdr_stream stream) {
  FDR_CTX(ctx, C);
  PolicyKey k;
  int rc = policy_key(policy, &k);
  if (rc) return rc;
  LanesArgs la;
  rc = lanes_args(lanes, n_lanes, k.n_params, &la);
  if (rc) return rc;
  if (!x || !out0 || (!k.discrete && !out1)) return set_error(FDR_ERR_INVALID, "NULL x/out");
  if (n_lanes == 0) return FDR_OK;
  return launch_policy_forward(k, la, n_lanes, policy->bn_mean, policy->bn_var, x, out0, out1,
                               (hipStream_t)stream);
}

int fdr_rollout(fdr_ctx* ctx, const fdr_policy_desc* policy, const fdr_env_desc* env,
                const fdr_lanes_desc* lanes, int32_t n_lanes, uint64_t seed, int32_t jiggle,
                const float* obs_mean, const float* obs_std, double* ret, double* ent,
                int32_t* steps, double* norm2, fdr_stream stream) {
  return fdr_rollout_states(ctx, policy, env, lanes, n_lanes, seed, jiggle, obs_mean, obs_std, ret, ent, steps,
                            norm2, nullptr, stream);
}

int fdr_rollout_states(fdr_ctx* ctx, const fdr_policy_desc* policy, const fdr_env_desc* env,
                       const fdr_lanes_desc* lanes, int32_t n_lanes, uint64_t seed, int32_t jiggle,
                       const float* obs_mean, const float* obs_std, double* ret, double* ent,
                       int32_t* steps, double* norm2, float* states, fdr_stream stream) {
  fdr_rollout_extras x{};
  x.states = states;
  return fdr_rollout_ex(ctx, policy, env, lanes, n_lanes, seed, jiggle, obs_mean, obs_std, ret, ent, steps, norm2,
                        &x, stream);
}

int fdr_obs_stats_merge(fdr_ctx* ctx, const float* mean, const float* m2, const int32_t* count, int32_t n, int32_t dim,
                        float* acc_mean, float* acc_m2, int64_t* acc_count, fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (n < 0 || dim <= 0) return set_error(FDR_ERR_INVALID, "bad sizes");
  if ((n > 0 && (!mean || !m2 || !count)) || !acc_mean || !acc_m2 || !acc_count)
    return set_error(FDR_ERR_INVALID, "NULL pointer");
  return launch_obs_stats_merge(mean, m2, count, n, dim, acc_mean, acc_m2, acc_count, (hipStream_t)stream);
}

int fdr_rollout_ex(fdr_ctx* ctx, const fdr_policy_desc* policy, const fdr_env_desc* env,
                   const fdr_lanes_desc* lanes, int32_t n_lanes, uint64_t seed, int32_t jiggle,
                   const float* obs_mean, const float* obs_std, double* ret, double* ent, int32_t* steps,
                   double* norm2, const fdr_rollout_extras* extras, fdr_stream stream) {
  FDR_CTX(ctx, C);
  PolicyKey k;
  int rc = policy_key(policy, &k);
  if (rc) return rc;
  RolloutArgs a;
  std::memset(&a, 0, sizeof(a));
  rc = lanes_args(lanes, n_lanes, k.n_params, &a.lanes);
  if (rc) return rc;
  if (!env) return set_error(FDR_ERR_INVALID, "env desc is NULL");
  if (!ret || !ent || !steps) return set_error(FDR_ERR_INVALID, "NULL output");
  if ((obs_mean == nullptr) != (obs_std == nullptr))
    return set_error(FDR_ERR_INVALID, "obs_mean and obs_std must both be given or both NULL");
  if (env->episode_len <= 0 || env->episode_len >= (1 << 28))
    return set_error(FDR_ERR_INVALID, "episode_len out of range");
  if (env->obs_dim != k.n_in || env->act_dim != k.n_act)
    return set_error(FDR_ERR_INVALID, "env obs/act dims do not match the policy");
  if (env->kind == FDR_ENV_SYNTH) {
    if (!env->M || !env->K || !env->s0) return set_error(FDR_ERR_INVALID, "synthetic env needs M, K, s0");
    if (!(env->done_threshold >= 0.f) || env->done_threshold > 3.0e38f)
      return set_error(FDR_ERR_INVALID, "done_threshold must be finite and >= 0");
    if (env->done_threshold > 0.f && (env->done_dim < 0 || env->done_dim >= env->obs_dim))
      return set_error(FDR_ERR_INVALID, "done_dim out of range");
  } else if (env->kind == FDR_ENV_TRAP) {
    if (!env->walkable || env->map_w <= 0 || env->map_h <= 0)
      return set_error(FDR_ERR_INVALID, "trap env needs the walkable map");
    if (!k.discrete || k.n_in != 2 || k.n_act != 9)
      return set_error(FDR_ERR_INVALID, "trap env needs a DiscretePolicy(2, 9)");
  } else {
    return set_error(FDR_ERR_INVALID, "unknown env kind");
  }
  if (n_lanes == 0) return FDR_OK;
  a.n_lanes = n_lanes;
  a.T = env->episode_len;
  a.key = mix64(seed);
  a.jiggle = jiggle;
  a.bn_mean = policy->bn_mean;
  a.bn_var = policy->bn_var;
  a.obs_mean = obs_mean;
  a.obs_std = obs_std;
  a.M = env->M;
  a.K = env->K;
  a.s0 = env->s0;
  a.done_thr = env->kind == FDR_ENV_SYNTH ? env->done_threshold : 0.f;
  a.done_dim = env->kind == FDR_ENV_SYNTH && env->done_threshold > 0.f ? env->done_dim : 0;
  a.walkable = env->walkable;
  a.map_w = env->map_w;
  a.map_h = env->map_h;
  // environment.py:21 -> tile_map.get_node(width*r//2, height*r//2) with r = 7
  a.trap_start_col = (env->map_w * 7 / 2) / 7;
  a.trap_start_row = (env->map_h * 7 / 2) / 7;
  a.ret = ret;
  a.ent = ent;
  a.steps = steps;
  a.norm2 = norm2;
  if (extras) {
    a.states = extras->states;
    if (extras->obs_mean || extras->obs_m2 || extras->obs_count) {
      if (!extras->obs_mean || !extras->obs_m2 || !extras->obs_count)
        return set_error(FDR_ERR_INVALID, "obs_mean, obs_m2 and obs_count must be given together");
      a.os_mean = extras->obs_mean;
      a.os_m2 = extras->obs_m2;
      a.os_count = extras->obs_count;
      a.os_chance = extras->obs_chance;
    }
    a.u_inject = extras->u_inject;
    if (a.u_inject && a.os_mean)
      return set_error(FDR_ERR_UNSUPPORTED, "u_inject is not combined with the obs statistics");
  }
  return launch_rollout(*C, k, env->kind, a, (hipStream_t)stream);
}

int fdr_fd_weights(fdr_ctx* ctx, const double* rewards_all, int32_t n_all, double policy_reward,
                   int32_t lane_lo, int32_t n_local, const int8_t* sign_local,
                   const double* norm2_local, int32_t lanes_per_dir, float sigma, double* coef,
                   fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (!rewards_all || !sign_local || !norm2_local || !coef)
    return set_error(FDR_ERR_INVALID, "NULL pointer");
  if (n_all <= 0 || lane_lo < 0 || n_local < 0 || lane_lo + n_local > n_all)
    return set_error(FDR_ERR_INVALID, "bad lane range");
  if (lanes_per_dir < 1 || n_local % lanes_per_dir != 0)
    return set_error(FDR_ERR_INVALID, "n_local must be a multiple of lanes_per_dir");
  return launch_fd_weights(rewards_all, n_all, policy_reward, lane_lo, n_local, sign_local,
                           norm2_local, lanes_per_dir, sigma, coef, (hipStream_t)stream);
}

int64_t fdr_fd_grad_workspace_bytes(int32_t n_dirs, int64_t n_params) {
  return grad_workspace_bytes(n_dirs, n_params);
}

int fdr_fd_grad(fdr_ctx* ctx, const float* table, int64_t table_size, const int64_t* idx,
                const double* coef, int32_t n_dirs, int64_t n_params, double* g, void* workspace,
                int64_t workspace_bytes, fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (!table || !g || n_params <= 0 || table_size < n_params || n_dirs < 0)
    return set_error(FDR_ERR_INVALID, "bad arguments");
  if (n_dirs == 0) {
    const hipError_t e = hipMemsetAsync(g, 0, n_params * sizeof(double), (hipStream_t)stream);
    return e == hipSuccess ? FDR_OK : set_error(FDR_ERR_HIP, hipGetErrorString(e));
  }
  if (!idx || !coef) return set_error(FDR_ERR_INVALID, "NULL idx/coef");
  return launch_fd_grad(table, table_size, idx, coef, n_dirs, n_params, g, workspace,
                        workspace_bytes, (hipStream_t)stream);
}

int64_t fdr_dsgd_workspace_bytes(int64_t n_params) { return dsgd_workspace_bytes(n_params); }

int fdr_dsgd_step(fdr_ctx* ctx, float* theta, const double* g, int64_t n_params, double lr,
                  double lr_scale, double* out, void* workspace, int64_t workspace_bytes,
                  fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (!theta || !g || !out || n_params <= 0) return set_error(FDR_ERR_INVALID, "bad arguments");
  return launch_dsgd_ex(theta, g, 0, n_params, lr, lr_scale, nullptr, out, workspace, workspace_bytes,
                        (hipStream_t)stream);
}

int fdr_dsgd_step_ex(fdr_ctx* ctx, float* theta, const double* src, int32_t src_is_moments, int64_t n_params,
                     double lr, double lr_scale, double* g_out, double* out, void* workspace, int64_t workspace_bytes,
                     fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (!theta || !src || !out || n_params <= 0) return set_error(FDR_ERR_INVALID, "bad arguments");
  return launch_dsgd_ex(theta, src, src_is_moments ? 1 : 0, n_params, lr, lr_scale, g_out, out, workspace,
                        workspace_bytes, (hipStream_t)stream);
}

int64_t fdr_fd_grad_fused_workspace_bytes(int32_t n_dirs, int32_t lanes_per_dir, int64_t n_params, int32_t mode) {
  if (lanes_per_dir < 1) return -1;
  return fused_workspace_bytes(n_dirs, n_dirs * lanes_per_dir, n_params, mode);
}

int64_t fdr_fd_grad_fused_counter_bytes(int32_t n_dirs, int64_t n_params) {
  return n_params > 0 ? fused_counter_bytes(n_dirs, n_params) : -1;
}

int64_t fdr_fd_grad_fused_out_len(int32_t mode, int64_t n_params, int32_t n_all) {
  if (n_params <= 0) return -1;
  if (mode == FDR_WEIGHT_ZSCORE || mode == FDR_WEIGHT_CENTERED_RANK) return n_params;
  if (mode == FDR_WEIGHT_MOMENTS) return n_all > 0 ? 2 * n_params + 1 + n_all : -1;
  return -1;
}

static int fd_grad_fused_impl(const float* table, int64_t table_size, const int64_t* idx_local, int32_t n_dirs,
                              int64_t n_params, const double* rewards_all, int32_t n_all, double policy_reward,
                              int32_t lane_lo, const int8_t* sign_local, const double* norm2_local, int32_t lanes_per_dir,
                              float sigma, int32_t mode, double* out, float* theta, double lr, double lr_scale,
                              float* hist, double* dsgd_out, void* workspace, int64_t workspace_bytes,
                              fdr_stream stream) {
  if (!table || !out || n_params <= 0 || table_size < n_params || n_dirs < 0)
    return set_error(FDR_ERR_INVALID, "bad arguments");
  if (mode != FDR_WEIGHT_ZSCORE && mode != FDR_WEIGHT_CENTERED_RANK && mode != FDR_WEIGHT_MOMENTS)
    return set_error(FDR_ERR_INVALID, "unknown weighting mode");
  if (lanes_per_dir < 1) return set_error(FDR_ERR_INVALID, "lanes_per_dir < 1");
  if (n_dirs == 0) return set_error(FDR_ERR_INVALID, "no directions (DSGD would divide by ||g|| = 0)");
  const int n_local = n_dirs * lanes_per_dir;
  if (!idx_local || !rewards_all || !sign_local || !norm2_local) return set_error(FDR_ERR_INVALID, "NULL pointer");
  if (n_all <= 0 || lane_lo < 0 || lane_lo + n_local > n_all) return set_error(FDR_ERR_INVALID, "bad lane range");
  return launch_fd_grad_fused(table, table_size, idx_local, n_dirs, n_params, rewards_all, n_all, policy_reward,
                              lane_lo, sign_local, norm2_local, lanes_per_dir, sigma, mode, out, theta, lr, lr_scale,
                              hist, dsgd_out, workspace, workspace_bytes, (hipStream_t)stream);
}

int fdr_fd_grad_fused(fdr_ctx* ctx, const float* table, int64_t table_size, const int64_t* idx_local, int32_t n_dirs,
                      int64_t n_params, const double* rewards_all, int32_t n_all, double policy_reward, int32_t lane_lo,
                      const int8_t* sign_local, const double* norm2_local, int32_t lanes_per_dir, float sigma,
                      int32_t mode, double* out, int64_t out_len, void* workspace, int64_t workspace_bytes,
                      fdr_stream stream) {
  FDR_CTX(ctx, C);
  const int64_t need = fdr_fd_grad_fused_out_len(mode, n_params, n_all);
  if (need > 0 && out_len < need) return set_error(FDR_ERR_INVALID, "out_len below fdr_fd_grad_fused_out_len");
  return fd_grad_fused_impl(table, table_size, idx_local, n_dirs, n_params, rewards_all, n_all, policy_reward, lane_lo,
                            sign_local, norm2_local, lanes_per_dir, sigma, mode, out, nullptr, 0.0, 0.0, nullptr,
                            nullptr, workspace, workspace_bytes, stream);
}

int fdr_fd_step(fdr_ctx* ctx, const float* table, int64_t table_size, const int64_t* idx_local, int32_t n_dirs,
                int64_t n_params, const double* rewards_all, int32_t n_all, double policy_reward,
                const int8_t* sign_local, const double* norm2_local, int32_t lanes_per_dir, float sigma, int32_t mode,
                float* theta, double lr, double lr_scale, double* g, float* theta_hist, double* out, void* workspace,
                int64_t workspace_bytes, fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (!theta || !g || !out) return set_error(FDR_ERR_INVALID, "NULL theta / g / out");
  if (mode == FDR_WEIGHT_MOMENTS) return set_error(FDR_ERR_INVALID, "fdr_fd_step takes z-score or centred-rank weights");
  if (n_all != n_dirs * lanes_per_dir) return set_error(FDR_ERR_INVALID, "fdr_fd_step is single-process: n_all = n_local");
  return fd_grad_fused_impl(table, table_size, idx_local, n_dirs, n_params, rewards_all, n_all, policy_reward, 0,
                            sign_local, norm2_local, lanes_per_dir, sigma, mode, g, theta, lr, lr_scale, theta_hist,
                            out, workspace, workspace_bytes, stream);
}

int fdr_rank_weights(fdr_ctx* ctx, const double* rewards_all, int32_t n_all, int32_t lane_lo, int32_t n_local,
                     double* w, fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (!rewards_all || !w || n_all <= 0 || lane_lo < 0 || n_local < 0 || lane_lo + n_local > n_all)
    return set_error(FDR_ERR_INVALID, "bad arguments");
  return launch_rank_weights(rewards_all, n_all, lane_lo, n_local, w, (hipStream_t)stream);
}

}  // extern "C"

// ---- ImpalaPolicy ----------------------------------------------------------------------------
int64_t fdr_impala_num_params(int32_t n_act) {
  impala::Layout L;
  return impala::make_layout(n_act, &L) ? L.P : -1;
}

int64_t fdr_impala_num_bn_stats(void) {
  impala::Layout L;
  impala::make_layout(1, &L);
  return L.n_bn_stats;
}

static int impala_layout(const fdr_impala_desc* d, impala::Layout* L) {
  if (!d) return set_error(FDR_ERR_INVALID, "impala desc is NULL");
  if (!impala::make_layout(d->n_act, L)) return set_error(FDR_ERR_UNSUPPORTED, "n_act must be in 1..32");
  if (d->n_params != L->P) return set_error(FDR_ERR_INVALID, "n_params does not match the ImpalaCNN layout");
  return FDR_OK;
}

int64_t fdr_impala_workspace_bytes(const fdr_impala_desc* d, int32_t n_lanes) {
  impala::Layout L;
  if (!d || n_lanes < 0 || !impala::make_layout(d->n_act, &L)) return -1;
  return impala::plan(L, n_lanes, d->envs_per_lane, d->episode_len, d->entropy != 0, d->fp16 != 0, d->pairs != 0).total;
}

int fdr_impala_rollout(fdr_ctx* ctx, const fdr_impala_desc* d, const fdr_lanes_desc* lanes,
                       int32_t n_lanes, uint64_t seed, int32_t jiggle, double* ret, double* ent,
                       int32_t* steps, double* norm2, int32_t* actions, float* probs, void* ws,
                       int64_t ws_bytes, fdr_stream stream) {
  FDR_CTX(ctx, C);
  impala::Layout L;
  int rc = impala_layout(d, &L);
  if (rc) return rc;
  impala::RolloutCall c{};
  rc = lanes_args(lanes, n_lanes, L.P, &c.lanes);
  if (rc) return rc;
  const int E = d->envs_per_lane;
  if (E != 1 && E != 2 && E != 4 && E != 8) return set_error(FDR_ERR_UNSUPPORTED, "envs_per_lane must be 1, 2, 4 or 8");
  if (d->episode_len <= 0 || d->episode_len >= (1 << 20)) return set_error(FDR_ERR_INVALID, "episode_len out of range");
  if (!ret || !ent || !steps) return set_error(FDR_ERR_INVALID, "NULL output");
  c.ctx = C;
  c.layout = &L;
  c.n_lanes = n_lanes;
  c.envs = E;
  c.T = d->episode_len;
  c.entropy = d->entropy != 0;
  c.jiggle = jiggle;
  c.fp16 = d->fp16 != 0;
  c.pairs = d->pairs != 0;
  if (c.pairs && (n_lanes & 1)) return set_error(FDR_ERR_INVALID, "pairs: n_lanes must be even");
  c.seed = seed;
  c.env_seed = d->env_seed;
  c.bn_mean = d->bn_mean;
  c.bn_var = d->bn_var;
  c.ret = ret;
  c.ent = ent;
  c.steps = steps;
  c.norm2 = norm2;
  c.actions = actions;
  c.probs = probs;
  return impala::launch_rollout(c, ws, ws_bytes, (hipStream_t)stream);
}

int64_t fdr_impala_forward_workspace_bytes(int32_t n_act, int32_t n_envs, int32_t fp16) {
  impala::Layout L;
  if (n_envs < 0 || !impala::make_layout(n_act, &L)) return -1;
  return impala::forward_workspace_bytes(L, n_envs, fp16 != 0);
}

int fdr_impala_forward(fdr_ctx* ctx, const fdr_impala_desc* d, const float* theta, int32_t n_envs,
                       const float* frames, const float* reward, const float* notdone, float* h,
                       float* c, float* probs, float* feat, void* ws, int64_t ws_bytes,
                       fdr_stream stream) {
  FDR_CTX(ctx, C);
  impala::Layout L;
  int rc = impala_layout(d, &L);
  if (rc) return rc;
  if (!theta || !frames || !h || !c || !probs) return set_error(FDR_ERR_INVALID, "NULL pointer");
  if (n_envs < 0) return set_error(FDR_ERR_INVALID, "n_envs < 0");
  impala::ForwardCall f{};
  f.layout = &L;
  f.fp16 = d->fp16 != 0;
  f.theta = theta;
  f.n_envs = n_envs;
  f.frames = frames;
  f.reward = reward;
  f.notdone = notdone;
  f.h = h;
  f.c = c;
  f.probs = probs;
  f.feat_out = feat;
  f.bn_mean = d->bn_mean;
  f.bn_var = d->bn_var;
  return impala::launch_forward(f, ws, ws_bytes, (hipStream_t)stream);
}

int64_t fdr_impala_bn_refresh_workspace_bytes(int32_t n) { return n < 0 ? -1 : impala::vbn_workspace_bytes(n); }

int fdr_impala_bn_refresh(fdr_ctx* ctx, const fdr_impala_desc* d, const float* theta, int32_t n, const float* frames,
                          const float* reward, int32_t first_done, float* h, float* c, float momentum, float* bn_mean,
                          float* bn_var, void* ws, int64_t ws_bytes, fdr_stream stream) {
  FDR_CTX(ctx, C);
  impala::Layout L;
  int rc = impala_layout(d, &L);
  if (rc) return rc;
  if (!theta || !frames || !bn_mean || !bn_var) return set_error(FDR_ERR_INVALID, "NULL pointer");
  if ((h == nullptr) != (c == nullptr)) return set_error(FDR_ERR_INVALID, "h and c must both be given or both NULL");
  if (n < 2) return set_error(FDR_ERR_INVALID, "train-mode BatchNorm1d needs n >= 2 samples");
  impala::VbnCall v{&L, theta, n, frames, reward, first_done != 0, h, c, momentum, bn_mean, bn_var};
  return impala::launch_vbn(v, ws, ws_bytes, (hipStream_t)stream);
}

int64_t fdr_impala_strategies_workspace_bytes(const fdr_impala_desc* d, int32_t n_lanes, int32_t n_states) {
  impala::Layout L;
  if (!d || n_lanes < 0 || n_states < 0 || !impala::make_layout(d->n_act, &L)) return -1;
  return impala::strategies_workspace_bytes(L, n_lanes, n_states, d->fp16 != 0, d->pairs != 0);
}

int fdr_impala_strategies(fdr_ctx* ctx, const fdr_impala_desc* d, const fdr_lanes_desc* lanes, int32_t n_lanes,
                          int32_t n_states, const float* frames, const float* reward, float* h, float* c,
                          float* probs, void* ws, int64_t ws_bytes, fdr_stream stream) {
  FDR_CTX(ctx, C);
  impala::Layout L;
  int rc = impala_layout(d, &L);
  if (rc) return rc;
  impala::StrategiesCall sc{};
  rc = lanes_args(lanes, n_lanes, L.P, &sc.lanes);
  if (rc) return rc;
  if (n_states < 0 || n_states > (1 << 20)) return set_error(FDR_ERR_INVALID, "n_states out of range");
  if (n_states > 0 && (!frames || !probs)) return set_error(FDR_ERR_INVALID, "NULL frames / probs");
  if ((h == nullptr) != (c == nullptr)) return set_error(FDR_ERR_INVALID, "h and c must both be given or both NULL");
  sc.layout = &L;
  sc.n_lanes = n_lanes;
  sc.n_states = n_states;
  sc.fp16 = d->fp16 != 0;
  sc.pairs = d->pairs != 0;
  if (sc.pairs && (n_lanes & 1)) return set_error(FDR_ERR_INVALID, "pairs: n_lanes must be even");
  sc.frames = frames;
  sc.reward = reward;
  sc.h = h;
  sc.c = c;
  sc.probs = probs;
  sc.bn_mean = d->bn_mean;
  sc.bn_var = d->bn_var;
  return impala::launch_strategies(sc, ws, ws_bytes, (hipStream_t)stream);
}

int fdr_impala_env_frames(uint64_t env_seed, int32_t n_act, int64_t env_id, int32_t t0, int32_t n,
                          const int32_t* actions, float* frames, float* reward, fdr_stream stream) {
  if (n_act < 1 || n_act > impala::kMaxAct) return set_error(FDR_ERR_INVALID, "n_act must be in 1..32");
  if (n < 0 || t0 < 0 || t0 + (int64_t)n >= (1 << 20) || env_id < 0) return set_error(FDR_ERR_INVALID, "bad range");
  if (n > 0 && !frames) return set_error(FDR_ERR_INVALID, "NULL frames");
  return impala::launch_env_frames(env_seed, n_act, (uint64_t)env_id, t0, n, actions, frames, reward,
                                   (hipStream_t)stream);
}

int fdr_impala_profile(int32_t enable) { return fdr_ctx_impala_profile(nullptr, enable); }
int fdr_impala_profile_read(double* ms) { return fdr_ctx_impala_profile_read(nullptr, ms); }
int fdr_impala_debug_clock(uint64_t* buf) { return fdr_ctx_impala_debug_clock(nullptr, buf); }
int fdr_impala_set_replay_gemm(int32_t on) { return fdr_ctx_set_replay_gemm(nullptr, on); }

int fdr_strategy_distances(fdr_ctx* ctx, const float* strategies, int32_t n, const float* archive, int32_t n_archive,
                           int32_t n_states, int32_t dim, int32_t kind, double* dists, double* min_dist,
                           int32_t* argmin, fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (n < 0 || n_archive <= 0 || n_states <= 0 || dim <= 0) return set_error(FDR_ERR_INVALID, "bad sizes");
  if (n > 0 && (!strategies || !archive)) return set_error(FDR_ERR_INVALID, "NULL pointer");
  if (kind != FDR_DIST_L2 && kind != FDR_DIST_TVD && kind != FDR_DIST_W2)
    return set_error(FDR_ERR_INVALID, "unknown distance kind");
  if (kind == FDR_DIST_W2 && (dim & 1)) return set_error(FDR_ERR_INVALID, "W2 needs dim = 2k ([mean | std])");
  return launch_strategy_dist(strategies, n, archive, n_archive, n_states, dim, kind, dists, min_dist, argmin,
                              (hipStream_t)stream);
}

static int lambda_row(const float* table, int64_t table_size, const int64_t* idx, const int8_t* sign,
                      const int32_t* slot, int32_t n, int64_t P, float sigma, const float* drift, int32_t n_slots,
                      LambdaRow* R) {
  if (n < 0 || P <= 0 || table_size < P) return set_error(FDR_ERR_INVALID, "bad sizes");
  if (n > 0 && (!table || !idx)) return set_error(FDR_ERR_INVALID, "NULL pointer");
  if (n_slots < 0 || (n_slots > 0 && !drift)) return set_error(FDR_ERR_INVALID, "drift missing");
  *R = LambdaRow{table, table_size - P, idx, sign, slot, drift, n_slots, P, sigma};
  return FDR_OK;
}

int fdr_fd_lambda_norms(fdr_ctx* ctx, const float* table, int64_t table_size, const int64_t* idx, const int8_t* sign,
                        const int32_t* slot, int32_t n, int64_t n_params, float sigma, const float* drift,
                        int32_t n_slots, double* norm2, fdr_stream stream) {
  FDR_CTX(ctx, C);
  LambdaRow R;
  int rc = lambda_row(table, table_size, idx, sign, slot, n, n_params, sigma, drift, n_slots, &R);
  if (rc) return rc;
  if (!norm2) return set_error(FDR_ERR_INVALID, "NULL output");
  return launch_lambda_norms(R, n, norm2, (hipStream_t)stream);
}

int fdr_fd_grad_lambda(fdr_ctx* ctx, const float* table, int64_t table_size, const int64_t* idx, const int8_t* sign,
                       const int32_t* slot, const double* coef, int32_t n, int64_t n_params, float sigma,
                       const float* drift, int32_t n_slots, double* g, void* ws, int64_t ws_bytes,
                       fdr_stream stream) {
  FDR_CTX(ctx, C);
  LambdaRow R;
  int rc = lambda_row(table, table_size, idx, sign, slot, n, n_params, sigma, drift, n_slots, &R);
  if (rc) return rc;
  if (!g || (n > 0 && !coef)) return set_error(FDR_ERR_INVALID, "NULL pointer");
  if (n == 0) return set_error(FDR_ERR_INVALID, "no returns");
  return launch_lambda_grad(R, coef, n, g, ws, ws_bytes, (hipStream_t)stream);
}

int64_t fdr_bn_refresh_workspace_bytes(int32_t n) { return n < 0 ? -1 : bn_refresh_workspace_bytes(n); }

int fdr_bn_refresh(fdr_ctx* ctx, const fdr_policy_desc* policy, const float* theta, const float* x, int32_t n,
                   float momentum, float* bn_mean, float* bn_var, void* ws, int64_t ws_bytes, fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (!policy || policy->kind != FDR_POLICY_DISCRETE || policy->hidden != kHidden)
    return set_error(FDR_ERR_UNSUPPORTED, "BN refresh is defined for the DiscretePolicy (hidden 64)");
  if (policy->n_in <= 0 || policy->n_in > 64) return set_error(FDR_ERR_UNSUPPORTED, "n_in must be in 1..64");
  if (!theta || !x || !bn_mean || !bn_var) return set_error(FDR_ERR_INVALID, "NULL pointer");
  if (n < 2) return set_error(FDR_ERR_INVALID, "train-mode BatchNorm needs n >= 2 samples");
  return launch_bn_refresh(policy->n_in, theta, x, n, momentum, bn_mean, bn_var, ws, ws_bytes, (hipStream_t)stream);
}

// ---- AtariPolicy ---------------------------------------------------------------------------------------
int64_t fdr_atari_num_params(int32_t n_act) { return atari::num_params(n_act); }

int64_t fdr_atari_workspace_bytes(const fdr_atari_desc* d, int32_t n_lanes) {
  if (!d || n_lanes < 0) return -1;
  return atari::workspace_bytes(d->n_act, n_lanes, d->envs_per_lane);
}

int fdr_atari_rollout(fdr_ctx* ctx, const fdr_atari_desc* d, const fdr_lanes_desc* lanes, int32_t n_lanes,
                      uint64_t seed, int32_t jiggle, double* ret, double* ent, int32_t* steps, double* norm2,
                      int32_t* actions, float* probs, void* ws, int64_t ws_bytes, fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (!d) return set_error(FDR_ERR_INVALID, "atari desc is NULL");
  const int64_t P = atari::num_params(d->n_act);
  if (P < 0) return set_error(FDR_ERR_UNSUPPORTED, "n_act must be in 1..32");
  if (d->n_params != P) return set_error(FDR_ERR_INVALID, "n_params does not match the AtariPolicy layout");
  const int E = d->envs_per_lane;
  if (E != 1 && E != 2 && E != 4) return set_error(FDR_ERR_UNSUPPORTED, "envs_per_lane must be 1, 2 or 4");
  if (d->episode_len <= 0 || d->episode_len >= (1 << 20)) return set_error(FDR_ERR_INVALID, "episode_len out of range");
  if (!ret || !ent || !steps) return set_error(FDR_ERR_INVALID, "NULL output");
  LanesArgs la;
  int rc = lanes_args(lanes, n_lanes, P, &la);
  if (rc) return rc;
  return atari::launch_rollout(d->n_act, E, d->episode_len, d->env_seed, la, n_lanes, seed, jiggle, d->bn_mean,
                               d->bn_var, ret, ent, steps, norm2, actions, probs, ws, ws_bytes, (hipStream_t)stream);
}

int64_t fdr_atari_forward_workspace_bytes(int32_t n_act, int32_t n) {
  return n < 0 ? -1 : atari::forward_workspace_bytes(n_act, n);
}

int fdr_atari_env_frames(uint64_t env_seed, int64_t env_id, int32_t t0, int32_t n, float* frames, fdr_stream stream) {
  if (n < 0 || t0 < 0 || t0 + (int64_t)n >= (1 << 20) || env_id < 0 || env_id >= (1ll << 31))
    return set_error(FDR_ERR_INVALID, "bad range");
  if (n > 0 && !frames) return set_error(FDR_ERR_INVALID, "NULL frames");
  return atari::launch_env_frames(env_seed, (uint64_t)env_id, t0, n, frames, (hipStream_t)stream);
}

int fdr_atari_forward(fdr_ctx* ctx, const fdr_atari_desc* d, const float* theta, int32_t n, const float* frames,
                      float* probs, float* feat, void* ws, int64_t ws_bytes, fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (!d) return set_error(FDR_ERR_INVALID, "atari desc is NULL");
  const int64_t P = atari::num_params(d->n_act);
  if (P < 0) return set_error(FDR_ERR_UNSUPPORTED, "n_act must be in 1..32");
  if (d->n_params != P) return set_error(FDR_ERR_INVALID, "n_params does not match the AtariPolicy layout");
  if (!theta || !frames || !probs || n < 0) return set_error(FDR_ERR_INVALID, "NULL pointer / bad n");
  return atari::launch_forward(d->n_act, theta, n, frames, d->bn_mean, d->bn_var, probs, feat, ws, ws_bytes,
                               (hipStream_t)stream);
}

int64_t fdr_atari_bn_refresh_workspace_bytes(int32_t n) { return atari::vbn_workspace_bytes(n); }

int fdr_atari_bn_refresh(fdr_ctx* ctx, const fdr_atari_desc* d, const float* theta, int32_t n, const float* frames,
                         float momentum, float* bn_mean, float* bn_var, void* ws, int64_t ws_bytes, fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (!d) return set_error(FDR_ERR_INVALID, "atari desc is NULL");
  const int64_t P = atari::num_params(d->n_act);
  if (P < 0) return set_error(FDR_ERR_UNSUPPORTED, "n_act must be in 1..32");
  if (d->n_params != P) return set_error(FDR_ERR_INVALID, "n_params does not match the AtariPolicy layout");
  if (!theta || !frames || !bn_mean || !bn_var) return set_error(FDR_ERR_INVALID, "NULL pointer");
  if (n < 2) return set_error(FDR_ERR_INVALID, "train-mode BatchNorm1d needs n >= 2 samples");
  return atari::launch_vbn(theta, n, frames, momentum, bn_mean, bn_var, ws, ws_bytes, (hipStream_t)stream);
}

int64_t fdr_atari_strategies_workspace_bytes(const fdr_atari_desc* d, int32_t n_lanes, int32_t n_states) {
  if (!d) return -1;
  return atari::strategies_workspace_bytes(d->n_act, n_lanes, n_states);
}

int fdr_atari_strategies(fdr_ctx* ctx, const fdr_atari_desc* d, const fdr_lanes_desc* lanes, int32_t n_lanes,
                         int32_t n_states, const float* frames, float* probs, void* ws, int64_t ws_bytes,
                         fdr_stream stream) {
  FDR_CTX(ctx, C);
  if (!d) return set_error(FDR_ERR_INVALID, "atari desc is NULL");
  const int64_t P = atari::num_params(d->n_act);
  if (P < 0) return set_error(FDR_ERR_UNSUPPORTED, "n_act must be in 1..32");
  if (d->n_params != P) return set_error(FDR_ERR_INVALID, "n_params does not match the AtariPolicy layout");
  if (n_states < 0 || (n_states > 0 && (!frames || !probs))) return set_error(FDR_ERR_INVALID, "NULL pointer / bad Z");
  LanesArgs la;
  int rc = lanes_args(lanes, n_lanes, P, &la);
  if (rc) return rc;
  return atari::launch_strategies(d->n_act, la, n_lanes, n_states, frames, d->bn_mean, d->bn_var, probs, ws, ws_bytes,
                                  (hipStream_t)stream);
}

// ---------------------------------------------------------------------------------------------
// Host index draw (utils/noise_sources.py:44-47: one RandomState.randint(0, max_idx) per sample).  MT19937
// (Matsumoto & Nishimura 1998, the generator behind numpy's legacy RandomState) advanced in place from the
// state numpy reports (key[624], pos), and numpy's masked rejection for ranges that fit 32 bits: each draw takes
// 32-bit words masked by the smallest all-ones mask >= max_idx - 1 until one is <= max_idx - 1.  numpy makes
// one indirect generator call and one unpredictable branch per word (~11 ns per index on the build host); a block
// of tempered words with a branch-free compaction takes ~2.5 ns, which keeps an 8-rank step's 16,384-index draw
// (every rank consumes the whole stream) well under the rollout it overlaps.
// ---------------------------------------------------------------------------------------------
namespace {
constexpr int kMtN = 624, kMtM = 397;

void mt_refill(uint32_t* key) {
  auto mix = [](uint32_t hi, uint32_t lo, uint32_t far) {
    const uint32_t y = (hi & 0x80000000u) | (lo & 0x7fffffffu);
    return far ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  };
  int i = 0;
  for (; i < kMtN - kMtM; ++i) key[i] = mix(key[i], key[i + 1], key[i + kMtM]);
  for (; i < kMtN - 1; ++i) key[i] = mix(key[i], key[i + 1], key[i + kMtM - kMtN]);
  key[kMtN - 1] = mix(key[kMtN - 1], key[0], key[kMtM - 1]);
}

inline uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  return y ^ (y >> 18);
}
}  // namespace

extern "C" int fdr_noise_draw_indices(uint32_t* key, int32_t* pos, int64_t max_idx, int32_t n, int64_t* out) {
  using namespace fdr;
  if (!key || !pos || (n > 0 && !out) || n < 0) return set_error(FDR_ERR_INVALID, "NULL pointer / bad n");
  if (max_idx < 1) return set_error(FDR_ERR_INVALID, "max_idx must be >= 1");
  if (*pos < 0 || *pos > kMtN) return set_error(FDR_ERR_INVALID, "MT19937 pos out of range");
  const uint64_t rng = (uint64_t)max_idx - 1;  // inclusive range of randint(0, max_idx)
  if (rng > 0xFFFFFFFFull) return set_error(FDR_ERR_UNSUPPORTED, "index range wider than 32 bits");
  if (rng == 0) {  // numpy returns the offset without drawing
    for (int32_t i = 0; i < n; ++i) out[i] = 0;
    return FDR_OK;
  }
  uint32_t mask = (uint32_t)rng;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  // a refill block at a time: temper + mask the block's remaining words (vectorised), then a branch-free
  // compaction keeps the accepted ones; the last block stops at the word that completes the n-th index, as
  // numpy's loop does (no extra words consumed)
  int p = *pos;
  int32_t k = 0;
  uint32_t buf[kMtN];
  while (k < n) {
    if (p == kMtN) {
      mt_refill(key);
      p = 0;
    }
    const int m = kMtN - p;
    for (int i = 0; i < m; ++i) buf[i] = mt_temper(key[p + i]) & mask;
    if (n - k >= m) {  // the whole block fits: k < n at every write
      for (int i = 0; i < m; ++i) {
        out[k] = buf[i];
        k += buf[i] <= (uint32_t)rng;
      }
      p += m;
    } else {
      int i = 0;
      for (; i < m && k < n; ++i) {
        out[k] = buf[i];
        k += buf[i] <= (uint32_t)rng;
      }
      p += i;
    }
  }
  *pos = p;
  return FDR_OK;
}
