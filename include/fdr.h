/*
 * fdr.h -- C ABI of the MI355X finite-difference rollout + gradient engine (libfdr.so).
 *
 * This is the drop-in boundary for the reference's perturbation-evaluation hot path
 * (nexus-rl/dfd-starter).  The reference has no FFI layer: its boundary is a set of Python
 * duck-typed interfaces.  Each entry point below names the reference
 * interface it replaces; the Python host layer (dfd-starter_amd/fdr/_lib.py, ctypes) binds
 * exactly these symbols -- INTEGRATION.md shows the binding a maintainer would add.
 *
 * Conventions
 *   - Every pointer argument is a DEVICE pointer owned by the caller (PyTorch-ROCm tensors),
 *     unless documented as host.  Nothing here allocates or frees memory.
 *   - Every compute call is asynchronous on the caller's stream (`fdr_stream` = hipStream_t;
 *     NULL = the legacy default stream) and performs no host synchronisation, no allocation and
 *     no host<->device copy, so the calls can be captured into a hipGraph.
 *   - Return value: FDR_OK or an error code; fdr_last_error() gives a thread-local message.
 *     No C++ exception crosses this boundary.
 *   - Numerics: see DESIGN.md.  theta' (fdr_perturb, and the in-kernel perturbation of
 *     fdr_rollout / fdr_policy_forward) is bit-exact with the reference's numpy f32 arithmetic.
 */
#ifndef FDR_H_
#define FDR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FDR_OK 0
#define FDR_ERR_INVALID 1     /* bad argument (null pointer, size, shape mismatch) */
#define FDR_ERR_UNSUPPORTED 2 /* policy/env shape with no compiled kernel instance */
#define FDR_ERR_HIP 3         /* HIP runtime error (launch failure, no device) */
#define FDR_ERR_WORKSPACE 4   /* caller's workspace too small */

typedef void* fdr_stream; /* hipStream_t */

/* Policy families (policies/discrete.py:34-48, policies/mujoco.py:32-41). */
#define FDR_POLICY_DISCRETE 0 /* BN-Linear-ReLU-BN-Linear-ReLU-BN-Linear-Softmax, hidden 64 */
#define FDR_POLICY_MUJOCO 1   /* Linear-Tanh-Linear-Tanh-Linear-tanh head, hidden 64 */

/* Environments run inside the rollout kernel. */
#define FDR_ENV_SYNTH 0 /* contractive linear-tanh system (DESIGN.md "Synthetic envs") */
#define FDR_ENV_TRAP 1  /* custom_envs/simple_trap_env (integer-exact) */

typedef struct fdr_policy_desc {
  int32_t kind;     /* FDR_POLICY_* */
  int32_t n_in;     /* observation size (policy.input_shape) */
  int32_t n_act;    /* discrete: number of actions; mujoco: action dims (head = 2*n_act) */
  int32_t hidden;   /* must be 64 (hard-coded by the reference) */
  int64_t n_params; /* P = len(get_trainable_flat()) */
  /* discrete only: eval-mode BatchNorm running stats of the 3 BN layers, concatenated
     [n_in | 64 | 64] (policies/discrete.py:38,42,46); NULL = (mean 0, var 1). */
  const float* bn_mean;
  const float* bn_var;
} fdr_policy_desc;

typedef struct fdr_env_desc {
  int32_t kind;        /* FDR_ENV_* */
  int32_t obs_dim;     /* must equal policy n_in */
  int32_t act_dim;     /* must equal policy n_act */
  int32_t episode_len; /* fixed episode length T (FDR_ENV_TRAP: 201, environment.py:19,43) */
  const float* M;      /* SYNTH: [obs_dim, obs_dim] row-major */
  const float* K;      /* SYNTH: [obs_dim, act_dim] row-major */
  const float* s0;     /* SYNTH: [obs_dim] reset state */
  const uint8_t* walkable; /* TRAP: [map_h, map_w] 1 = walkable (tile_map.py:40) */
  int32_t map_w, map_h;
  /* SYNTH (fdr 0.4): > 0 = a terminating env -- an episode ends after the step whose next state has
     |s'[done_dim]| > done_threshold (CartPole-style failure; worker/agent.py:50-52: done -> reset, break), or at
     episode_len (the time limit); steps / ret / ent then cover the steps taken.  0 = fixed-length episodes. */
  float done_threshold;
  int32_t done_dim;
} fdr_env_desc;

/* Where each lane's parameter vector comes from:
 *   theta'_l[p] = base[l * base_stride + p] (+ sign_l * fl32(sigma * table[idx_l + p]))
 * base_stride = 0 -> every lane shares theta (the FD case); table = NULL -> no perturbation.
 * Replaces worker/worker.py:26-30 (flat + sigma * noise) without materialising theta'. */
typedef struct fdr_lanes_desc {
  const float* base;
  int64_t base_stride;
  const float* table;   /* shared noise table (utils/noise_sources.py:40), may be NULL */
  int64_t table_size;
  const int64_t* idx;   /* [n_lanes] table offsets, 0 <= idx <= table_size - P */
  const int8_t* sign;   /* [n_lanes] +1 / -1 (antithetic) / 0 (unperturbed, eval lane) */
  float sigma;          /* noise_std */
  const int8_t* deterministic; /* [n_lanes] 1 = argmax/mean action; NULL -> all stochastic */
  int64_t lane_offset;  /* global id of lane 0: keys the action random stream, so a lane draws the
                           same numbers whichever GPU shard evaluates it */
} fdr_lanes_desc;

/* ---- context / errors ----------------------------------------------------------------
 * An fdr_ctx is the engine state of ONE device: the rollout kernel selection (fdr_ctx_set_rollout_impl) and the
 * diagnostics state of include/fdr_diag.h.  Every compute call takes a ctx; the caller's current HIP device must be
 * the ctx's device (FDR_ERR_INVALID otherwise).  A ctx is not shared across threads without external locking; two
 * contexts -- on one device or on two -- are independent.  ctx = NULL selects the process-wide default context
 * (device-agnostic; FDR_ROLLOUT in the environment sets its initial rollout selection, and new contexts copy it). */
const char* fdr_version(void); /* "fdr 0.5 gfx950" (0.5: fdr_impala_bn_refresh, fdr_atari_bn_refresh, fdr_atari_strategies; 0.4:
                                  fdr_env_desc.done_threshold / done_dim) */
const char* fdr_last_error(void);
typedef struct fdr_ctx fdr_ctx;
int fdr_ctx_create(int device, fdr_ctx** out);
int fdr_ctx_destroy(fdr_ctx* ctx);
int fdr_ctx_device(const fdr_ctx* ctx);
/* per-context settings (ctx = NULL: the default context) */
int fdr_ctx_set_rollout_impl(fdr_ctx* ctx, int32_t impl);  /* FDR_ROLLOUT_* below */

/* ---- perturbation batch (worker/worker.py:26-30) ------------------------------------
 * out[l, p] = fl32(theta[p] + sign_l * fl32(fl32(sigma) * table[idx_l + p]))  (no FMA)   */
int fdr_perturb(fdr_ctx* ctx, const float* theta, int64_t n_params, const float* table,
                int64_t table_size, const int64_t* idx, const int8_t* sign, int32_t n_lanes,
                float sigma, float* out, fdr_stream stream);

/* ---- batched policy forward (policies/policy.py:26-29 + discrete.py / mujoco.py) -----
 * One observation per lane: x [n_lanes, n_in].  discrete: out0 = probs [n_lanes, n_act];
 * mujoco: out0 = mean, out1 = std [n_lanes, n_act].  Replaces Policy.forward / get_strategy. */
int fdr_policy_forward(fdr_ctx* ctx, const fdr_policy_desc* policy, const fdr_lanes_desc* lanes,
                       int32_t n_lanes, const float* x, float* out0, float* out1,
                       fdr_stream stream);

/* ---- batched episodes (worker/agent.py:20-71 + worker/worker.py:20-57) ----------------
 * Each lane runs one full episode of env `env` from reset with theta'_l, in ONE launch.
 *   ret   [n_lanes] f64  sum of rewards (+ counter-stream jiggle if `jiggle`, agent.py:69)
 *   ent   [n_lanes] f64  mean per-step policy entropy (discrete.py:26-29 / mujoco.py:24-26)
 *   steps [n_lanes] i32  env.step calls (agent.py:47)
 *   norm2 [n_lanes] f64  ||sign * fl32(sigma * eps_l)||^2, consumed by fdr_fd_weights
 *                        (learner/finite_differences.py:107); NULL allowed
 * obs_mean / obs_std: fixed observation statistics (agent.py:37-41), NULL = no normalisation.
 * seed: key of the counter random stream for stochastic actions. */
int fdr_rollout(fdr_ctx* ctx, const fdr_policy_desc* policy, const fdr_env_desc* env,
                const fdr_lanes_desc* lanes, int32_t n_lanes, uint64_t seed, int32_t jiggle,
                const float* obs_mean, const float* obs_std, double* ret, double* ent,
                int32_t* steps, double* norm2, fdr_stream stream);
/* Rollout kernel selection for the synthetic env (per context, fdr_ctx_set_rollout_impl; fdr_rollout_set_impl
 * sets the default context's; default from the FDR_ROLLOUT environment variable: "pair", "single", else
 * FDR_ROLLOUT_AUTO):
 *   FDR_ROLLOUT_PAIR    two lanes per wave (rollout_pair_kernel)
 *   FDR_ROLLOUT_SINGLE  one lane per wave (rollout_kernel); always used for the trap env and for
 *                       the Welford observation statistics of fdr_rollout_ex
 *   FDR_ROLLOUT_WIDE    one lane per wave with a 256-VGPR budget (rollout_kernel<WIDE>): loop invariants
 *                       in registers, readlane input broadcast, per-action candidate next states
 *   FDR_ROLLOUT_AUTO    the pair kernel when n_lanes >= 16 x CUs (two pair waves per SIMD), wide when
 *                       n_lanes <= 8 x CUs (every lane in one pass at 2 waves per SIMD), else single
 * All compute the same episodes; sums are ordered differently (parity tolerances hold for each).
 * "pair" / "single" / "wide" are also the FDR_ROLLOUT environment variable's values. */
#define FDR_ROLLOUT_PAIR 0
#define FDR_ROLLOUT_SINGLE 1
#define FDR_ROLLOUT_AUTO 2
#define FDR_ROLLOUT_WIDE 3
int fdr_rollout_set_impl(int32_t impl);

/* Same as fdr_rollout, and also writes every visited raw observation (before normalisation) to
 * states [n_lanes, T, n_in] f32 -- Agent.collect_return(save_states=True), worker/agent.py:36,58-59,
 * the eval states run_sequential.py:143 feeds into the novelty probe set zeta. */
int fdr_rollout_states(fdr_ctx* ctx, const fdr_policy_desc* policy, const fdr_env_desc* env,
                       const fdr_lanes_desc* lanes, int32_t n_lanes, uint64_t seed, int32_t jiggle,
                       const float* obs_mean, const float* obs_std, double* ret, double* ent,
                       int32_t* steps, double* norm2, float* states, fdr_stream stream);

/* General form: optional per-lane side outputs of the same episodes (each field NULL = off).
 *   states        [n_lanes, T, n_in] f32  visited raw observations (save_states)
 *   obs_mean/obs_m2 [n_lanes, n_in] f32, obs_count [n_lanes] i32: each lane's WelfordRunningStat
 *                 (utils/math_helpers.py:29-38) of the raw observations sampled with probability
 *                 obs_chance per step (worker/agent.py:37-39; coin = counter stream, k = 14);
 *                 merge them with fdr_obs_stats_merge.
 *   u_inject      [n_lanes, T, k] f32 (nullable; fdr 0.3): host-injected draws replacing the counter stream
 *                 (SURVEY 8b), k = 1 uniform in [0, 1) per step for a DiscretePolicy (inverse CDF,
 *                 policies/discrete.py:16-24) or k = n_act standard normals per step for a MujocoPolicy
 *                 (mean + std * z, policies/mujoco.py:15-22); lane l's step t reads u_inject[(l T + t) k ..];
 *                 deterministic lanes read nothing.  Replays episodes whose torch multinomial / Normal draws
 *                 were recorded (worker/agent.py:43).  Runs the one-lane kernel; not with obs statistics. */
typedef struct fdr_rollout_extras {
  float* states;
  float* obs_mean;
  float* obs_m2;
  int32_t* obs_count;
  float obs_chance;
  const float* u_inject;
} fdr_rollout_extras;
int fdr_rollout_ex(fdr_ctx* ctx, const fdr_policy_desc* policy, const fdr_env_desc* env,
                   const fdr_lanes_desc* lanes, int32_t n_lanes, uint64_t seed, int32_t jiggle,
                   const float* obs_mean, const float* obs_std, double* ret, double* ent, int32_t* steps,
                   double* norm2, const fdr_rollout_extras* extras, fdr_stream stream);

/* ---- noise-table index draw on the HOST (utils/noise_sources.py:44-47) -----------------------------
 * out[i], i < n: the indices n successive RandomState.randint(0, max_idx) calls return, drawn from the MT19937
 * state key [624] u32 / *pos (numpy RandomState.get_state()[1:3]) and advanced in place: 32-bit words masked by
 * the smallest all-ones mask >= max_idx - 1, rejected while > max_idx - 1 (numpy's legacy masked path).  HOST
 * pointers, no device work; FDR_ERR_UNSUPPORTED when max_idx - 1 needs more than 32 bits. */
int fdr_noise_draw_indices(uint32_t* key, int32_t* pos, int64_t max_idx, int32_t n, int64_t* out);

/* ---- obs statistics merge (utils/math_helpers.py:68-87, increment_from_obs_stats_update) --------
 * Folds n partial Welford statistics (mean/m2 [n, dim] f32, count [n] i32, e.g. from
 * fdr_rollout_ex) into the accumulator (acc_mean/acc_m2 [dim] f32, acc_count [1] i64, device,
 * in/out) in index order with the reference's f32 formulas; zero-count partials are skipped. */
int fdr_obs_stats_merge(fdr_ctx* ctx, const float* mean, const float* m2, const int32_t* count, int32_t n, int32_t dim,
                        float* acc_mean, float* acc_m2, int64_t* acc_count, fdr_stream stream);

/* ---- FD weighting (learner/finite_differences.py:40-49, utils/math_helpers.py:127-134) --
 * z = standardize(rewards_all - policy_reward) over ALL n_all lanes (f64, population std,
 * unchanged if std == 0); for the local lanes [lane_lo, lane_lo + n_local):
 *   coef[d] = sum over the lanes_per_dir lanes of direction d of  z_i * sign_i * sigma / norm2_i
 * so that g = sum_d coef[d] * table[idx_d : idx_d + P]  ==  sum_i z_i * lambda_i / ||lambda_i||^2.
 * Lanes with sign 0 contribute nothing (they must not be in rewards_all). */
int fdr_fd_weights(fdr_ctx* ctx, const double* rewards_all, int32_t n_all, double policy_reward,
                   int32_t lane_lo, int32_t n_local, const int8_t* sign_local,
                   const double* norm2_local, int32_t lanes_per_dir, float sigma, double* coef,
                   fdr_stream stream);

/* ---- noise-weighted gradient reduce (learner/finite_differences.py:49) -----------------
 * g[p] = sum_d coef[d] * table[idx[d] + p]   (f64, deterministic order)
 * workspace: device scratch of fdr_fd_grad_workspace_bytes(n_dirs, P) bytes. */
int64_t fdr_fd_grad_workspace_bytes(int32_t n_dirs, int64_t n_params);
int fdr_fd_grad(fdr_ctx* ctx, const float* table, int64_t table_size, const int64_t* idx,
                const double* coef, int32_t n_dirs, int64_t n_params, double* g, void* workspace,
                int64_t workspace_bytes, fdr_stream stream);

/* ---- fused weighting + gradient (one launch; learner/finite_differences.py:40-49) -----------------
 * out = sum over the n_dirs directions d of  coef_d * table[idx_local[d * lpd] : +P]  with the coefficients of
 * fdr_fd_weights formed inside the launch from the weights w_i of the local lanes [lane_lo, +n_dirs*lpd)
 * (idx_local, sign_local, norm2_local: one entry per local lane, lanes of a direction contiguous):
 *   FDR_WEIGHT_ZSCORE         w = standardize(rewards_all - policy_reward) over all n_all lanes (the
 *                             reference, utils/math_helpers.py:127-134); out = g [P] f64
 *   FDR_WEIGHT_CENTERED_RANK  w_i = rank_i / (n_all - 1) - 0.5, rank over rewards_all with ties broken by
 *                             lane index (build extension named by the north star; the standard ES
 *                             centred rank); out = g [P]
 *   FDR_WEIGHT_MOMENTS        the one-collective multi-GPU form of the z-score: rewards_all = the
 *                             n_local LOCAL rewards, n_all = the lanes of all ranks, lane_lo = this rank's
 *                             first global lane; with r' = r - policy_reward, out = [A | B | n_local |
 *                             r' slots [n_all]] (2P + 1 + n_all f64): A = sum_i r'_i v_i, B = sum_i v_i,
 *                             v_i = sign_i sigma eps_i / norm2_i, the slots hold this rank's r' at its
 *                             global lanes and 0 elsewhere.  Summed over ranks (one all-reduce) it holds
 *                             n_all and every lane's r', so fdr_dsgd_step_ex forms m and sd in two passes
 *                             as standardize_arr does and g = (A - m B) / sd (exact in real arithmetic;
 *                             antithetic pairs give B = 0 exactly).
 * Chunk partials are combined inside the launch (deterministic order).  workspace:
 * fdr_fd_grad_fused_workspace_bytes(n_dirs, lanes_per_dir, P, mode) bytes whose first
 * fdr_fd_grad_fused_counter_bytes(n_dirs, P) bytes must be zero before the first call on that workspace
 * (every call leaves them zero). */
#define FDR_WEIGHT_ZSCORE 0
#define FDR_WEIGHT_CENTERED_RANK 1
#define FDR_WEIGHT_MOMENTS 2
int64_t fdr_fd_grad_fused_workspace_bytes(int32_t n_dirs, int32_t lanes_per_dir, int64_t n_params, int32_t mode);
int64_t fdr_fd_grad_fused_counter_bytes(int32_t n_dirs, int64_t n_params);
/* Doubles `out` must hold: P (ZSCORE / CENTERED_RANK) or 2P + 1 + n_all (MOMENTS); -1 for bad arguments.
 * fdr 0.3: out_len (doubles) is checked against it -- the MOMENTS layout was 2P + 3 before 0.3. */
int64_t fdr_fd_grad_fused_out_len(int32_t mode, int64_t n_params, int32_t n_all);
int fdr_fd_grad_fused(fdr_ctx* ctx, const float* table, int64_t table_size, const int64_t* idx_local, int32_t n_dirs,
                      int64_t n_params, const double* rewards_all, int32_t n_all, double policy_reward, int32_t lane_lo,
                      const int8_t* sign_local, const double* norm2_local, int32_t lanes_per_dir, float sigma,
                      int32_t mode, double* out, int64_t out_len, void* workspace, int64_t workspace_bytes,
                      fdr_stream stream);
/* The whole single-process FD step (FiniteDifferences.step, learner/finite_differences.py:24-64, with DSGD
 * dynamic_sgd.py:19-39) in two launches: fdr_fd_grad_fused (mode ZSCORE or CENTERED_RANK over all n_all =
 * n_dirs * lanes_per_dir lanes) writing g [P] and each column block's sum fl32(-g)^2, then the DSGD update of
 * theta as fdr_dsgd_step (one workgroup per 256 parameters).  theta_hist [P] (nullable) receives the updated
 * theta (the learner's policy_history entry, finite_differences.py:75-78) without a separate copy.
 * out = [||d theta||, ||grad||].  workspace as fdr_fd_grad_fused. */
int fdr_fd_step(fdr_ctx* ctx, const float* table, int64_t table_size, const int64_t* idx_local, int32_t n_dirs,
                int64_t n_params, const double* rewards_all, int32_t n_all, double policy_reward,
                const int8_t* sign_local, const double* norm2_local, int32_t lanes_per_dir, float sigma, int32_t mode,
                float* theta, double lr, double lr_scale, double* g, float* theta_hist, double* out, void* workspace,
                int64_t workspace_bytes, fdr_stream stream);
/* The centred-rank weights alone: w [n_local] f64 for lanes [lane_lo, lane_lo + n_local) of rewards_all. */
int fdr_rank_weights(fdr_ctx* ctx, const double* rewards_all, int32_t n_all, int32_t lane_lo, int32_t n_local,
                     double* w, fdr_stream stream);

/* ---- delayed returns: lambda with policy drift (learner/finite_differences.py:66-73, 80-114) -----
 * Return i's perturbation lambda_i = fl32(sign_i * fl32(sigma * table[idx_i + p]) + D[slot_i][p]),
 * D = drift [n_slots, P] f32 (dist_map: theta of the return's epoch minus the current theta;
 * slot_i < 0 or slot == NULL: the current epoch, D = 0; sign == NULL: +1).
 *   fdr_fd_lambda_norms: norm2[i] = ||lambda_i||^2 (f64); NaN for an out-of-range offset.
 *   fdr_fd_grad_lambda:  g[p] = sum_i coef[i] * lambda_i[p] (f64, fixed order); with
 *                        coef = fdr_fd_weights(sign = +1, sigma = 1, lanes_per_dir = 1) this is
 *                        np.dot(z, lambda / ||lambda||^2).  workspace: fdr_fd_grad_workspace_bytes(n, P). */
int fdr_fd_lambda_norms(fdr_ctx* ctx, const float* table, int64_t table_size, const int64_t* idx, const int8_t* sign,
                        const int32_t* slot, int32_t n, int64_t n_params, float sigma, const float* drift,
                        int32_t n_slots, double* norm2, fdr_stream stream);
int fdr_fd_grad_lambda(fdr_ctx* ctx, const float* table, int64_t table_size, const int64_t* idx, const int8_t* sign,
                       const int32_t* slot, const double* coef, int32_t n, int64_t n_params, float sigma,
                       const float* drift, int32_t n_slots, double* g, void* workspace, int64_t workspace_bytes,
                       fdr_stream stream);

/* ---- BN running-stat refresh (policies/policy.py:31-34 compute_vbn, run_sequential.py:156-157) ------
 * DiscretePolicy only (the policy with BatchNorm1d layers): one train-mode pass of the buffer
 * x [n, n_in] through BN0-L1-ReLU-BN1-L2-ReLU-BN2 with theta; every BN normalises with its batch
 * statistics (biased variance) and updates its running stats in place:
 *   rm <- momentum * mean + (1 - momentum) * rm,  rv <- momentum * var * n / (n - 1) + (1 - momentum) * rv
 * bn_mean / bn_var: the [n_in | 64 | 64] f32 stats of fdr_policy_desc (torch momentum = 0.1); n >= 2.
 * workspace: fdr_bn_refresh_workspace_bytes(n) bytes. */
int64_t fdr_bn_refresh_workspace_bytes(int32_t n);
int fdr_bn_refresh(fdr_ctx* ctx, const fdr_policy_desc* policy, const float* theta, const float* x, int32_t n,
                   float momentum, float* bn_mean, float* bn_var, void* workspace, int64_t workspace_bytes,
                   fdr_stream stream);

/* ---- DSGD update (dsgd/dynamic_sgd.py:19-51, policies/policy.py:63-70) -----------------
 * grad = fl32(-g); norm = ||grad||; coef = lr * sqrt(P) * lr_scale / norm;
 * theta <- fl32(theta - fl32(fl32(coef) * grad)).
 * out[0] = ||theta_old - theta_new|| (learner/finite_differences.py:59), out[1] = ||grad||
 * (0 -> the reference's `assert norm > 0` failed; theta is left unchanged).  out: device f64[2].
 * workspace: fdr_dsgd_workspace_bytes(P) bytes. */
int64_t fdr_dsgd_workspace_bytes(int64_t n_params);
int fdr_dsgd_step(fdr_ctx* ctx, float* theta, const double* g, int64_t n_params, double lr,
                  double lr_scale, double* out, void* workspace, int64_t workspace_bytes,
                  fdr_stream stream);

/* DSGD from a gradient or from the summed moments of FDR_WEIGHT_MOMENTS (src_is_moments = 1: g = (A - m B) /
 * sd with m, sd the two-pass mean / population std of the n r' slots; sd == 0 -> g = A, as standardize_arr; g is
 * written to g_out).
 * P <= 65536: one fused launch (norm + update + ||d theta||).  out, workspace as fdr_dsgd_step. */
int fdr_dsgd_step_ex(fdr_ctx* ctx, float* theta, const double* src, int32_t src_is_moments, int64_t n_params,
                     double lr, double lr_scale, double* g_out, double* out, void* workspace, int64_t workspace_bytes,
                     fdr_stream stream);

/* ---- strategy distances / novelty (utils/math_helpers.py:147-222, strategy/) -----------------
 * strategies [n, Z, D] f32 = get_strategy over the Z probe states for n policies (e.g. every
 * perturbed lane); archive [H, Z, D] f32.  d[i][h] = mean over z of
 *   FDR_DIST_L2   || b - a ||_2                                   (l2_dist :166-170)
 *   FDR_DIST_TVD  sum_d |a - b|                                   (categorical_tvd :216-219)
 *   FDR_DIST_W2   ||m_a - m_b||^2 + sum(s_a + s_b - 2 sqrt(s_a s_b)), D = 2k = [mean | std]
 *                 (gaussian_wasserstein_dist_from_strategies :202-213)
 * f64 accumulation.  Outputs (each nullable): dists [n, H] f64; min_dist [n] f64 = the novelty of
 * compute_strategy_novelty (:147-155); argmin [n] i32 (first minimum).  Z * D <= 8192. */
#define FDR_DIST_L2 0
#define FDR_DIST_TVD 1
#define FDR_DIST_W2 2
int fdr_strategy_distances(fdr_ctx* ctx, const float* strategies, int32_t n, const float* archive, int32_t n_archive,
                           int32_t n_states, int32_t dim, int32_t kind, double* dists, double* min_dist,
                           int32_t* argmin, fdr_stream stream);

/* ---- ImpalaPolicy (policies/impala.py:8-186) on the synthetic frame env --------------------
 * The IMPALA conv stack runs on f32 MFMA tiles (one workgroup per env, activations resident in
 * LDS), the fc + LSTM + head per lane; theta'_l is gathered once per rollout into a per-lane
 * pack in the workspace.  Frames: uint8-valued 3x64x64 counter-hash frames and a +-1/0 reward
 * (DESIGN.md "Impala path"; oracle/impala.py restates both). */
typedef struct fdr_impala_desc {
  int32_t n_act;         /* A = policy output size (env action_space.n), 1..32 */
  int32_t envs_per_lane; /* E in {1, 2, 4, 8}: envs evaluated with one theta' (BASELINE config 4) */
  int32_t episode_len;   /* T: fixed-length synthetic episodes */
  int32_t entropy;       /* 1 = the reference's end-of-episode entropy pass (worker/agent.py:60-66):
                            every visited obs replayed through the LSTM from the final state;
                            0 = skip it (ent = 0) */
  uint64_t env_seed;     /* synthetic frame / reward stream */
  int64_t n_params;      /* must equal fdr_impala_num_params(n_act) */
  const float* bn_mean;  /* eval-mode BN running stats, modules() order, concatenated:
                            fdr_impala_num_bn_stats() floats; NULL = mean 0 */
  const float* bn_var;   /* NULL = var 1 */
  int32_t fp16;          /* 1 = fp16 mode (BASELINE config 5): theta' rounded to f16 for the convs, fc and
                            LSTM; f16 activations in the conv stack on f16 MFMA, f32 accumulation, state
                            and head (DESIGN.md "fp16 mode"); 0 = f32 throughout */
  int32_t pairs;         /* 1 = lanes 2p, 2p+1 are an antithetic pair (same table offset -- a pair whose
                            offsets differ reports norm2 = NaN on both lanes; each sign +-1 or 0 -- a sign-0
                            lane runs theta; n_lanes even; E <= 4) -- the rollout's fc / LSTM step streams the pair's
                            fl32(sigma eps) once and theta's shared pack, forming each lane's weights in
                            registers (half the core kernel's HBM bytes; f32: the per-lane
                            weights bit for bit, fp16: f16(theta) + s f16(sigma eps)); 0 = per lane */
} fdr_impala_desc;

/* len(ImpalaPolicy.get_trainable_flat()) for n_act actions; -1 if n_act is out of range. */
int64_t fdr_impala_num_params(int32_t n_act);
/* total number of BatchNorm running-mean (= running-var) entries of the ImpalaCNN */
int64_t fdr_impala_num_bn_stats(void);

/* Each lane l evaluates theta'_l (lanes desc as for fdr_rollout) on envs l*E .. l*E+E-1, each one
 * full episode from reset, returns laid out [n_lanes * E] (lane-major):
 *   ret, ent (f64), steps (i32) per env; norm2 [n_lanes] f64 per lane;
 *   actions [n_lanes*E, T] i32 and probs [n_lanes*E, T, A] f32 optional (NULL) per-step traces.
 * workspace: fdr_impala_workspace_bytes(desc, n_lanes) bytes (theta' packs + per-step state).
 * Replaces Worker.collect_returns with an ImpalaPolicy (worker/worker.py:20-38). */
int64_t fdr_impala_workspace_bytes(const fdr_impala_desc* desc, int32_t n_lanes);
int fdr_impala_rollout(fdr_ctx* ctx, const fdr_impala_desc* desc, const fdr_lanes_desc* lanes,
                       int32_t n_lanes, uint64_t seed, int32_t jiggle, double* ret, double* ent,
                       int32_t* steps, double* norm2, int32_t* actions, float* probs, void* workspace,
                       int64_t workspace_bytes, fdr_stream stream);

/* ---- AtariPolicy (policies/atari.py:7-51) on the synthetic stacked-frame env ------------
 * 4 x 84 x 84 counter-hash frames (oracle/atari.py), the reward of the Impala frame env; conv 8x8 s4 and
 * 4x4 s2 on f32 MFMA with BN + ReLU in LDS, fc 2592 -> 256 + BN1d + ReLU + head per lane.
 * bn_mean / bn_var: running stats [16 | 32 | 256] (NULL = 0 / 1).  Outputs as fdr_impala_rollout;
 * entropy = mean per-step Categorical entropy (stateless policy).  envs_per_lane in {1, 2, 4}. */
typedef struct fdr_atari_desc {
  int32_t n_act;
  int32_t envs_per_lane;
  int32_t episode_len;
  int32_t reserved;
  uint64_t env_seed;
  int64_t n_params;       /* must equal fdr_atari_num_params(n_act) */
  const float* bn_mean;
  const float* bn_var;
} fdr_atari_desc;
int64_t fdr_atari_num_params(int32_t n_act);
int64_t fdr_atari_workspace_bytes(const fdr_atari_desc* desc, int32_t n_lanes);
int fdr_atari_rollout(fdr_ctx* ctx, const fdr_atari_desc* desc, const fdr_lanes_desc* lanes, int32_t n_lanes,
                      uint64_t seed, int32_t jiggle, double* ret, double* ent, int32_t* steps, double* norm2,
                      int32_t* actions, float* probs, void* workspace, int64_t workspace_bytes, fdr_stream stream);
/* AtariPolicy.forward for n frames [n, 4, 84, 84] (f32, raw 0..255 as the reference feeds them):
 * probs [n, A]; feat [n, 2592] optional.  workspace: fdr_atari_forward_workspace_bytes(n_act, n). */
/* The synthetic stacked-frame env's observations [n, 4, 84, 84] f32 (0..255) of global env env_id (= lane_offset * E
 * + lane * E + e of a rollout) at steps t0 .. t0+n-1 -- the frames do not depend on the actions.  The eval states
 * (worker/agent.py:36,58-59) that become zeta for AtariPolicy novelty (run_sequential.py:142-143). */
int fdr_atari_env_frames(uint64_t env_seed, int64_t env_id, int32_t t0, int32_t n, float* frames, fdr_stream stream);
int64_t fdr_atari_forward_workspace_bytes(int32_t n_act, int32_t n);
int fdr_atari_forward(fdr_ctx* ctx, const fdr_atari_desc* desc, const float* theta, int32_t n, const float* frames,
                      float* probs, float* feat, void* workspace, int64_t workspace_bytes, fdr_stream stream);

/* AtariPolicy.compute_vbn (policies/policy.py:31-34 on atari.py:36-51): one train-mode pass of the VBN buffer of
 * n >= 2 frames [n, 4, 84, 84] f32 (raw 0..255).  Each of the three BatchNorms (2d(16), 2d(32), 1d(256))
 * normalises with its batch statistics (biased variance, double accumulation) and updates its running stats in place
 * in bn_mean / bn_var [16 | 32 | 256] (rm <- momentum * mean + (1 - momentum) * rm, rv with the unbiased variance);
 * the head feeds no statistic.  Only n_act and n_params of desc are read.
 * workspace: fdr_atari_bn_refresh_workspace_bytes(n) bytes (~2.9 MB + 37 KB per frame). */
int64_t fdr_atari_bn_refresh_workspace_bytes(int32_t n);
int fdr_atari_bn_refresh(fdr_ctx* ctx, const fdr_atari_desc* desc, const float* theta, int32_t n, const float* frames,
                         float momentum, float* bn_mean, float* bn_var, void* workspace, int64_t workspace_bytes,
                         fdr_stream stream);

/* AtariPolicy.get_strategy (policies/atari.py:30-31) of every lane's theta'_l (lanes as for fdr_atari_rollout) over
 * Z shared probe frames [Z, 4, 84, 84] f32 (0..255): probs [n_lanes, Z, A] -- the lane novelty's strategies
 * (worker/worker.py:53, strategy/strategy_handler.py:25-30) in one prep / conv / core launch per 256 lanes.
 * workspace: fdr_atari_strategies_workspace_bytes(desc, n_lanes, Z) bytes. */
int64_t fdr_atari_strategies_workspace_bytes(const fdr_atari_desc* desc, int32_t n_lanes, int32_t n_states);
int fdr_atari_strategies(fdr_ctx* ctx, const fdr_atari_desc* desc, const fdr_lanes_desc* lanes, int32_t n_lanes,
                         int32_t n_states, const float* frames, float* probs, void* workspace, int64_t workspace_bytes,
                         fdr_stream stream);

/* One step of ImpalaPolicy.forward (policies/impala.py:18-19, 144-186) for n_envs independent
 * envs sharing theta [P]: frames [n_envs, 3, 64, 64] f32 (0..255), reward [n_envs] (NULL = 0),
 * notdone [n_envs] (NULL = 1; multiplies the incoming state), h / c [n_envs, 256] updated in
 * place, probs [n_envs, A] out, feat [n_envs, 2048] out (optional: relu'd conv features).
 * Only desc->n_act, n_params, bn_mean, bn_var are read.
 * workspace: fdr_impala_forward_workspace_bytes(n_act, n_envs) bytes. */
int64_t fdr_impala_forward_workspace_bytes(int32_t n_act, int32_t n_envs, int32_t fp16);
int fdr_impala_forward(fdr_ctx* ctx, const fdr_impala_desc* desc, const float* theta, int32_t n_envs,
                       const float* frames, const float* reward, const float* notdone, float* h,
                       float* c, float* probs, float* feat, void* workspace, int64_t workspace_bytes,
                       fdr_stream stream);

/* ImpalaPolicy.get_strategy over a probe set (policies/impala.py:24-27, strategy/strategy_point.py:17-25,
 * strategy/strategy_handler.py:25-31) for every lane's theta'_l: the Z stacked obs run through the network as
 * ONE batch_first LSTM sequence (B = 1, T = Z, policies/impala.py:118, 161-176), exactly as the reference's
 * _get_stacked_obs batch does.  frames [Z, 3, 64, 64] f32 (0..255) and reward [Z] (NULL = 0) are shared by
 * all lanes; h / c [n_lanes, 256] = the state the sequence starts from, updated in place to its end state
 * (NULL = the reset state, which is the state Worker._build_ret scores novelty in: worker/agent.py:66 resets
 * the policy before compute_novelty).  probs [n_lanes, Z, A] f32 out.  Only n_act, n_params, fp16, pairs, bn_mean,
 * bn_var of desc are read; fp16 with pairs (lanes as for fdr_impala_rollout, n_lanes % 4 == 0, ctx core_mfma >= 1)
 * runs the recurrence in the rollout's pair form on MFMA; a pair whose two lanes carry different table offsets then
 * gets NaN probabilities on both lanes (it would otherwise run lane 2p + 1 on lane 2p's noise).
 * workspace: fdr_impala_strategies_workspace_bytes(desc, n_lanes, Z) bytes. */
int64_t fdr_impala_strategies_workspace_bytes(const fdr_impala_desc* desc, int32_t n_lanes, int32_t n_states);
int fdr_impala_strategies(fdr_ctx* ctx, const fdr_impala_desc* desc, const fdr_lanes_desc* lanes, int32_t n_lanes,
                          int32_t n_states, const float* frames, const float* reward, float* h, float* c,
                          float* probs, void* workspace, int64_t workspace_bytes, fdr_stream stream);

/* ImpalaPolicy.compute_vbn (policies/impala.py:12-16, run_sequential.py:156-157): one train-mode pass of the VBN
 * buffer of n >= 2 obs -- frames [n, 3, 64, 64] f32 (0..255), reward [n] (NULL = 0) -- stacked as the reference
 * stacks them (B = n, T = 1).  Every BatchNorm normalises with its batch statistics (biased variance; double
 * accumulation) and updates its running stats in place, in modules() order as fdr_impala_desc.bn_mean:
 *   rm <- momentum * mean + (1 - momentum) * rm,  rv <- momentum * var * N / (N - 1) + (1 - momentum) * rv
 * (N = n * H * W per channel); the LSTM reads the n obs as ONE sequence from the carried state h / c [256]
 * (in/out; NULL = zero state, not written), zeroed first iff first_done (the first obs' done flag,
 * impala.py:165-176), and h / c receive the end-of-sequence state (impala.py:184).  Only n_act and n_params of
 * desc are read.  workspace: fdr_impala_bn_refresh_workspace_bytes(n) bytes (~0.4 MB per obs). */
int64_t fdr_impala_bn_refresh_workspace_bytes(int32_t n);
int fdr_impala_bn_refresh(fdr_ctx* ctx, const fdr_impala_desc* desc, const float* theta, int32_t n,
                          const float* frames, const float* reward, int32_t first_done, float* h, float* c,
                          float momentum, float* bn_mean, float* bn_var, void* workspace, int64_t workspace_bytes,
                          fdr_stream stream);

/* Observations of the synthetic frame env outside a rollout (eval states and the probe set zeta,
 * run_sequential.py:142-143, 198-213): frames [n, 3, 64, 64] f32 (0..255) of global env `env_id`
 * (= lane_offset * E + lane * E + e of a rollout) at steps t0 .. t0+n-1, and -- given the actions [n] i32
 * taken at those steps (NULL -> 0) -- reward [n] f32 (nullable) that each step returns. */
int fdr_impala_env_frames(uint64_t env_seed, int32_t n_act, int64_t env_id, int32_t t0, int32_t n,
                          const int32_t* actions, float* frames, float* reward, fdr_stream stream);

#ifdef __cplusplus
}
#endif
#endif /* FDR_H_ */
