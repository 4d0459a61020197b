"""ctypes binding of libfdr.so (include/fdr.h) -- the only path to the HIP kernels.

There is deliberately no fallback: if libfdr.so is missing or cannot be loaded, importing this
module raises, and every product call that needs the GPU fails loudly.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FDR_LIB", os.path.join(_HERE, "libfdr.so"))

FDR_OK, FDR_ERR_INVALID, FDR_ERR_UNSUPPORTED, FDR_ERR_HIP, FDR_ERR_WORKSPACE = 0, 1, 2, 3, 4
FDR_POLICY_DISCRETE, FDR_POLICY_MUJOCO = 0, 1
FDR_ENV_SYNTH, FDR_ENV_TRAP = 0, 1
FDR_DIST_L2, FDR_DIST_TVD, FDR_DIST_W2 = 0, 1, 2
FDR_ROLLOUT_PAIR, FDR_ROLLOUT_SINGLE, FDR_ROLLOUT_AUTO, FDR_ROLLOUT_WIDE = 0, 1, 2, 3
FDR_WEIGHT_ZSCORE, FDR_WEIGHT_CENTERED_RANK, FDR_WEIGHT_MOMENTS = 0, 1, 2

EXPORTS = ("fdr_version", "fdr_last_error", "fdr_ctx_create", "fdr_ctx_destroy", "fdr_ctx_device",
           "fdr_perturb", "fdr_policy_forward", "fdr_rollout", "fdr_fd_weights",
           "fdr_fd_grad_workspace_bytes", "fdr_fd_grad", "fdr_dsgd_workspace_bytes", "fdr_dsgd_step",
           "fdr_impala_num_params", "fdr_impala_num_bn_stats", "fdr_impala_workspace_bytes",
           "fdr_impala_rollout", "fdr_impala_forward_workspace_bytes", "fdr_impala_forward",
           "fdr_impala_profile", "fdr_impala_profile_read", "fdr_impala_debug_clock",
           "fdr_strategy_distances", "fdr_rollout_states", "fdr_rollout_ex", "fdr_obs_stats_merge",
           "fdr_fd_lambda_norms", "fdr_fd_grad_lambda", "fdr_bn_refresh_workspace_bytes", "fdr_bn_refresh",
           "fdr_atari_num_params", "fdr_atari_workspace_bytes", "fdr_atari_rollout",
           "fdr_atari_forward_workspace_bytes", "fdr_atari_forward", "fdr_atari_env_frames", "fdr_rollout_set_impl",
           "fdr_impala_set_replay_gemm", "fdr_impala_strategies_workspace_bytes", "fdr_impala_strategies",
           "fdr_impala_env_frames", "fdr_fd_grad_fused_workspace_bytes", "fdr_fd_grad_fused_counter_bytes",
           "fdr_fd_grad_fused_out_len",
           "fdr_fd_grad_fused", "fdr_rank_weights", "fdr_dsgd_step_ex", "fdr_fd_step",
           "fdr_ctx_set_rollout_impl", "fdr_ctx_set_replay_gemm", "fdr_ctx_impala_profile",
           "fdr_ctx_impala_profile_read", "fdr_ctx_impala_debug_clock", "fdr_noise_draw_indices",
           "fdr_impala_bn_refresh_workspace_bytes", "fdr_impala_bn_refresh", "fdr_atari_strategies_workspace_bytes",
           "fdr_atari_strategies", "fdr_atari_bn_refresh_workspace_bytes", "fdr_atari_bn_refresh")


class FDRError(RuntimeError):
    pass


class PolicyDesc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("n_in", ctypes.c_int32), ("n_act", ctypes.c_int32),
                ("hidden", ctypes.c_int32), ("n_params", ctypes.c_int64),
                ("bn_mean", ctypes.c_void_p), ("bn_var", ctypes.c_void_p)]


class EnvDesc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("obs_dim", ctypes.c_int32), ("act_dim", ctypes.c_int32),
                ("episode_len", ctypes.c_int32), ("M", ctypes.c_void_p), ("K", ctypes.c_void_p),
                ("s0", ctypes.c_void_p), ("walkable", ctypes.c_void_p), ("map_w", ctypes.c_int32),
                ("map_h", ctypes.c_int32), ("done_threshold", ctypes.c_float), ("done_dim", ctypes.c_int32)]


class LanesDesc(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("base_stride", ctypes.c_int64), ("table", ctypes.c_void_p),
                ("table_size", ctypes.c_int64), ("idx", ctypes.c_void_p), ("sign", ctypes.c_void_p),
                ("sigma", ctypes.c_float), ("deterministic", ctypes.c_void_p), ("lane_offset", ctypes.c_int64)]


class RolloutExtras(ctypes.Structure):
    _fields_ = [("states", ctypes.c_void_p), ("obs_mean", ctypes.c_void_p), ("obs_m2", ctypes.c_void_p),
                ("obs_count", ctypes.c_void_p), ("obs_chance", ctypes.c_float), ("u_inject", ctypes.c_void_p)]


class AtariDesc(ctypes.Structure):
    _fields_ = [("n_act", ctypes.c_int32), ("envs_per_lane", ctypes.c_int32), ("episode_len", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("env_seed", ctypes.c_uint64), ("n_params", ctypes.c_int64),
                ("bn_mean", ctypes.c_void_p), ("bn_var", ctypes.c_void_p)]


class ImpalaDesc(ctypes.Structure):
    _fields_ = [("n_act", ctypes.c_int32), ("envs_per_lane", ctypes.c_int32), ("episode_len", ctypes.c_int32),
                ("entropy", ctypes.c_int32), ("env_seed", ctypes.c_uint64), ("n_params", ctypes.c_int64),
                ("bn_mean", ctypes.c_void_p), ("bn_var", ctypes.c_void_p), ("fp16", ctypes.c_int32),
                ("pairs", ctypes.c_int32)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("libfdr.so not found at %s -- build it with `python -c 'import __graft_entry__ as g; "
                          "g.build()'` (or `make -C dfd-starter_amd/csrc`)" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    P, I32, I64, F32, F64, U64 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float,
                                  ctypes.c_double, ctypes.c_uint64)
    sig = {
        "fdr_version": (ctypes.c_char_p, []),
        "fdr_last_error": (ctypes.c_char_p, []),
        "fdr_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
        "fdr_ctx_destroy": (ctypes.c_int, [P]),
        "fdr_ctx_device": (ctypes.c_int, [P]),
        "fdr_perturb": (ctypes.c_int, [P, P, I64, P, I64, P, P, I32, F32, P, P]),
        "fdr_policy_forward": (ctypes.c_int, [P, ctypes.POINTER(PolicyDesc), ctypes.POINTER(LanesDesc), I32, P,
                                              P, P, P]),
        "fdr_rollout": (ctypes.c_int, [P, ctypes.POINTER(PolicyDesc), ctypes.POINTER(EnvDesc),
                                       ctypes.POINTER(LanesDesc), I32, U64, I32, P, P, P, P, P, P, P]),
        "fdr_rollout_states": (ctypes.c_int, [P, ctypes.POINTER(PolicyDesc), ctypes.POINTER(EnvDesc),
                                              ctypes.POINTER(LanesDesc), I32, U64, I32, P, P, P, P, P, P, P, P]),
        "fdr_rollout_ex": (ctypes.c_int, [P, ctypes.POINTER(PolicyDesc), ctypes.POINTER(EnvDesc),
                                          ctypes.POINTER(LanesDesc), I32, U64, I32, P, P, P, P, P, P,
                                          ctypes.POINTER(RolloutExtras), P]),
        "fdr_obs_stats_merge": (ctypes.c_int, [P, P, P, P, I32, I32, P, P, P, P]),
        "fdr_noise_draw_indices": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_int32), I64, I32, P]),
        "fdr_fd_lambda_norms": (ctypes.c_int, [P, P, I64, P, P, P, I32, I64, F32, P, I32, P, P]),
        "fdr_fd_grad_lambda": (ctypes.c_int, [P, P, I64, P, P, P, P, I32, I64, F32, P, I32, P, P, I64, P]),
        "fdr_bn_refresh_workspace_bytes": (I64, [I32]),
        "fdr_bn_refresh": (ctypes.c_int, [P, ctypes.POINTER(PolicyDesc), P, P, I32, F32, P, P, P, I64, P]),
        "fdr_atari_num_params": (I64, [I32]),
        "fdr_atari_workspace_bytes": (I64, [ctypes.POINTER(AtariDesc), I32]),
        "fdr_atari_rollout": (ctypes.c_int, [P, ctypes.POINTER(AtariDesc), ctypes.POINTER(LanesDesc), I32, U64, I32,
                                             P, P, P, P, P, P, P, I64, P]),
        "fdr_atari_forward_workspace_bytes": (I64, [I32, I32]),
        "fdr_atari_forward": (ctypes.c_int, [P, ctypes.POINTER(AtariDesc), P, I32, P, P, P, P, I64, P]),
        "fdr_atari_strategies_workspace_bytes": (I64, [ctypes.POINTER(AtariDesc), I32, I32]),
        "fdr_atari_strategies": (ctypes.c_int, [P, ctypes.POINTER(AtariDesc), ctypes.POINTER(LanesDesc), I32, I32, P, P,
                                                P, I64, P]),
        "fdr_atari_bn_refresh_workspace_bytes": (I64, [I32]),
        "fdr_atari_bn_refresh": (ctypes.c_int, [P, ctypes.POINTER(AtariDesc), P, I32, P, F32, P, P, P, I64, P]),
        "fdr_rollout_set_impl": (ctypes.c_int, [I32]),
        "fdr_ctx_set_rollout_impl": (ctypes.c_int, [P, I32]),
        "fdr_ctx_set_replay_gemm": (ctypes.c_int, [P, I32]),
        "fdr_ctx_impala_profile": (ctypes.c_int, [P, I32]),
        "fdr_ctx_impala_profile_read": (ctypes.c_int, [P, P]),
        "fdr_ctx_impala_debug_clock": (ctypes.c_int, [P, P]),
        "fdr_impala_set_replay_gemm": (ctypes.c_int, [I32]),
        "fdr_fd_weights": (ctypes.c_int, [P, P, I32, F64, I32, I32, P, P, I32, F32, P, P]),
        "fdr_fd_grad_workspace_bytes": (I64, [I32, I64]),
        "fdr_fd_grad": (ctypes.c_int, [P, P, I64, P, P, I32, I64, P, P, I64, P]),
        "fdr_dsgd_workspace_bytes": (I64, [I64]),
        "fdr_fd_grad_fused_workspace_bytes": (I64, [I32, I32, I64, I32]),
        "fdr_fd_grad_fused_counter_bytes": (I64, [I32, I64]),
        "fdr_fd_grad_fused_out_len": (I64, [I32, I64, I32]),
        "fdr_fd_grad_fused": (ctypes.c_int, [P, P, I64, P, I32, I64, P, I32, F64, I32, P, P, I32, F32, I32, P, I64, P,
                                             I64, P]),
        "fdr_rank_weights": (ctypes.c_int, [P, P, I32, I32, I32, P, P]),
        "fdr_fd_step": (ctypes.c_int, [P, P, I64, P, I32, I64, P, I32, F64, P, P, I32, F32, I32, P, F64, F64, P, P, P,
                                       P, I64, P]),
        "fdr_dsgd_step_ex": (ctypes.c_int, [P, P, P, I32, I64, F64, F64, P, P, P, I64, P]),
        "fdr_dsgd_step": (ctypes.c_int, [P, P, P, I64, F64, F64, P, P, I64, P]),
        "fdr_atari_env_frames": (ctypes.c_int, [ctypes.c_uint64, I64, I32, I32, P, P]),
        "fdr_impala_num_params": (I64, [I32]),
        "fdr_impala_num_bn_stats": (I64, []),
        "fdr_impala_bn_refresh_workspace_bytes": (I64, [I32]),
        "fdr_impala_bn_refresh": (ctypes.c_int, [P, ctypes.POINTER(ImpalaDesc), P, I32, P, P, I32, P, P, F32, P, P, P,
                                                 I64, P]),
        "fdr_impala_workspace_bytes": (I64, [ctypes.POINTER(ImpalaDesc), I32]),
        "fdr_impala_rollout": (ctypes.c_int, [P, ctypes.POINTER(ImpalaDesc), ctypes.POINTER(LanesDesc), I32, U64,
                                              I32, P, P, P, P, P, P, P, I64, P]),
        "fdr_impala_forward_workspace_bytes": (I64, [I32, I32, I32]),
        "fdr_impala_env_frames": (ctypes.c_int, [U64, I32, I64, I32, I32, P, P, P, P]),
        "fdr_impala_strategies_workspace_bytes": (I64, [ctypes.POINTER(ImpalaDesc), I32, I32]),
        "fdr_impala_strategies": (ctypes.c_int, [P, ctypes.POINTER(ImpalaDesc), ctypes.POINTER(LanesDesc), I32, I32,
                                                 P, P, P, P, P, P, I64, P]),
        "fdr_impala_profile": (ctypes.c_int, [I32]),
        "fdr_impala_profile_read": (ctypes.c_int, [P]),
        "fdr_impala_debug_clock": (ctypes.c_int, [P]),
        "fdr_strategy_distances": (ctypes.c_int, [P, P, I32, P, I32, I32, I32, I32, P, P, P, P]),
        "fdr_impala_forward": (ctypes.c_int, [P, ctypes.POINTER(ImpalaDesc), P, I32, P, P, P, P, P, P, P, P, I64,
                                              P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc, what=""):
    if rc != FDR_OK:
        msg = lib.fdr_last_error().decode(errors="replace")
        raise FDRError("%s failed (code %d): %s" % (what, rc, msg))


def version():
    return lib.fdr_version().decode()
