"""Device-level operations of the FD engine: thin torch-tensor wrappers over the C ABI.

PyTorch-ROCm is plumbing here (device memory, streams, torch.distributed); every computation
runs in libfdr.so.  All calls are asynchronous on the current HIP stream.
"""
import ctypes

import torch

from . import _lib
from ._lib import check, lib


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(device=None):
    """The current HIP stream of `device` as a C pointer (torch's raw-stream accessor: a few us cheaper per call
    than building the Stream object)."""
    if _RAW_STREAM is not None:
        if isinstance(device, torch.device) and device.index is not None:
            idx = device.index
        elif isinstance(device, int):
            idx = device
        else:
            idx = torch.cuda.current_device() if device is None else torch.device(device).index
            idx = torch.cuda.current_device() if idx is None else idx
        return ctypes.c_void_p(_RAW_STREAM(idx))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Context(object):
    """One fdr_ctx (include/fdr.h): the engine state of one device -- rollout kernel selection, Impala phase
    profiling, replay GEMM switch, debug clocks.  engine.context(device) holds the default one per device;
    further contexts are independent (e.g. two rollout selections side by side in one process)."""

    def __init__(self, device=None):
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        h = ctypes.c_void_p()
        check(lib.fdr_ctx_create(int(dev.index), ctypes.byref(h)), "fdr_ctx_create")
        self.handle = h

    def set_rollout_impl(self, impl):
        """"pair" | "single" | "wide" | "auto" (FDR_ROLLOUT_*)."""
        code = {"pair": _lib.FDR_ROLLOUT_PAIR, "single": _lib.FDR_ROLLOUT_SINGLE, "auto": _lib.FDR_ROLLOUT_AUTO,
                "wide": _lib.FDR_ROLLOUT_WIDE}[impl]
        check(lib.fdr_ctx_set_rollout_impl(self.handle, code), "fdr_ctx_set_rollout_impl")

    def set_replay_gemm(self, on):
        """Diagnostics (include/fdr_diag.h): the entropy replay's input projection as a GEMM per chunk (default) or
        streamed per step -- bit-identical gates."""
        check(lib.fdr_ctx_set_replay_gemm(self.handle, 1 if on else 0), "fdr_ctx_set_replay_gemm")

    def impala_profile(self, enable):
        check(lib.fdr_ctx_impala_profile(self.handle, 1 if enable else 0), "fdr_ctx_impala_profile")

    def impala_profile_read(self):
        out = (ctypes.c_double * 3)()
        check(lib.fdr_ctx_impala_profile_read(self.handle, ctypes.cast(out, ctypes.c_void_p)),
              "fdr_ctx_impala_profile_read")
        return tuple(out)

    def impala_debug_clock(self, buf):
        check(lib.fdr_ctx_impala_debug_clock(self.handle, None if buf is None else ctypes.c_void_p(buf.data_ptr())),
              "fdr_ctx_impala_debug_clock")

    def __del__(self):
        try:
            lib.fdr_ctx_destroy(self.handle)
        except Exception:
            pass


_CTX = {}


def context(device=None):
    """The engine's context of `device` (created on first use)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    c = _CTX.get(dev)
    if c is None:
        c = _CTX[dev] = Context(dev)
    return c


def _c(device=None, ctx=None):
    return (ctx if ctx is not None else context(device)).handle


class PolicySpec(object):
    """Shape of a policy family (policies/discrete.py:34-48, policies/mujoco.py:32-41)."""

    def __init__(self, kind, n_in, n_act, n_params):
        assert kind in ("discrete", "mujoco")
        self.kind, self.n_in, self.n_act, self.n_params = kind, int(n_in), int(n_act), int(n_params)

    def desc(self, bn_mean=None, bn_var=None):
        return _lib.PolicyDesc(_lib.FDR_POLICY_DISCRETE if self.kind == "discrete" else _lib.FDR_POLICY_MUJOCO,
                               self.n_in, self.n_act, 64, self.n_params,
                               None if bn_mean is None else bn_mean.data_ptr(),
                               None if bn_var is None else bn_var.data_ptr())


def _check_dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("fdr: tensors must live on the GPU (got %s)" % t.device)


def lanes_desc(base, base_stride, table=None, idx=None, sign=None, sigma=0.0, deterministic=None, lane_offset=0):
    _check_dev(base, table, idx, sign, deterministic)
    if base.dtype != torch.float32 or not base.is_contiguous():
        raise ValueError("base must be contiguous float32")
    if idx is not None and idx.dtype != torch.int64:
        raise ValueError("idx must be int64")
    if sign is not None and sign.dtype != torch.int8:
        raise ValueError("sign must be int8")
    if deterministic is not None and deterministic.dtype != torch.int8:
        raise ValueError("deterministic must be int8")
    d = _lib.LanesDesc(base.data_ptr(), int(base_stride),
                       None if table is None else table.data_ptr(),
                       0 if table is None else table.numel(),
                       None if idx is None else idx.data_ptr(),
                       None if sign is None else sign.data_ptr(),
                       float(sigma),
                       None if deterministic is None else deterministic.data_ptr(),
                       int(lane_offset))
    # the descriptor holds raw device pointers: keep the tensors alive as long as it lives, or the
    # caching allocator may hand their blocks to the next allocation before the kernel runs
    d._refs = (base, table, idx, sign, deterministic)
    return d


def perturb(theta, table, idx, sign, sigma):
    """theta' = theta + sign * fl32(sigma * table[idx:idx+P]) -> [n, P] (worker/worker.py:28)."""
    _check_dev(theta, table, idx, sign)
    n, P = idx.numel(), theta.numel()
    out = torch.empty((n, P), dtype=torch.float32, device=theta.device)
    check(lib.fdr_perturb(_c(theta.device), _p(theta), P, _p(table), table.numel(), _p(idx), _p(sign), n,
                          float(sigma), _p(out), _stream(theta.device)), "fdr_perturb")
    return out


def policy_forward(spec, lanes, n_lanes, x, bn_mean=None, bn_var=None):
    """One observation per lane.  discrete -> probs [n, A]; mujoco -> (mean, std) [n, A]."""
    _check_dev(x, bn_mean, bn_var)
    x = x.to(torch.float32).contiguous()
    dev = x.device
    out0 = torch.empty((n_lanes, spec.n_act), dtype=torch.float32, device=dev)
    out1 = None if spec.kind == "discrete" else torch.empty_like(out0)
    pd = spec.desc(bn_mean, bn_var)
    check(lib.fdr_policy_forward(_c(dev), ctypes.byref(pd), ctypes.byref(lanes), n_lanes, _p(x), _p(out0),
                                 _p(out1), _stream(dev)), "fdr_policy_forward")
    return out0 if out1 is None else (out0, out1)


class RolloutResult(object):
    """SoA result of one batched rollout (the FDReturn fields, learner/fd_return.py:5-16)."""

    def __init__(self, ret, ent, steps, norm2):
        self.reward, self.entropy, self.timesteps, self.norm2 = ret, ent, steps, norm2


def rollout(spec, env, lanes, n_lanes, seed, jiggle=True, obs_mean=None, obs_std=None,
            bn_mean=None, bn_var=None, out=None, device=None, states=None, obs_stats=None, ctx=None,
            u_inject=None):
    """fdr_rollout; fdr_rollout_ex when states (f32 [n_lanes, T, n_in] device tensor) is given,
    obs_stats = the per-step sampling chance (-> out.obs_mean / obs_m2 / obs_count per lane), or u_inject =
    host-injected draws (f32 [n_lanes, T, k] device tensor: k = 1 uniform per step for a discrete policy, n_act
    normals for a continuous one) replacing the counter stream."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    _check_dev(obs_mean, obs_std, bn_mean, bn_var)
    if out is None:  # the four outputs in one allocation (one caching-allocator call per rollout)
        buf = torch.empty(28 * n_lanes, dtype=torch.uint8, device=dev)
        out = RolloutResult(buf[:8 * n_lanes].view(torch.float64), buf[8 * n_lanes:16 * n_lanes].view(torch.float64),
                            buf[24 * n_lanes:].view(torch.int32), buf[16 * n_lanes:24 * n_lanes].view(torch.float64))
    pd = spec.desc(bn_mean, bn_var)
    ed = env.desc()
    if states is not None or obs_stats is not None or u_inject is not None:
        x = _lib.RolloutExtras(None, None, None, None, 0.0, None)
        if u_inject is not None:
            _check_dev(u_inject)
            k = 1 if spec.kind == "discrete" else spec.n_act
            if u_inject.dtype != torch.float32 or not u_inject.is_contiguous() or \
                    u_inject.numel() != n_lanes * env.episode_len * k:
                raise ValueError("u_inject must be contiguous float32 [n_lanes, T, %d]" % k)
            x.u_inject = u_inject.data_ptr()
        if states is not None:
            _check_dev(states)
            if states.dtype != torch.float32 or not states.is_contiguous() or \
                    states.numel() != n_lanes * env.episode_len * spec.n_in:
                raise ValueError("states must be contiguous float32 [n_lanes, T, n_in]")
            x.states = states.data_ptr()
        if obs_stats is not None:
            chance = float(obs_stats)
            out.obs_mean = torch.empty((n_lanes, spec.n_in), dtype=torch.float32, device=dev)
            out.obs_m2 = torch.empty_like(out.obs_mean)
            out.obs_count = torch.empty(n_lanes, dtype=torch.int32, device=dev)
            x.obs_mean, x.obs_m2, x.obs_count = out.obs_mean.data_ptr(), out.obs_m2.data_ptr(), \
                out.obs_count.data_ptr()
            x.obs_chance = chance
        check(lib.fdr_rollout_ex(_c(dev, ctx), ctypes.byref(pd), ctypes.byref(ed), ctypes.byref(lanes), n_lanes,
                                 ctypes.c_uint64(seed & ((1 << 64) - 1)), 1 if jiggle else 0, _p(obs_mean),
                                 _p(obs_std), _p(out.reward), _p(out.entropy), _p(out.timesteps),
                                 _p(out.norm2), ctypes.byref(x), _stream(dev)), "fdr_rollout_ex")
        return out
    check(lib.fdr_rollout(_c(dev, ctx), ctypes.byref(pd), ctypes.byref(ed), ctypes.byref(lanes), n_lanes,
                          ctypes.c_uint64(seed & ((1 << 64) - 1)), 1 if jiggle else 0, _p(obs_mean),
                          _p(obs_std), _p(out.reward), _p(out.entropy), _p(out.timesteps), _p(out.norm2),
                          _stream(dev)), "fdr_rollout")
    return out


def fd_weights(rewards_all, policy_reward, lane_lo, sign_local, norm2_local, lanes_per_dir, sigma, coef=None):
    _check_dev(rewards_all, sign_local, norm2_local)
    n_local = sign_local.numel()
    n_dirs = n_local // lanes_per_dir
    if coef is None:
        coef = torch.empty(n_dirs, dtype=torch.float64, device=rewards_all.device)
    check(lib.fdr_fd_weights(_c(rewards_all.device), _p(rewards_all), rewards_all.numel(), float(policy_reward), int(lane_lo),
                             n_local, _p(sign_local), _p(norm2_local), int(lanes_per_dir), float(sigma),
                             _p(coef), _stream(rewards_all.device)), "fdr_fd_weights")
    return coef


_WS = {}


def _workspace(key, nbytes, device, zeroed=False):
    """Per-(purpose, device) scratch, grown on demand.  zeroed: allocated zero-filled (the in-launch
    counters of fdr_fd_grad_fused must start at zero; every call leaves them zero)."""
    buf = _WS.get((key, device))
    if buf is None or buf.numel() < nbytes:
        n = max(int(nbytes), 16)
        buf = torch.zeros(n, dtype=torch.uint8, device=device) if zeroed else \
            torch.empty(n, dtype=torch.uint8, device=device)
        _WS[(key, device)] = buf
    return buf


_WS_ZERO_PREFIX = {}


_FUSED_SIZES = {}


def _fused_workspace(mode, n_dirs, lanes_per_dir, n_params, device):
    """The fdr_fd_grad_fused / fdr_fd_step workspace with its ticket-counter prefix guaranteed zero.

    A call leaves exactly its own counter prefix, fdr_fd_grad_fused_counter_bytes(n_dirs, P), at zero; the bytes
    behind it hold that call's slabs / partials.  A later call whose prefix is longer (more column blocks) would
    find non-zero counters there, so the prefix is re-zeroed (on the current stream, ahead of the launch)
    whenever it grows past what is known to be zero."""
    key = ("fused_%d" % mode, device)
    old = _WS.get(key)
    skey = (mode, n_dirs, int(lanes_per_dir), n_params)
    sizes = _FUSED_SIZES.get(skey)
    if sizes is None:  # the library's size queries, once per shape
        sizes = _FUSED_SIZES[skey] = (lib.fdr_fd_grad_fused_workspace_bytes(n_dirs, int(lanes_per_dir), n_params, mode),
                                      int(lib.fdr_fd_grad_fused_counter_bytes(n_dirs, n_params)))
    nb, cb = sizes
    ws = _workspace(key[0], nb, device, zeroed=True)
    if ws is not old:
        _WS_ZERO_PREFIX[key] = ws.numel()
    if cb > _WS_ZERO_PREFIX.get(key, 0):
        ws[:cb].zero_()
    _WS_ZERO_PREFIX[key] = cb
    return ws


WEIGHT_MODES = {"zscore": _lib.FDR_WEIGHT_ZSCORE, "centred_rank": _lib.FDR_WEIGHT_CENTERED_RANK,
                "moments": _lib.FDR_WEIGHT_MOMENTS}


def fd_grad_fused(table, idx_local, rewards_all, policy_reward, lane_lo, sign_local, norm2_local, lanes_per_dir, sigma,
                  n_params, mode="zscore", out=None, n_all=None):
    """Weights + noise-weighted gradient in one launch (fdr_fd_grad_fused).  idx_local / sign_local / norm2_local:
    one entry per local lane.  mode "zscore" / "centred_rank" -> g f64 [P]; "moments" (rewards_all = the local
    rewards, n_all = the lanes of all ranks, lane_lo = this rank's first global lane) ->
    [A | B | n_local | r' slots [n_all]] f64 [2P + 1 + n_all]."""
    _check_dev(table, idx_local, rewards_all, sign_local, norm2_local)
    dev = table.device
    n_dirs = idx_local.numel() // int(lanes_per_dir)
    m = WEIGHT_MODES[mode]
    if n_all is None:
        n_all = rewards_all.numel() + (int(lane_lo) if mode == "moments" else 0)
    n_out = int(lib.fdr_fd_grad_fused_out_len(m, n_params, int(n_all)))
    if n_out <= 0:
        raise ValueError("fd_grad_fused: bad mode / P / n_all")
    if out is None:
        out = torch.empty(n_out, dtype=torch.float64, device=dev)
    elif out.numel() < n_out:
        raise ValueError("fd_grad_fused: out holds %d doubles, needs %d" % (out.numel(), n_out))
    ws = _fused_workspace(m, n_dirs, lanes_per_dir, n_params, dev)
    check(lib.fdr_fd_grad_fused(_c(dev), _p(table), table.numel(), _p(idx_local), n_dirs, n_params, _p(rewards_all),
                                int(n_all), float(policy_reward), int(lane_lo), _p(sign_local), _p(norm2_local),
                                int(lanes_per_dir), float(sigma), m, _p(out), out.numel(), _p(ws), ws.numel(),
                                _stream(dev)),
          "fdr_fd_grad_fused")
    return out


def fd_step(table, idx_local, rewards, policy_reward, sign_local, norm2_local, lanes_per_dir, sigma, theta, lr,
            lr_scale, mode="zscore", g=None, out=None, theta_hist=None):
    """The single-process FD step (fdr_fd_step): weights + gradient (-> g) in one launch, DSGD on theta in place in
    a second; theta_hist (f32 [P], optional) receives the updated theta.  Returns device f64[2] =
    (||d theta||, ||grad||)."""
    _check_dev(table, idx_local, rewards, sign_local, norm2_local, theta, g, theta_hist)
    dev = table.device
    P = theta.numel()
    n_dirs = idx_local.numel() // int(lanes_per_dir)
    m = WEIGHT_MODES[mode]
    if g is None:
        g = torch.empty(P, dtype=torch.float64, device=dev)
    if out is None:
        out = torch.empty(2, dtype=torch.float64, device=dev)
    ws = _fused_workspace(m, n_dirs, lanes_per_dir, P, dev)
    check(lib.fdr_fd_step(_c(dev), _p(table), table.numel(), _p(idx_local), n_dirs, P, _p(rewards), rewards.numel(),
                          float(policy_reward), _p(sign_local), _p(norm2_local), int(lanes_per_dir), float(sigma), m,
                          _p(theta), float(lr), float(lr_scale), _p(g), _p(theta_hist), _p(out), _p(ws), ws.numel(),
                          _stream(dev)), "fdr_fd_step")
    return out


def rank_weights(rewards_all, lane_lo, n_local):
    """Centred-rank weights of lanes [lane_lo, lane_lo + n_local) over rewards_all (f64 [n_local])."""
    _check_dev(rewards_all)
    w = torch.empty(n_local, dtype=torch.float64, device=rewards_all.device)
    check(lib.fdr_rank_weights(_c(rewards_all.device), _p(rewards_all), rewards_all.numel(), int(lane_lo), int(n_local), _p(w),
                               _stream(rewards_all.device)), "fdr_rank_weights")
    return w


def dsgd_step_ex(theta, src, moments, lr, lr_scale, g_out=None, out=None):
    """DSGD from g (moments=False) or from summed moments (g = (A - m B) / sd written to g_out)."""
    _check_dev(theta, src, g_out)
    dev = theta.device
    if out is None:
        out = torch.empty(2, dtype=torch.float64, device=dev)
    nb = lib.fdr_dsgd_workspace_bytes(theta.numel())
    ws = _workspace("dsgd", nb, dev)
    check(lib.fdr_dsgd_step_ex(_c(dev), _p(theta), _p(src), 1 if moments else 0, theta.numel(), float(lr), float(lr_scale),
                               _p(g_out), _p(out), _p(ws), ws.numel(), _stream(dev)), "fdr_dsgd_step_ex")
    return out


def fd_grad(table, idx_dirs, coef, n_params, g=None):
    _check_dev(table, idx_dirs, coef)
    dev = table.device
    n_dirs = idx_dirs.numel()
    if g is None:
        g = torch.empty(n_params, dtype=torch.float64, device=dev)
    nb = lib.fdr_fd_grad_workspace_bytes(n_dirs, n_params)
    ws = _workspace("grad", nb, dev)
    check(lib.fdr_fd_grad(_c(dev), _p(table), table.numel(), _p(idx_dirs), _p(coef), n_dirs, n_params, _p(g),
                          _p(ws), ws.numel(), _stream(dev)), "fdr_fd_grad")
    return g


def dsgd_step(theta, g, lr, lr_scale, out=None):
    """In-place theta update; returns device f64[2] = (||d theta||, ||grad||)."""
    _check_dev(theta, g)
    dev = theta.device
    if out is None:
        out = torch.empty(2, dtype=torch.float64, device=dev)
    nb = lib.fdr_dsgd_workspace_bytes(theta.numel())
    ws = _workspace("dsgd", nb, dev)
    check(lib.fdr_dsgd_step(_c(dev), _p(theta), _p(g), theta.numel(), float(lr), float(lr_scale), _p(out), _p(ws),
                            ws.numel(), _stream(dev)), "fdr_dsgd_step")
    return out


# ---- ImpalaPolicy (policies/impala.py) --------------------------------------------------------
def impala_num_params(n_act):
    return int(lib.fdr_impala_num_params(int(n_act)))


def impala_num_bn_stats():
    return int(lib.fdr_impala_num_bn_stats())


class ImpalaSpec(object):
    """Shape of an ImpalaPolicy rollout: A actions, E envs per perturbation, T-step episodes."""

    def __init__(self, n_act, envs_per_lane=1, episode_len=1, entropy=True, env_seed=0, fp16=False, pairs=False):
        """pairs: lanes 2p, 2p+1 are antithetic pairs -- the rollout's core step streams each pair's sigma-eps once
        (fdr_impala_desc.pairs; f32: bit-identical to the per-lane form, fp16: within the fp16 tolerance)."""
        self.n_act, self.envs_per_lane, self.episode_len = int(n_act), int(envs_per_lane), int(episode_len)
        self.entropy, self.env_seed, self.fp16 = bool(entropy), int(env_seed), bool(fp16)
        self.pairs = bool(pairs)
        self.n_params = impala_num_params(n_act)
        if self.n_params < 0:
            raise ValueError("n_act out of range")

    def desc(self, bn_mean=None, bn_var=None):
        _check_dev(bn_mean, bn_var)
        for t in (bn_mean, bn_var):
            if t is not None and (t.dtype != torch.float32 or t.numel() != impala_num_bn_stats()):
                raise ValueError("BN stats must be float32[%d]" % impala_num_bn_stats())
        return _lib.ImpalaDesc(self.n_act, self.envs_per_lane, self.episode_len, 1 if self.entropy else 0,
                               self.env_seed & ((1 << 64) - 1), self.n_params,
                               None if bn_mean is None else bn_mean.data_ptr(),
                               None if bn_var is None else bn_var.data_ptr(), 1 if self.fp16 else 0,
                               1 if self.pairs else 0)


def impala_rollout(spec, lanes, n_lanes, seed, jiggle=True, bn_mean=None, bn_var=None, record=False, out=None,
                   device=None, ctx=None):
    """fdr_impala_rollout: returns RolloutResult with per-env [n_lanes*E] fields, norm2 per lane,
    plus .actions [n_lanes*E, T] / .probs [n_lanes*E, T, A] when record=True."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    n_env = n_lanes * spec.envs_per_lane
    if out is None:
        out = RolloutResult(torch.empty(n_env, dtype=torch.float64, device=dev),
                            torch.empty(n_env, dtype=torch.float64, device=dev),
                            torch.empty(n_env, dtype=torch.int32, device=dev),
                            torch.empty(n_lanes, dtype=torch.float64, device=dev))
    out.actions = torch.empty((n_env, spec.episode_len), dtype=torch.int32, device=dev) if record else None
    out.probs = torch.empty((n_env, spec.episode_len, spec.n_act), dtype=torch.float32, device=dev) if record \
        else None
    d = spec.desc(bn_mean, bn_var)
    nb = lib.fdr_impala_workspace_bytes(ctypes.byref(d), n_lanes)
    if nb < 0:
        raise ValueError("bad impala spec")
    ws = _workspace("impala", nb, dev)
    check(lib.fdr_impala_rollout(_c(dev, ctx), ctypes.byref(d), ctypes.byref(lanes), n_lanes,
                                 ctypes.c_uint64(seed & ((1 << 64) - 1)), 1 if jiggle else 0, _p(out.reward),
                                 _p(out.entropy), _p(out.timesteps), _p(out.norm2), _p(out.actions), _p(out.probs),
                                 _p(ws), ws.numel(), _stream(dev)), "fdr_impala_rollout")
    return out


def impala_forward(spec, theta, frames, h, c, reward=None, notdone=None, bn_mean=None, bn_var=None, feat=False):
    """One ImpalaCNN step for n envs sharing theta; h, c [n, 256] are updated in place.
    Returns probs [n, A] (and the relu'd conv features [n, 2048] if feat)."""
    _check_dev(theta, frames, h, c, reward, notdone)
    dev = theta.device
    frames = frames.to(torch.float32).reshape(-1, 3 * 64 * 64).contiguous()
    n = frames.shape[0]
    for t in (h, c):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != n * 256:
            raise ValueError("h / c must be contiguous float32 [n, 256]")
    if reward is not None:
        reward = reward.to(torch.float32).reshape(-1).contiguous()
    if notdone is not None:
        notdone = notdone.to(torch.float32).reshape(-1).contiguous()
    probs = torch.empty((n, spec.n_act), dtype=torch.float32, device=dev)
    f = torch.empty((n, 2048), dtype=torch.float32, device=dev) if feat else None
    d = spec.desc(bn_mean, bn_var)
    nb = lib.fdr_impala_forward_workspace_bytes(spec.n_act, n, 1 if spec.fp16 else 0)
    ws = _workspace("impala_fwd", nb, dev)
    check(lib.fdr_impala_forward(_c(dev), ctypes.byref(d), _p(theta), n, _p(frames), _p(reward), _p(notdone), _p(h),
                                 _p(c), _p(probs), _p(f), _p(ws), ws.numel(), _stream(dev)), "fdr_impala_forward")
    return (probs, f) if feat else probs


def impala_strategies(spec, lanes, n_lanes, frames, reward=None, h=None, c=None, bn_mean=None, bn_var=None):
    """get_strategy of n_lanes ImpalaPolicy parameter vectors over the Z shared probe obs: the stacked obs
    run as ONE LSTM sequence per lane (policies/impala.py:24-27) from (h, c) [n_lanes, 256] (updated in
    place) or from the reset state (None).  frames [Z, 3, 64, 64] (0..255), reward [Z] -> probs
    [n_lanes, Z, A] f32."""
    dev = frames.device
    _check_dev(frames, reward, h, c)
    frames = frames.to(torch.float32).reshape(-1, 3 * 64 * 64).contiguous()
    Z = frames.shape[0]
    if reward is not None:
        reward = reward.to(torch.float32).reshape(-1).contiguous()
        if reward.numel() != Z:
            raise ValueError("reward must have one entry per probe frame")
    if (h is None) != (c is None):
        raise ValueError("give both h and c, or neither")
    for t in (h, c):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != n_lanes * 256):
            raise ValueError("h / c must be contiguous float32 [n_lanes, 256]")
    probs = torch.empty((n_lanes, Z, spec.n_act), dtype=torch.float32, device=dev)
    d = spec.desc(bn_mean, bn_var)
    nb = lib.fdr_impala_strategies_workspace_bytes(ctypes.byref(d), n_lanes, Z)
    if nb < 0:
        raise ValueError("bad impala spec")
    ws = _workspace("impala_strat", nb, dev)
    check(lib.fdr_impala_strategies(_c(dev), ctypes.byref(d), ctypes.byref(lanes), n_lanes, Z, _p(frames), _p(reward),
                                    _p(h), _p(c), _p(probs), _p(ws), ws.numel(), _stream(dev)),
          "fdr_impala_strategies")
    return probs


def impala_bn_refresh(spec, theta, frames, bn_mean, bn_var, reward=None, first_done=False, h=None, c=None,
                      momentum=0.1):
    """ImpalaPolicy.compute_vbn on the device (policies/impala.py:12-16): a train-mode pass of the n-obs buffer
    frames [n, 3, 64, 64] (0..255) / reward [n] updates bn_mean / bn_var (modules() order) in place; the LSTM runs
    the n obs as one sequence from (h, c) [256] (zeroed first if first_done; None: zero state) and leaves its end
    state in h / c."""
    _check_dev(theta, frames, bn_mean, bn_var, reward, h, c)
    dev = theta.device
    frames = frames.to(torch.float32).reshape(-1, 3 * 64 * 64).contiguous()
    n = frames.shape[0]
    if reward is not None:
        reward = reward.to(torch.float32).reshape(-1).contiguous()
        if reward.numel() != n:
            raise ValueError("reward must have one entry per buffer frame")
    if (h is None) != (c is None):
        raise ValueError("give both h and c, or neither")
    for t in (h, c, bn_mean, bn_var):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
            raise ValueError("h / c / bn_mean / bn_var must be contiguous float32")
    if h is not None and (h.numel() != 256 or c.numel() != 256):
        raise ValueError("h / c must hold 256 floats")
    if n < 2:
        raise ValueError("Expected more than 1 value per channel when training (compute_vbn needs >= 2 obs)")
    d = spec.desc(None, None)
    ws = _workspace("impala_vbn", lib.fdr_impala_bn_refresh_workspace_bytes(n), dev)
    check(lib.fdr_impala_bn_refresh(_c(dev), ctypes.byref(d), _p(theta), n, _p(frames), _p(reward),
                                    1 if first_done else 0, _p(h), _p(c), float(momentum), _p(bn_mean), _p(bn_var),
                                    _p(ws), ws.numel(), _stream(dev)), "fdr_impala_bn_refresh")


def impala_env_frames(env_seed, n_act, env_id, t0, n, actions=None, device=None):
    """The frame env's observations frame_t (t0 <= t < t0 + n) of global env env_id -> (frames [n, 3, 64, 64]
    f32, rewards [n] f32 returned by the steps given actions [n] (device i32; None -> 0))."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if actions is not None:
        _check_dev(actions)
        actions = actions.to(torch.int32).reshape(-1).contiguous()
        if actions.numel() != n:
            raise ValueError("actions must have n entries")
    frames = torch.empty((n, 3, 64, 64), dtype=torch.float32, device=dev)
    reward = torch.empty(n, dtype=torch.float32, device=dev)
    check(lib.fdr_impala_env_frames(ctypes.c_uint64(int(env_seed) & ((1 << 64) - 1)), int(n_act), int(env_id), int(t0),
                                    int(n), _p(actions), _p(frames), _p(reward), _stream(dev)), "fdr_impala_env_frames")
    return frames, reward


def impala_profile(enable, device=None):
    """Phase timing of the device's Impala rollouts (its engine context)."""
    context(device).impala_profile(enable)


def impala_profile_read(device=None):
    """(conv_ms, core_ms, replay_ms) summed over the last profiled fdr_impala_rollout (host sync)."""
    return context(device).impala_profile_read()


# ---- strategy distances / novelty (utils/math_helpers.py:147-222) ---------------------------------
DIST_KINDS = {"l2": _lib.FDR_DIST_L2, "tvd": _lib.FDR_DIST_TVD, "w2": _lib.FDR_DIST_W2}


def strategy_distances(strategies, archive, kind, full=False):
    """strategies [n, Z, D], archive [H, Z, D] (f32 device) -> (min [n] f64, argmin [n] i32[, dists [n, H]])."""
    _check_dev(strategies, archive)
    S = strategies.to(torch.float32).contiguous()
    B = archive.to(torch.float32).contiguous()
    n, Z, D = S.shape
    H = B.shape[0]
    if tuple(B.shape[1:]) != (Z, D):
        raise ValueError("archive shape %s does not match strategies %s" % (tuple(B.shape), tuple(S.shape)))
    dev = S.device
    mn = torch.empty(n, dtype=torch.float64, device=dev)
    am = torch.empty(n, dtype=torch.int32, device=dev)
    dd = torch.empty((n, H), dtype=torch.float64, device=dev) if full else None
    check(lib.fdr_strategy_distances(_c(dev), _p(S), n, _p(B), H, Z, D, DIST_KINDS[kind], _p(dd), _p(mn), _p(am),
                                     _stream(dev)), "fdr_strategy_distances")
    return (mn, am, dd) if full else (mn, am)


def lane_strategies(spec, lanes_fn, n_lanes, zeta, bn_mean=None, bn_var=None):
    """get_strategy (discrete: probs; mujoco: [mean | std]) of n_lanes policies over the Z probe
    states zeta -> f32 [n_lanes, Z, D].  lanes_fn(Z) must return a lanes descriptor of n_lanes * Z
    (policy, state) pairs, policy-major (every lane field repeated Z times)."""
    _check_dev(zeta)
    Z = zeta.shape[0]
    x = zeta.to(torch.float32).reshape(Z, -1).repeat(n_lanes, 1).contiguous()
    out = policy_forward(spec, lanes_fn(Z), n_lanes * Z, x, bn_mean, bn_var)
    if isinstance(out, tuple):
        out = torch.cat(out, dim=-1)
    return out.reshape(n_lanes, Z, -1)


def obs_stats_merge(mean, m2, count, acc_mean, acc_m2, acc_count):
    """Fold per-lane Welford partials into the device accumulator (in place, lane order)."""
    _check_dev(mean, m2, count, acc_mean, acc_m2, acc_count)
    n, d = mean.shape
    check(lib.fdr_obs_stats_merge(_c(mean.device), _p(mean), _p(m2), _p(count), n, d, _p(acc_mean), _p(acc_m2), _p(acc_count),
                                  _stream(mean.device)), "fdr_obs_stats_merge")


# ---- delayed returns: lambda with policy drift (learner/finite_differences.py:66-114) -------------
def fd_lambda_norms(table, idx, sign, slot, sigma, drift, n_params):
    """||fl32(sign * fl32(sigma * eps_i) + D[slot_i])||^2 per return (f64 [n])."""
    _check_dev(table, idx, sign, slot, drift)
    n = idx.numel()
    n2 = torch.empty(n, dtype=torch.float64, device=table.device)
    ns = 0 if drift is None else drift.shape[0]
    check(lib.fdr_fd_lambda_norms(_c(table.device), _p(table), table.numel(), _p(idx), _p(sign), _p(slot), n, n_params,
                                  float(sigma), _p(drift), ns, _p(n2), _stream(table.device)), "fdr_fd_lambda_norms")
    return n2


def fd_grad_lambda(table, idx, sign, slot, coef, sigma, drift, n_params, g=None):
    """g = sum_i coef_i * lambda_i (f64 [P])."""
    _check_dev(table, idx, sign, slot, coef, drift)
    dev = table.device
    n = idx.numel()
    if g is None:
        g = torch.empty(n_params, dtype=torch.float64, device=dev)
    ns = 0 if drift is None else drift.shape[0]
    nb = lib.fdr_fd_grad_workspace_bytes(n, n_params)
    ws = _workspace("grad", nb, dev)
    check(lib.fdr_fd_grad_lambda(_c(dev), _p(table), table.numel(), _p(idx), _p(sign), _p(slot), _p(coef), n, n_params,
                                 float(sigma), _p(drift), ns, _p(g), _p(ws), ws.numel(), _stream(dev)),
          "fdr_fd_grad_lambda")
    return g


def bn_refresh(spec, theta, x, bn_mean, bn_var, momentum=0.1):
    """compute_vbn on the device: updates bn_mean / bn_var (f32, [n_in | 64 | 64]) in place."""
    _check_dev(theta, x, bn_mean, bn_var)
    x = x.to(torch.float32).reshape(-1, spec.n_in).contiguous()
    n = x.shape[0]
    pd = spec.desc(None, None)
    ws = _workspace("vbn", lib.fdr_bn_refresh_workspace_bytes(n), x.device)
    check(lib.fdr_bn_refresh(_c(x.device), ctypes.byref(pd), _p(theta), _p(x), n, float(momentum), _p(bn_mean), _p(bn_var),
                             _p(ws), ws.numel(), _stream(x.device)), "fdr_bn_refresh")


# ---- AtariPolicy (policies/atari.py) -------------------------------------------------------------------
def atari_num_params(n_act):
    return int(lib.fdr_atari_num_params(int(n_act)))


class AtariSpec(object):
    def __init__(self, n_act, envs_per_lane=1, episode_len=1, env_seed=0):
        self.n_act, self.envs_per_lane, self.episode_len = int(n_act), int(envs_per_lane), int(episode_len)
        self.env_seed = int(env_seed)
        self.n_params = atari_num_params(n_act)
        if self.n_params < 0:
            raise ValueError("n_act out of range")

    def desc(self, bn_mean=None, bn_var=None):
        _check_dev(bn_mean, bn_var)
        for t in (bn_mean, bn_var):
            if t is not None and (t.dtype != torch.float32 or t.numel() != 16 + 32 + 256):
                raise ValueError("BN stats must be float32[304]")
        return _lib.AtariDesc(self.n_act, self.envs_per_lane, self.episode_len, 0, self.env_seed & ((1 << 64) - 1),
                              self.n_params, None if bn_mean is None else bn_mean.data_ptr(),
                              None if bn_var is None else bn_var.data_ptr())


def atari_rollout(spec, lanes, n_lanes, seed, jiggle=True, bn_mean=None, bn_var=None, record=False, device=None):
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    n_env = n_lanes * spec.envs_per_lane
    out = RolloutResult(torch.empty(n_env, dtype=torch.float64, device=dev),
                        torch.empty(n_env, dtype=torch.float64, device=dev),
                        torch.empty(n_env, dtype=torch.int32, device=dev),
                        torch.empty(n_lanes, dtype=torch.float64, device=dev))
    out.actions = torch.empty((n_env, spec.episode_len), dtype=torch.int32, device=dev) if record else None
    out.probs = torch.empty((n_env, spec.episode_len, spec.n_act), dtype=torch.float32, device=dev) if record \
        else None
    d = spec.desc(bn_mean, bn_var)
    nb = lib.fdr_atari_workspace_bytes(ctypes.byref(d), n_lanes)
    ws = _workspace("atari", nb, dev)
    check(lib.fdr_atari_rollout(_c(dev), ctypes.byref(d), ctypes.byref(lanes), n_lanes,
                                ctypes.c_uint64(seed & ((1 << 64) - 1)), 1 if jiggle else 0, _p(out.reward),
                                _p(out.entropy), _p(out.timesteps), _p(out.norm2), _p(out.actions), _p(out.probs),
                                _p(ws), ws.numel(), _stream(dev)), "fdr_atari_rollout")
    return out


def atari_env_frames(env_seed, env_id, t0, n, device=None):
    """The stacked-frame env's observations [n, 4, 84, 84] f32 of global env env_id at steps t0 .. t0 + n - 1
    (fdr_atari_env_frames; independent of the actions)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    out = torch.empty((int(n), 4, 84, 84), dtype=torch.float32, device=dev)
    check(lib.fdr_atari_env_frames(ctypes.c_uint64(int(env_seed) & ((1 << 64) - 1)), int(env_id), int(t0), int(n),
                                   _p(out), _stream(dev)), "fdr_atari_env_frames")
    return out


def atari_forward(spec, theta, frames, bn_mean=None, bn_var=None, feat=False):
    _check_dev(theta, frames)
    frames = frames.to(torch.float32).reshape(-1, 4 * 84 * 84).contiguous()
    n = frames.shape[0]
    dev = theta.device
    probs = torch.empty((n, spec.n_act), dtype=torch.float32, device=dev)
    f = torch.empty((n, 2592), dtype=torch.float32, device=dev) if feat else None
    d = spec.desc(bn_mean, bn_var)
    ws = _workspace("atari_fwd", lib.fdr_atari_forward_workspace_bytes(spec.n_act, n), dev)
    check(lib.fdr_atari_forward(_c(dev), ctypes.byref(d), _p(theta), n, _p(frames), _p(probs), _p(f), _p(ws), ws.numel(),
                                _stream(dev)), "fdr_atari_forward")
    return (probs, f) if feat else probs


def atari_bn_refresh(spec, theta, frames, bn_mean, bn_var, momentum=0.1):
    """AtariPolicy.compute_vbn on the device (policies/policy.py:31-34): a train-mode pass of the n frames
    [n, 4, 84, 84] (0..255) updating the running stats bn_mean / bn_var [16 | 32 | 256] in place (fdr_atari_bn_refresh).
    n >= 2 (torch's train-mode BatchNorm1d raises for one value per channel)."""
    _check_dev(frames)
    dev = frames.device
    frames = frames.to(torch.float32).reshape(-1, 4 * 84 * 84).contiguous()
    n = frames.shape[0]
    if n < 2:
        raise ValueError("Expected more than 1 value per channel when training (compute_vbn needs >= 2 obs)")
    d = spec.desc(None, None)
    ws = _workspace("atari_vbn", lib.fdr_atari_bn_refresh_workspace_bytes(n), dev)
    check(lib.fdr_atari_bn_refresh(_c(dev), ctypes.byref(d), _p(theta), n, _p(frames), float(momentum), _p(bn_mean),
                                   _p(bn_var), _p(ws), ws.numel(), _stream(dev)), "fdr_atari_bn_refresh")


def atari_strategies(spec, lanes, n_lanes, frames, bn_mean=None, bn_var=None):
    """AtariPolicy.get_strategy of n_lanes parameter vectors (lanes descriptor) over the Z shared probe frames
    [Z, 4, 84, 84] (0..255) -> probs [n_lanes, Z, A] f32, batched (fdr_atari_strategies)."""
    _check_dev(frames)
    dev = frames.device
    frames = frames.to(torch.float32).reshape(-1, 4 * 84 * 84).contiguous()
    Z = frames.shape[0]
    probs = torch.empty((n_lanes, Z, spec.n_act), dtype=torch.float32, device=dev)
    d = spec.desc(bn_mean, bn_var)
    nb = lib.fdr_atari_strategies_workspace_bytes(ctypes.byref(d), n_lanes, Z)
    if nb < 0:
        raise ValueError("bad atari spec")
    ws = _workspace("atari_strat", nb, dev)
    check(lib.fdr_atari_strategies(_c(dev), ctypes.byref(d), ctypes.byref(lanes), n_lanes, Z, _p(frames), _p(probs),
                                   _p(ws), ws.numel(), _stream(dev)), "fdr_atari_strategies")
    return probs
