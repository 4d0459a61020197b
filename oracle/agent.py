"""Episode loop restatement (one lane) and the batched-lane evaluation the GPU path computes.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

``collect_return`` follows worker/agent.py:20-71 step by step:
  * obs normalisation clip((o - mean) / std, -10, 10) with FIXED learner stats (:37-41); the
    per-step Welford sampling (:38-39) belongs to the obs-stats row and is not
    restated here;
  * action = get_action(obs, deterministic) (:43), env.step (:44), reward += rew, steps += 1;
  * on done: obs = env.reset(); break (:50-52); ts_limit 10000 (:12);
  * entropy = policy.get_entropy(states) over every visited (normalised) state (:60-65);
  * reward += jiggle (:69) -- either the reference's Agent.rng.choice((-1e-12, 1e-12)) or the
    build's counter stream (oracle/rng.py) for GPU parity.

``evaluate_lanes`` is the batched semantics of the HIP rollout kernel (DESIGN.md "Rollout"):
lane l runs theta'_l = perturb(theta, idx_l, sign_l) for one full episode from reset; stochastic
actions come from the counter stream keyed by (seed, lane, t, k); entropy is the mean of the
per-step policy entropies (same probabilities as the reference's end-of-episode batched forward).
"""
import numpy as np

from . import obs_stats
from . import policies as pol
from . import rng as crng
from .noise import perturb

TS_LIMIT = 10000


def collect_return(policy, env, obs, deterministic, noise_fn, jiggle_fn, mean=None, std=None):
    """Returns (reward f64, entropy, steps, last_obs).  noise_fn(t) -> injected noise for step t."""
    reward, steps, states = 0.0, 0, []
    for t in range(TS_LIMIT):
        if mean is not None:
            obs = np.clip(np.subtract(obs, mean) / std, -10, 10)
        states.append(obs)
        action = policy.act(obs, deterministic, None if deterministic else noise_fn(t))
        obs, rew, done, _ = env.step(action)
        reward += rew
        steps += 1
        if done:
            obs = env.reset()
            break
    entropy = policy.entropy(np.asarray(states))
    reward += jiggle_fn()
    return reward, entropy, steps, obs


def evaluate_lanes(kind, n_in, n_act, theta, table, idx, sign, sigma, env, seed,
                   deterministic=False, bn_stats=None, obs_mean=None, obs_std=None, jiggle=True,
                   obs_chance=None, record_states=False, lane_ids=None):
    """Batched numpy reference of fdr_rollout (synthetic env).  Returns ret, ent, steps, norm2
    (+ the per-lane Welford statistics if obs_chance, + states [L, T, n_in] if record_states).
    lane_ids: the global lane ids keying the counter stream (default 0 .. L-1), for sampled lanes of a
    larger launch."""
    L = len(idx)
    thetas = perturb(theta, table, idx, sign, sigma)
    # squared norm of lambda = sign * fl32(sigma * eps) -- what the FD learner divides by
    P = thetas.shape[1]
    s32 = np.float32(sigma)
    norm2 = np.array([float(np.dot((table[int(i):int(i) + P] * s32).astype(np.float64),
                                   (table[int(i):int(i) + P] * s32).astype(np.float64)))
                      if sg != 0 else 0.0 for i, sg in zip(idx, sign)])
    obs = env.reset()
    lanes = np.arange(L, dtype=np.uint64) if lane_ids is None else np.asarray(lane_ids, dtype=np.uint64)
    ret = np.zeros(L, dtype=np.float64)
    ent = np.zeros(L, dtype=np.float64)
    det = np.broadcast_to(np.asarray(deterministic, dtype=bool), (L,))
    T = env.episode_len
    stats = [obs_stats.Welford(n_in) for _ in range(L)] if obs_chance is not None else None
    states = np.zeros((L, T, n_in), np.float32) if record_states else None
    alive = np.ones(L, bool)
    steps = np.zeros(L, np.int64)
    for t in range(T):
        if record_states:
            states[alive, t] = obs[alive]
        if stats is not None:   # worker/agent.py:37-39 (raw obs, before normalisation)
            coin = obs_stats.lane_coins(seed, lanes, t, obs_chance) & alive
            for l in np.nonzero(coin)[0]:
                stats[l].update(obs[l])
        x = obs
        if obs_mean is not None:
            x = np.clip((x - obs_mean) / obs_std, -10, 10).astype(np.float32)
        if kind == "discrete":
            p = pol.lanes_forward(kind, n_in, n_act, thetas, x, bn_stats)
            u = crng.uniform(seed, lanes, t, 0)
            act = np.array([int(np.argmax(p[l])) if det[l] else pol.categorical_inverse_cdf(p[l], u[l])
                            for l in range(L)])
            step_ent = pol.categorical_entropy(p)
        else:
            mean, std = pol.lanes_forward(kind, n_in, n_act, thetas, x)
            z = crng.normal(seed, lanes[:, None], t, np.arange(n_act, dtype=np.uint64)[None, :])
            act = np.where(det[:, None], mean, (mean + std * z).astype(np.float32)).astype(np.float32)
            step_ent = pol.normal_entropy(std)
        obs, r = env.step(act)
        # a terminating env (worker/agent.py:50-52): a lane's episode ends after its failing step -- that step's
        # reward and entropy count, later steps of the batch do not
        ret += np.where(alive, r, 0.0)
        ent += np.where(alive, step_ent, 0.0)
        steps += alive
        alive &= ~env.failed()
        if not alive.any():
            break
    ent /= steps
    if jiggle:
        ret += crng.jiggle(seed, lanes)
    out = (ret, ent, steps.astype(np.int32), norm2)
    if stats is not None:
        out = out + (stats,)
    if record_states:
        out = out + (states,)
    return out


def reference_collect_loop(kind, n_in, n_act, T, seconds, wid, sigma=0.02):
    """Worker.collect_returns + Agent.collect_return in the reference's own per-step form, for the on-box CPU
    baseline (bench.py cpu_baseline): per episode perturb theta (worker/worker.py:26-32), then per step a
    batch-1 torch forward and torch distribution sampling (policies/discrete.py:16-24, mujoco.py:15-22),
    env.step, and the end-of-episode batched entropy forward (worker/agent.py:60-66).  Runs whole episodes
    until `seconds` have passed; returns (env steps, episodes, elapsed s)."""
    import time
    import torch
    from torch.distributions import Categorical, Normal
    from .envs import SyntheticEnv
    from .noise import NoiseTable
    from .policies import TorchPolicy
    torch.manual_seed(124 + wid)
    pol = TorchPolicy(kind, n_in, n_act, seed=124)
    theta = pol.get_flat()
    tab = NoiseTable(1 << 22, theta.size, 124 + wid)
    env = SyntheticEnv(n_in, n_act, kind == "discrete", T)
    rng = np.random.RandomState(wid)
    steps = episodes = 0
    t0 = time.perf_counter()
    with torch.no_grad():
        while time.perf_counter() - t0 < seconds:
            idx = int(tab.sample_indices(1)[0])
            pol.set_flat(theta + np.float32(sigma) * tab.decode(idx))
            obs, states, reward = env.reset(), [], 0.0
            for _ in range(T):
                states.append(obs)
                out = pol.forward(obs)
                if kind == "discrete":
                    a = int(Categorical(probs=out).sample().item())
                else:
                    a = Normal(out[0], out[1]).sample().numpy().reshape(-1)
                obs, r, done, _ = env.step(a)
                reward += r
                steps += 1
                if done:
                    break
            out = pol.forward(np.asarray(states))
            ent = (Categorical(probs=out).entropy().mean() if kind == "discrete"
                   else Normal(out[0], out[1]).entropy().sum(-1).mean()).item()
            reward += rng.choice((-1e-12, 1e-12))
            pol.set_flat(theta)
            episodes += 1
    return steps, episodes, time.perf_counter() - t0


def reference_learner_step_seconds(P, n_returns, sigma=0.02, lr=0.01, repeats=2):
    """FiniteDifferences.step (learner/finite_differences.py:24-64) restated on n_returns returns: decode +
    lambda / ||lambda||^2 + z-score + the B x P dot + DSGD, on one core; median wall seconds."""
    import time
    from .learner import dsgd_step, fd_gradient
    rs = np.random.RandomState(0)
    table = rs.randn(1 << 23).astype(np.float32)
    theta = (rs.randn(P) * 0.1).astype(np.float32)
    idx = rs.randint(0, table.size - P, size=n_returns)
    sign = np.ones(n_returns, np.int8)
    rew = rs.randn(n_returns)
    times = []
    for _ in range(repeats):
        t0 = time.perf_counter()
        g, _ = fd_gradient(table, P, idx, sign, rew, 0.0, sigma)
        dsgd_step(theta, g, lr)
        times.append(time.perf_counter() - t0)
    return float(np.median(times))
