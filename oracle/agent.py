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
                   obs_chance=None, record_states=False):
    """Batched numpy reference of fdr_rollout (synthetic env).  Returns ret, ent, steps, norm2
    (+ the per-lane Welford statistics if obs_chance, + states [L, T, n_in] if record_states)."""
    L = len(idx)
    thetas = perturb(theta, table, idx, sign, sigma)
    # squared norm of lambda = sign * fl32(sigma * eps) -- what the FD learner divides by
    P = thetas.shape[1]
    s32 = np.float32(sigma)
    norm2 = np.array([float(np.dot((table[int(i):int(i) + P] * s32).astype(np.float64),
                                   (table[int(i):int(i) + P] * s32).astype(np.float64)))
                      if sg != 0 else 0.0 for i, sg in zip(idx, sign)])
    obs = env.reset()
    lanes = np.arange(L, dtype=np.uint64)
    ret = np.zeros(L, dtype=np.float64)
    ent = np.zeros(L, dtype=np.float64)
    det = np.broadcast_to(np.asarray(deterministic, dtype=bool), (L,))
    T = env.episode_len
    stats = [obs_stats.Welford(n_in) for _ in range(L)] if obs_chance is not None else None
    states = np.zeros((L, T, n_in), np.float32) if record_states else None
    for t in range(T):
        if record_states:
            states[:, t] = obs
        if stats is not None:   # worker/agent.py:37-39 (raw obs, before normalisation)
            coin = obs_stats.lane_coins(seed, lanes, t, obs_chance)
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
            ent += pol.categorical_entropy(p)
        else:
            mean, std = pol.lanes_forward(kind, n_in, n_act, thetas, x)
            z = crng.normal(seed, lanes[:, None], t, np.arange(n_act, dtype=np.uint64)[None, :])
            act = np.where(det[:, None], mean, (mean + std * z).astype(np.float32)).astype(np.float32)
            ent += pol.normal_entropy(std)
        obs, r = env.step(act)
        ret += r
    ent /= T
    if jiggle:
        ret += crng.jiggle(seed, lanes)
    out = (ret, ent, np.full(L, T, dtype=np.int32), norm2)
    if stats is not None:
        out = out + (stats,)
    if record_states:
        out = out + (states,)
    return out
