"""Environments for the hot path: build-defined synthetic envs + the trap env restatement.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Synthetic fixed-length envs (DESIGN.md "Synthetic envs"): the container has
no MuJoCo / ALE / gym, so "CartPole-shaped" and "HalfCheetah-shaped" workloads use a contractive
linear-tanh system with the real observation/action shapes:

    M = 0.9 * G / ||G||_2,  G ~ randn(obs, obs)              (RandomState(env_seed), f64 -> f32)
    K = randn(obs, act_dim) * 0.5 / sqrt(act_dim)             (same stream)
    s0 = 0.5 * randn(obs)                                     (same stream)
    step(a):  u = K[:, a] (discrete)  |  K @ a (continuous)
              s <- tanh(M s + u)   (f32);  reward = s[0];  t += 1;  done = t >= T
              (terminating variant, done_threshold > 0:  done also when |s[done_dim]| > done_threshold)

The per-step contract (obs returned after the step, reward, done, reset on done) is that of a
gym env as consumed by worker/agent.py:35-52.

TrapEnv restates custom_envs/simple_trap_env/{environment.py:8-61, tile_map.py:11-56,
node.py:9-14}: the walkable bitmap is a data fixture (tests/golden/trap_map.npz) taken from the
reference's own TileMap; action a moves (dx, dy) = (a // 3 - 1, a % 3 - 1) unless the target is
out of the map (stay, tile_map.py:19-23) or not walkable (stay, node.py:12-13); reward is the
x-displacement in pixels (environment.py:40-42); done when the pre-increment step counter is
>= 200 (environment.py:43-45), i.e. 201 steps per episode.  The action-log side effect of
environment.py:50-52,63-75 is deliberately omitted.
"""
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
TRAP_MAP_PATH = os.path.join(os.path.dirname(_HERE), "tests", "golden", "trap_map.npz")


def synthetic_params(obs_dim, act_dim, env_seed=0):
    rng = np.random.RandomState(env_seed)
    G = rng.randn(obs_dim, obs_dim)
    M = (0.9 * G / np.linalg.norm(G, 2)).astype(np.float32)
    K = (rng.randn(obs_dim, act_dim) * (0.5 / np.sqrt(act_dim))).astype(np.float32)
    s0 = (0.5 * rng.randn(obs_dim)).astype(np.float32)
    return M, K, s0


class SyntheticEnv(object):
    """One env instance (gym-style API) -- used by the per-lane CPU loop."""

    def __init__(self, obs_dim, act_dim, discrete, episode_len, env_seed=0, done_threshold=0.0, done_dim=0):
        self.done_threshold, self.done_dim = float(done_threshold), int(done_dim)
        self.obs_dim = obs_dim
        self.act_dim = act_dim
        self.discrete = discrete
        self.episode_len = episode_len
        self.M, self.K, self.s0 = synthetic_params(obs_dim, act_dim, env_seed)
        self.s = self.s0.copy()
        self.t = 0

    def reset(self):
        self.s = self.s0.copy()
        self.t = 0
        return self.s.copy()

    def step(self, action):
        if self.discrete:
            u = self.K[:, int(action)]
        else:
            a = np.asarray(action, dtype=np.float32).reshape(self.act_dim)
            u = self.K @ a
        self.s = np.tanh(self.M @ self.s + u).astype(np.float32)
        self.t += 1
        done = self.t >= self.episode_len or (self.done_threshold > 0 and abs(self.s[self.done_dim]) > self.done_threshold)
        return self.s.copy(), float(self.s[0]), bool(done), {}


class BatchedSyntheticEnv(object):
    """Same dynamics over L lanes at once (numpy), for batched parity checks."""

    def __init__(self, obs_dim, act_dim, discrete, episode_len, n_lanes, env_seed=0, done_threshold=0.0, done_dim=0):
        self.done_threshold, self.done_dim = float(done_threshold), int(done_dim)
        self.obs_dim, self.act_dim, self.discrete = obs_dim, act_dim, discrete
        self.episode_len = episode_len
        self.M, self.K, self.s0 = synthetic_params(obs_dim, act_dim, env_seed)
        self.n = n_lanes
        self.s = np.tile(self.s0, (n_lanes, 1))

    def reset(self):
        self.s = np.tile(self.s0, (self.n, 1))
        return self.s.copy()

    def step(self, actions):
        if self.discrete:
            u = self.K.T[np.asarray(actions, dtype=np.int64)]          # [L, obs]
        else:
            u = np.einsum("oa,la->lo", self.K, np.asarray(actions, dtype=np.float32))
        pre = np.einsum("ok,lk->lo", self.M, self.s).astype(np.float32) + u
        self.s = np.tanh(pre).astype(np.float32)
        return self.s.copy(), self.s[:, 0].astype(np.float64)

    def failed(self):
        """Per lane: the state after the last step ends the episode (terminating variant; the T limit aside)."""
        if self.done_threshold <= 0:
            return np.zeros(self.n, bool)
        return np.abs(self.s[:, self.done_dim]) > self.done_threshold


def load_trap_map(path=TRAP_MAP_PATH):
    with np.load(path) as z:
        return z["walkable"].astype(bool)


class TrapEnv(object):
    """custom_envs/simple_trap_env/environment.py:8-61 (state machine only)."""

    NODE_RADIUS = 7            # tile_map.py:6
    MAX_X, MAX_Y = 1918, 1071  # environment.py:23-24
    EPISODE_LENGTH = 200       # environment.py:19

    def __init__(self, walkable=None):
        self.walkable = load_trap_map() if walkable is None else walkable
        self.height, self.width = self.walkable.shape
        # environment.py:21 -> tile_map.get_node(width*r//2, height*r//2) (tile_map.py:51-56)
        r = self.NODE_RADIUS
        self.start_col = (self.width * r // 2) // r
        self.start_row = (self.height * r // 2) // r
        self.goal_x = self.MAX_X   # environment.py:29
        self.reset()

    def reset(self):
        self.col, self.row = self.start_col, self.start_row
        self.current_step = 0
        return self.form_obs()

    def form_obs(self):
        # environment.py:59-61 (x, y are pixel coordinates = tile index * node_radius)
        return np.asarray([self.col * self.NODE_RADIUS / self.MAX_X, self.row * self.NODE_RADIUS / self.MAX_Y])

    def step(self, action):
        a = int(action)
        prev_x = self.col * self.NODE_RADIUS
        if 0 <= a < 9:                                   # node.py:10-11
            tc = self.col + a // 3 - 1                   # tile_map.py:15-18 link order
            tr = self.row + a % 3 - 1
            if 0 <= tc < self.width and 0 <= tr < self.height and self.walkable[tr, tc]:
                self.col, self.row = tc, tr
        curr_x = self.col * self.NODE_RADIUS
        reward = (self.goal_x - prev_x) - (self.goal_x - curr_x)   # environment.py:40-42
        done = self.current_step >= self.EPISODE_LENGTH            # environment.py:43
        self.current_step += 1
        return self.form_obs(), reward, done, {}
