"""GPU-resident environments stepped inside the rollout kernel.

The reference steps gym envs on the host (worker/agent.py:44).  The MI355X engine fuses the env
into the rollout kernel, so an env here is a *descriptor*: device tensors + shape, handed to
``fdr_rollout`` through ``fdr_env_desc`` (include/fdr.h).

* ``SyntheticEnv`` -- the build-defined fixed-length workload (DESIGN.md "Synthetic envs"):
  contractive linear-tanh dynamics with the real obs/action shapes ("CartPole-shaped" obs 4 /
  2 actions; "HalfCheetah-shaped" obs 17 / 6 action dims):
      M = 0.9 G / ||G||_2, G ~ randn(obs, obs);  K = randn(obs, act) * 0.5 / sqrt(act);
      s0 = 0.5 randn(obs)   (one RandomState(env_seed) stream, in that order)
      s <- tanh(M s + K a)  (a one-hot for discrete actions);  reward = s[0];  done at t = T.
  With ``done_threshold`` > 0 the env also TERMINATES (CartPole-style failure, fdr 0.4): done after the step whose
  next state has |s[done_dim]| > done_threshold -- episodes then end before T, per lane (worker/agent.py:50-52).
* ``TrapEnv`` -- custom_envs/simple_trap_env (environment.py:8-61) on the GPU, integer-exact:
  the reference's walkable bitmap ships as data (custom_envs/simple_trap_env/trap_map.npz).
* ``StackedFrameEnv`` -- the same hash frames as 4 x 84 x 84 stacks for AtariPolicy (fdr_atari_rollout).
* ``FrameEnv`` -- the Atari/procgen-shaped workload of BASELINE configs 4/5 for ImpalaPolicy:
  uint8-valued 3x64x64 frames from a counter hash of (env, t, pixel), a +1/-1/0 reward for hitting
  a hashed target action (or its successor), fixed T; ``envs_per_lane`` envs share one theta'.
  Generated inside the conv kernel (never stored); oracle/impala.py restates it.
"""
import os

import numpy as np
import torch

from fdr import _lib

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRAP_MAP = os.path.join(_PKG, "custom_envs", "simple_trap_env", "trap_map.npz")

SHAPES = {
    "cartpole": dict(obs_dim=4, act_dim=2, discrete=True, episode_len=500),     # BASELINE config 2
    "halfcheetah": dict(obs_dim=17, act_dim=6, discrete=False, episode_len=1000),  # config 3
    # CartPole-shaped with failure termination (|s[1]| > 0.4, a pole-angle analogue), 500-step time limit
    # (thresholds chosen so a random-init policy's episodes spread from a few steps to the limit)
    "cartpole_term": dict(obs_dim=4, act_dim=2, discrete=True, episode_len=500, done_threshold=0.4, done_dim=1),
    # Hopper-shaped (obs 11, act 3) with an "unhealthy" termination on state element 1, 1000-step limit
    "hopper_term": dict(obs_dim=11, act_dim=3, discrete=False, episode_len=1000, done_threshold=0.5, done_dim=1),
}


def synthetic_matrices(obs_dim, act_dim, env_seed=0):
    rng = np.random.RandomState(env_seed)
    G = rng.randn(obs_dim, obs_dim)
    M = (0.9 * G / np.linalg.norm(G, 2)).astype(np.float32)
    K = (rng.randn(obs_dim, act_dim) * (0.5 / np.sqrt(act_dim))).astype(np.float32)
    s0 = (0.5 * rng.randn(obs_dim)).astype(np.float32)
    return M, K, s0


class SyntheticEnv(object):
    def __init__(self, obs_dim, act_dim, discrete, episode_len, env_seed=0, device=None, done_threshold=0.0,
                 done_dim=0):
        self.obs_dim, self.act_dim, self.discrete = int(obs_dim), int(act_dim), bool(discrete)
        self.episode_len = int(episode_len)
        self.done_threshold, self.done_dim = float(done_threshold), int(done_dim)
        if self.done_threshold < 0 or not (0 <= self.done_dim < self.obs_dim):
            raise ValueError("done_threshold must be >= 0 and done_dim in [0, obs_dim)")
        self.env_seed = env_seed
        self.M_host, self.K_host, self.s0_host = synthetic_matrices(obs_dim, act_dim, env_seed)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.M = torch.as_tensor(self.M_host, device=self.device).contiguous()
        self.K = torch.as_tensor(self.K_host, device=self.device).contiguous()
        self.s0 = torch.as_tensor(self.s0_host, device=self.device).contiguous()

    @classmethod
    def named(cls, name, device=None, **kw):
        cfg = dict(SHAPES[name])
        cfg.update(kw)
        return cls(device=device, **cfg)

    def desc(self):
        return _lib.EnvDesc(_lib.FDR_ENV_SYNTH, self.obs_dim, self.act_dim, self.episode_len,
                            self.M.data_ptr(), self.K.data_ptr(), self.s0.data_ptr(), None, 0, 0,
                            self.done_threshold, self.done_dim)

    @property
    def terminates(self):
        """Episodes may end before episode_len (steps then vary per lane)."""
        return self.done_threshold > 0


class TrapEnv(object):
    """custom_envs/simple_trap_env.Environment, stepped on the GPU (201 steps per episode)."""
    obs_dim, act_dim, discrete = 2, 9, True
    episode_len = 201   # environment.py:19,43: done when the pre-increment step counter >= 200

    def __init__(self, device=None):
        with np.load(TRAP_MAP) as z:
            walk = z["walkable"].astype(np.uint8)
        self.map_h, self.map_w = walk.shape
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.walkable = torch.as_tensor(walk, device=self.device).contiguous()

    def desc(self):
        return _lib.EnvDesc(_lib.FDR_ENV_TRAP, 2, 9, self.episode_len, None, None, None,
                            self.walkable.data_ptr(), self.map_w, self.map_h, 0.0, 0)


class FrameEnv(object):
    """Synthetic frame env for ImpalaPolicy rollouts (fdr_impala_rollout)."""
    obs_shape = (64, 64, 3)

    def __init__(self, n_act, episode_len=1000, envs_per_lane=4, env_seed=0, entropy=True, fp16=False):
        self.fp16 = bool(fp16)
        self.act_dim = int(n_act)
        self.episode_len = int(episode_len)
        self.envs_per_lane = int(envs_per_lane)
        self.env_seed = int(env_seed)
        self.entropy = bool(entropy)

    def spec(self):
        from fdr import engine
        return engine.ImpalaSpec(self.act_dim, self.envs_per_lane, self.episode_len, entropy=self.entropy,
                                 env_seed=self.env_seed, fp16=self.fp16)


class StackedFrameEnv(FrameEnv):
    """Synthetic 4 x 84 x 84 frame stacks for AtariPolicy rollouts (fdr_atari_rollout)."""
    obs_shape = (84, 84, 4)

    def spec(self):
        from fdr import engine
        return engine.AtariSpec(self.act_dim, self.envs_per_lane, self.episode_len, env_seed=self.env_seed)
