"""Agent -- worker/agent.py:5-71.  Owns the policy and the (GPU-resident) env.

The per-step host loop of the reference is replaced by whole-episode rollouts inside the
fdr_rollout kernel; ``collect_return`` keeps the single-episode API by launching one lane.
Observation normalisation uses FIXED learner statistics (agent.py:37-41), passed to the kernel.
The per-step Welford sampling of agent.py:37-39 is built: with ``normalize_obs`` every
lane samples its raw observations inside the rollout (``fdr_rollout_ex`` per-lane partials, the same
coin chance), and the learner folds them in lane order with ``fdr_obs_stats_merge``
(``Worker.launch`` passes the chance; ``learner.fd_return.obs_partials`` carries the partials).
"""
import numpy as np
import torch

from fdr import engine
from utils.math_helpers import WelfordRunningStat

TS_LIMIT = 10000     # agent.py:12


class Agent(object):
    def __init__(self, policy, env, random_seed, normalize_obs=False, obs_stats_update_chance=0.01):
        self.policy = policy
        self.env = env
        self.rng = np.random.RandomState(random_seed)
        self.random_seed = random_seed
        self._ts_pending = []          # device step counts not yet folded in (add_timesteps)
        self.cumulative_timesteps = 0
        self.ts_limit = TS_LIMIT
        if env.episode_len > self.ts_limit:
            raise ValueError("episode_len %d exceeds the reference's ts_limit %d" % (env.episode_len, self.ts_limit))
        self.obs_stats = WelfordRunningStat(policy.input_shape)
        self.normalize_obs = normalize_obs
        self.obs_stats_update_chance = obs_stats_update_chance
        self.saved_states = []
        self._episodes = 0

    @property
    def cumulative_timesteps(self):
        """env.step calls so far (agent.py:55).  Device counts queued by add_timesteps are summed on read, so a
        batched step over a terminating env needs no host sync to count its true steps."""
        if self._ts_pending:
            self._ts_host += int(torch.stack(self._ts_pending).sum().item())
            self._ts_pending = []
        return self._ts_host

    @cumulative_timesteps.setter
    def cumulative_timesteps(self, v):
        self._ts_pending = []
        self._ts_host = int(v)

    def add_timesteps(self, steps_dev):
        """Queue a device tensor of per-lane step counts (summed on the device now, read on demand)."""
        self._ts_pending.append(steps_dev.sum(dtype=torch.int64))

    def obs_norm_tensors(self, mean, std):
        if not self.normalize_obs:
            return None, None
        dev = self.policy.flat.device
        m = torch.as_tensor(np.broadcast_to(np.asarray(mean, np.float32), (self.policy.input_shape,)).copy(), device=dev)
        s = torch.as_tensor(np.broadcast_to(np.asarray(std, np.float32), (self.policy.input_shape,)).copy(), device=dev)
        return m, s

    def next_seed(self, n=1):
        """Key of the counter random stream for the next n episodes' action sampling."""
        s = (int(self.random_seed) * 1000003 + self._episodes) & ((1 << 63) - 1)
        self._episodes += n
        return s

    def collect_return(self, eval_run=False, save_states=False, mean=1, std=0):
        p = self.policy
        det = torch.full((1,), 1 if eval_run else 0, dtype=torch.int8, device=p.flat.device)
        lanes = engine.lanes_desc(p.flat, 0, deterministic=det)
        om, osd = self.obs_norm_tensors(mean, std)
        bm, bv = p.bn_stats()
        if p.KIND == "impala":   # one env, one episode of the synthetic frame env
            spec = engine.ImpalaSpec(p.output_shape, 1, self.env.episode_len, entropy=self.env.entropy,
                                     env_seed=self.env.env_seed, fp16=getattr(self.env, "fp16", False))
            res = engine.impala_rollout(spec, lanes, 1, self.next_seed(), jiggle=False, bn_mean=bm, bn_var=bv,
                                        device=p.flat.device)
        elif p.KIND == "atari":
            spec = engine.AtariSpec(p.output_shape, 1, self.env.episode_len, env_seed=self.env.env_seed)
            res = engine.atari_rollout(spec, lanes, 1, self.next_seed(), jiggle=False, bn_mean=bm, bn_var=bv,
                                       device=p.flat.device)
        else:
            res = engine.rollout(p.spec, self.env, lanes, 1, self.next_seed(), jiggle=False, obs_mean=om,
                                 obs_std=osd, bn_mean=bm, bn_var=bv, device=p.flat.device)
        steps = int(res.timesteps.item())
        self.cumulative_timesteps += steps
        reward = float(res.reward.item()) + self.rng.choice((-1e-12, 1e-12))   # agent.py:69
        if save_states:
            self.saved_states = []   # visited states are not materialised by the kernel
        return reward, float(res.entropy.item()), steps
