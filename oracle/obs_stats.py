"""WelfordRunningStat (utils/math_helpers.py:7-124) -- f32 restatement, and the rollout's sampled
per-lane statistics (worker/agent.py:37-39).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py); pinned by tests/golden/g10_welford.npz, produced
by the reference class itself.
"""
import numpy as np

from . import rng as crng


class Welford(object):
    def __init__(self, d):
        self.d = d
        self.mean_ = np.zeros(d, np.float32)     # running_mean
        self.m2 = np.zeros(d, np.float32)        # running_variance (sum of squared deviations)
        self.count = 0

    def update(self, x):
        """math_helpers.py:29-38."""
        cc = self.count
        self.count += 1
        delta = (np.asarray(x, np.float32) - self.mean_).astype(np.float32)
        delta_n = (delta / np.float32(self.count)).astype(np.float32)
        self.mean_ = (self.mean_ + delta_n).astype(np.float32)
        self.m2 = (self.m2 + ((delta * delta_n).astype(np.float32) * np.float32(cc))).astype(np.float32)

    def merge(self, mean, m2, count):
        """increment_from_obs_stats_update, math_helpers.py:68-87 (f32, the reference's order)."""
        count = int(count)
        if count == 0:
            return
        om = np.asarray(mean, np.float32)
        ov = np.asarray(m2, np.float32)
        c = self.count
        cnt = c + count
        md = (om - self.mean_).astype(np.float32)
        mds = (md * md).astype(np.float32)
        cm = ((np.float32(c) * self.mean_ + np.float32(count) * om) / np.float32(cnt)).astype(np.float32)
        t = (((mds * np.float32(c)).astype(np.float32) * np.float32(count)).astype(np.float32) / np.float32(cnt))
        self.m2 = ((self.m2 + ov).astype(np.float32) + t.astype(np.float32)).astype(np.float32)
        self.mean_ = cm
        self.count = cnt

    def serialize(self):
        return self.mean_.tolist() + self.m2.tolist() + [self.count]

    @property
    def mean(self):
        return np.zeros(self.d, np.float32) if self.count < 2 else self.mean_

    @property
    def std(self):
        if self.count < 2:
            return np.ones(self.d, np.float32)
        var = self.m2 / (self.count - 1)
        return np.sqrt(np.where(var == 0, 1.0, var)).astype(np.float32)


OBS_COIN_K = 14   # counter-stream k of the per-step obs-stat coin (fdr_rollout_ex)


def lane_coins(seed, lanes, t, chance):
    """Coin of lane(s) at step t: uniform(seed, lane, t, 14) < chance (replaces Agent.rng.uniform)."""
    return crng.uniform(seed, lanes, t, OBS_COIN_K) < np.float32(chance)
