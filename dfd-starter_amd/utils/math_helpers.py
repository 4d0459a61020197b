"""Host-side numerics of utils/math_helpers.py (z-score, affine map, Welford, strategy distances).

The hot-path forms of standardize_arr / the gradient live in the fdr_fd_weights kernel; these
host versions back the list-of-FDReturn API and the novelty archive.
"""
import numpy as np


class WelfordRunningStat(object):
    """utils/math_helpers.py:7-124 (parallel-merge form of Welford's running mean / variance)."""

    def __init__(self, shape):
        self.shape = shape
        self.ones = np.ones(shape=shape, dtype=np.float32)
        self.zeros = np.zeros(shape=shape, dtype=np.float32)
        self.running_mean = np.zeros(shape=shape, dtype=np.float32)
        self.running_variance = np.zeros(shape=shape, dtype=np.float32)
        self.count = 0

    def increment(self, samples, num):
        if num > 1:
            for i in range(num):
                self.update(samples[i])
        else:
            self.update(samples)

    def update(self, sample):
        if isinstance(sample, dict):
            sample = sample["frame"]
        prev = self.count
        self.count += 1
        delta = (sample - self.running_mean).reshape(self.running_mean.shape)
        delta_n = (delta / self.count).reshape(self.running_mean.shape)
        self.running_mean += delta_n
        self.running_variance += delta * delta_n * prev

    def reset(self):
        self.__init__(self.shape)

    @property
    def mean(self):
        return self.zeros if self.count < 2 else self.running_mean

    @property
    def std(self):
        if self.count < 2:
            return self.ones
        var = self.running_variance / (self.count - 1)
        return np.sqrt(np.where(var == 0, 1.0, var))

    def increment_from_obs_stats_update(self, upd):
        n = int(np.prod(self.shape))
        om = np.asarray(upd[:n], dtype=np.float32).reshape(self.running_mean.shape)
        ov = np.asarray(upd[n:-1], dtype=np.float32).reshape(self.running_variance.shape)
        oc = upd[-1]
        if oc == 0:
            return
        count = self.count + oc
        d = om - self.running_mean
        self.running_mean = (self.count * self.running_mean + oc * om) / count
        self.running_variance = self.running_variance + ov + d * d * self.count * oc / count
        self.count = count

    def serialize(self):
        return self.running_mean.ravel().tolist() + self.running_variance.ravel().tolist() + [self.count]

    def deserialize(self, other):
        self.reset()
        if other is None:
            return
        n = int(np.prod(self.shape))
        self.running_mean = np.reshape(np.asarray(other[:n], dtype=np.float32), self.shape)
        self.running_variance = np.reshape(np.asarray(other[n:-1], dtype=np.float32), self.shape)
        self.count = other[-1]


def standardize_arr(arr):
    x = np.asarray(arr)
    m, s = x.mean(), x.std()
    if s == 0:
        return x
    return (x - m) / s


def affine_transform(value, from_min, from_max, to_min, to_max):
    if from_max == from_min or to_max == to_min:
        return to_min
    return (value - from_min) * (to_max - to_min) / (from_max - from_min) + to_min


def compute_strategy_novelty(strategy, other_strategies, return_all_dists=False, distance_fn=None):
    dists = (distance_fn or l2_dist)(strategy, other_strategies)
    if return_all_dists:
        return np.min(dists).item(), dists
    return np.min(dists).item()


def compute_strategy_distance(a, b, distance_fn=None):
    return (distance_fn or l2_dist)(a, b).item()


def l2_dist(a, b):
    return np.linalg.norm(b - a, axis=-1).mean(axis=-1)


def categorical_tvd(p1, p2):
    return np.abs(np.subtract(p1, p2)).sum(axis=-1).mean(axis=-1)


def gaussian_wasserstein_dist(m1, s1, m2, s2):
    inside = s1 + s2 - 2 * np.sqrt(s1 * s2)
    return np.square(np.linalg.norm(m1 - m2, axis=-1)) + inside.sum(axis=-1)


def gaussian_wasserstein_dist_from_strategies(a, b):
    n1, n2 = a.shape[-1] // 2, b.shape[-1] // 2
    return gaussian_wasserstein_dist(a[..., :n1], a[..., n1:], b[..., :n2], b[..., n2:]).mean(axis=-1)
