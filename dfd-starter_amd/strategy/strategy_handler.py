"""Novelty archive -- the API of strategy/strategy_handler.py:6-31 (not a hot-path row).

A strategy is policy.get_strategy(zeta) (the HIP forward over the probe states zeta); novelty is
the minimum distance to the archived strategies (utils/math_helpers.py:147-155).  When the archive
is full, a new point replaces one member of the closest pair if it is more novel than that pair's
distance (sparse_history_manager.py:73-109, simplified bookkeeping).  Novelty is reported but, as in
the reference, not used by the objective (learner/finite_differences.py:48).
"""
import numpy as np

from utils import math_helpers


class StrategyHandler(object):
    def __init__(self, policy, strategy_distance_fn, max_history_size=200):
        self.policy = policy
        self.strategy_distance_fn = strategy_distance_fn
        self.max_history_size = max_history_size
        self.points = []              # flat parameter vectors (host)
        self.strategy_tensor = np.zeros(0)
        self.zeta = None

    def _strategy(self, flat):
        old = self.policy.get_trainable_flat()
        self.policy.set_trainable_flat(flat)
        s = self.policy.get_strategy(self.zeta)
        self.policy.set_trainable_flat(old)
        return s

    def add_policy(self, policy):
        flat = policy.get_trainable_flat()
        if len(self.points) < self.max_history_size or self.zeta is None or len(self.zeta) == 0:
            self.points.append(flat)
            if self.zeta is not None and len(self.zeta):
                self.set_zeta(self.zeta)
            return None
        s = self._strategy(flat)
        nov, dists = math_helpers.compute_strategy_novelty(s, self.strategy_tensor, True, self.strategy_distance_fn)
        n = len(self.points)
        pair = np.array([[math_helpers.compute_strategy_distance(self.strategy_tensor[i], self.strategy_tensor[j],
                                                                 self.strategy_distance_fn) if i != j else np.inf
                          for j in range(n)] for i in range(n)])
        i, j = np.unravel_index(np.argmin(pair), pair.shape)
        if nov > pair[i, j]:
            second = np.sort(pair, axis=1)[:, 1] if n > 2 else np.zeros(n)
            k = i if second[i] <= second[j] else j
            self.points[k] = flat
            self.strategy_tensor[k] = s
            return k
        return -1

    def set_zeta(self, zeta):
        if zeta is None or len(zeta) == 0:
            return
        self.zeta = np.asarray(zeta)
        self.strategy_tensor = np.asarray([self._strategy(f) for f in self.points])

    def compute_novelty(self, policy):
        if self.zeta is None or len(self.zeta) == 0 or self.strategy_tensor is None or len(self.strategy_tensor) < 2:
            return 0
        s = policy.get_strategy(self.zeta)
        return math_helpers.compute_strategy_novelty(s, self.strategy_tensor, distance_fn=self.strategy_distance_fn)
