"""SparseHistoryManager restatement (strategy/sparse_history_manager.py:6-148, strategy/strategy_point.py:27-39).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  The archive of strategy points with the reference's
known-distance table, closest / second-closest bookkeeping and least-novel replacement rule, on numpy
strategies.  Pinned by tests/golden/g12_history.npz (made by the reference's own SparseHistoryManager).
"""
import numpy as np

from .novelty import DISTANCES


class History(object):
    def __init__(self, kind, max_history_size):
        self.dist = DISTANCES[kind]
        self.max_history_size = max_history_size
        self.strategies = []          # None until evaluated (submit before set_zeta appends unevaluated points)
        self.known = {}               # (i, j), i < j -> distance, in insertion order (sparse_history_manager.py:59-67)
        self.worst_point_idx = 0
        self.closest = []
        self.second = []

    def _d(self, a, b):
        return float(np.mean(self.dist(a, b[None])))

    def submit(self, strategy, ready):
        """submit_policy (:17-30): append until full; once full and zeta is set, _replace_point."""
        if len(self.strategies) >= self.max_history_size and ready:
            return self._replace(strategy)
        self.strategies.append(strategy)
        return None

    def evaluate(self, strategies):
        """evaluate_strategies (:32-47) + _construct_table (:49-71)."""
        self.strategies = list(strategies)
        n = len(self.strategies)
        self.known = {}
        for i in range(n):
            for j in range(i + 1, n):
                self.known[(i, j)] = self._d(self.strategies[i], self.strategies[j])
        self._update()

    def _replace(self, strategy):
        """_replace_point (:73-109)."""
        dists = [self._d(strategy, s) for s in self.strategies]
        novelty = min(dists)
        idx = self.worst_point_idx
        current_worst = self.closest[idx][1]
        if novelty > current_worst or current_worst == np.inf:
            self.strategies[idx] = strategy
            for pair in self.known:
                if idx in pair:
                    self.known[pair] = dists[pair[1 - pair.index(idx)]]
            self._update()
            return idx
        return -1

    def _update(self):
        """_update_strategy_point_dists (:111-148) with StrategyPoint.add_dist (strategy_point.py:27-35)."""
        n = len(self.strategies)
        self.closest = [[None, np.inf] for _ in range(n)]
        self.second = [[None, np.inf] for _ in range(n)]
        for i in range(n):
            for key, val in self.known.items():
                if i in key:
                    c, s = self.closest[i], self.second[i]
                    if val < c[1]:
                        self.second[i] = c[:]
                        self.closest[i] = [key, val]
                    elif val < s[1] and key != c[0]:
                        self.second[i] = [key, val]
        worst_dist = np.inf
        for i in range(n):
            key, d = self.closest[i]
            if d < worst_dist:
                if key is None:
                    self.worst_point_idx = i
                    continue
                j = key[1 - key.index(i)]
                worst_dist = d
                self.worst_point_idx = i if self.second[i][1] < self.second[j][1] else j
