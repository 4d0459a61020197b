"""Novelty archive -- strategy/strategy_handler.py:6-31 + sparse_history_manager.py:6-148 on the GPU
(SURVEY 8f.2).

A strategy is ``policy.get_strategy(zeta)`` over the probe states zeta (discrete: probs; mujoco:
[mean | std]; ImpalaPolicy: probs of the zeta obs run as ONE LSTM sequence, policies/impala.py:24-27);
the archive holds up to ``max_history_size`` strategies as ONE device tensor [H, Z, D].  MLP strategies
come from the HIP policy forward over (policy, state) pairs (``engine.lane_strategies``), ImpalaPolicy
strategies from ``fdr_impala_strategies`` (conv stack over the shared zeta frames, per-lane fc / LSTM
sequence) started from the reset state -- the state Worker._build_ret scores novelty in
(worker/agent.py:66 resets the policy before worker.py:53).  Distances and novelty come from
``fdr_strategy_distances`` (the reference's
``l2_dist`` / ``categorical_tvd`` / ``gaussian_wasserstein_dist_from_strategies``, f64 accumulation).
AtariPolicy (stateless) strategies are its forward over the zeta frames (fdr_atari_strategies: every lane or
archived vector of a call batched, one prep / conv / core launch per 256 vectors).
``lane_novelty`` scores every perturbed lane of a batch in two launches -- the batched form of
``Worker._build_ret``'s per-return ``compute_novelty`` (worker/worker.py:53), which the reference
evaluates on the perturbed policy.  Replacement when full follows ``_replace_point`` /
``_update_strategy_point_dists`` (sparse_history_manager.py:73-148) on the pairwise distance table.

ImpalaPolicy archive state (``carry_state``): by default every archive strategy starts from the reset LSTM state (the
build's zero-state rule).  ``carry_state=True`` reproduces the reference as it is: every
StrategyPoint.evaluate_strategy (strategy_point.py:17-25) runs ``self.policy.get_strategy`` on the handler's ONE
policy object, so each evaluation continues the (h, c) the previous one left in it (policies/impala.py:24-27,
:136-138,184) -- set_zeta evaluates the points in archive order, submit_policy the candidate, compute_novelty the
scored policy, one launch each, all chained through ``policy.state``.  Pinned by G12-impala-unpatched.
``lane_novelty`` stays from the reset state in both modes: the reference's worker scores novelty right after
collect_return's policy.reset() (worker/agent.py:66, worker/worker.py:53).
"""
import numpy as np
import torch

from fdr import engine

# reference distance functions -> fdr_strategy_distances kinds (SURVEY finding 6: the reference's
# run_sequential passes gaussian_wasserstein_dist where the *_from_strategies form is meant)
KIND_BY_NAME = {"l2_dist": "l2", "categorical_tvd": "tvd", "gaussian_wasserstein_dist_from_strategies": "w2",
                "gaussian_wasserstein_dist": "w2"}


class StrategyHandler(object):
    def __init__(self, policy, strategy_distance_fn=None, max_history_size=200, fp16=False, carry_state=False):
        self.policy = policy
        self.fp16 = bool(fp16)        # ImpalaPolicy: strategies in the rollouts' fp16 mode (BASELINE config 5)
        if carry_state and policy.KIND != "impala":
            raise ValueError("carry_state applies to ImpalaPolicy (the only policy with recurrent state)")
        self.carry_state = bool(carry_state)
        self._zeta_done0 = False      # ImpalaPolicy: zeta's first done flag masks the carried state (impala.py:164-170)
        self.strategy_distance_fn = strategy_distance_fn
        name = getattr(strategy_distance_fn, "__name__", "l2_dist") if strategy_distance_fn is not None \
            else "l2_dist"                     # compute_strategy_novelty's default (math_helpers.py:148-149)
        if name not in KIND_BY_NAME:
            raise ValueError("unsupported strategy distance %r" % name)
        self.kind = KIND_BY_NAME[name]
        self.max_history_size = max_history_size
        self.points = []              # archived flat parameter vectors (host, as StrategyPoint.flat)
        self.archive = None           # device f32 [H, Z, D]
        self.pair = None              # host f64 [H, H] known distances (inf on the diagonal)
        self.worst_point_idx = 0
        self.zeta = None              # device f32 [Z, n_in]; ImpalaPolicy: (frames [Z, 3, 64, 64], reward [Z])

    # ---- strategies on the device ------------------------------------------------------------
    def _dev(self):
        return self.policy.flat.device

    def _strategies(self, lanes_fn, n, pairs=False):
        """get_strategy(zeta) of n parameter vectors; lanes_fn(Z) -> lanes descriptor (see engine.lane_strategies).
        pairs: lanes 2p, 2p+1 are antithetic pairs (ImpalaPolicy fp16: the recurrence in the rollout's pair form)."""
        p = self.policy
        bm, bv = p.bn_stats()
        if p.KIND == "impala":
            frames, reward = self.zeta
            spec = engine.ImpalaSpec(p.output_shape, fp16=self.fp16, pairs=pairs)
            return engine.impala_strategies(spec, lanes_fn(1), n, frames, reward, bn_mean=bm, bn_var=bv)
        if p.KIND != "discrete" and p.KIND != "mujoco":
            raise NotImplementedError("strategies of a %s policy" % p.KIND)
        return engine.lane_strategies(p.spec, lanes_fn, n, self.zeta, bm, bv)

    def _carried(self, flat):
        """StrategyPoint.evaluate_strategy with the reference's carried LSTM state: get_strategy of ONE parameter
        vector (device f32 [P]) from self.policy.state, which it leaves at the end-of-sequence state -> [1, Z, A]."""
        p = self.policy
        h, c = (s[:1].reshape(1, 256).clone().contiguous() for s in p.state)
        if self._zeta_done0:
            h.zero_()
            c.zero_()
        frames, reward = self.zeta
        bm, bv = p.bn_stats()
        probs = engine.impala_strategies(engine.ImpalaSpec(p.output_shape, fp16=self.fp16),
                                         engine.lanes_desc(flat, 0), 1, frames, reward, h, c, bm, bv)
        p.state = (h, c)
        return probs

    def _atari_strategies(self, thetas):
        """AtariPolicy.get_strategy (policies/atari.py:31-32: forward(zeta) probs, stateless) of each parameter
        vector in thetas (device f32 [k, P]) -> [k, Z, A]: fdr_atari_strategies over the zeta frames, one call."""
        p = self.policy
        bm, bv = p.bn_stats()
        thetas = thetas.contiguous()
        zeta = torch.as_tensor(self.zeta, dtype=torch.float32, device=self._dev())
        return engine.atari_strategies(p.spec, engine.lanes_desc(thetas, thetas.shape[1]), thetas.shape[0], zeta, bm, bv)

    def _strategies_of_flat(self, flat):
        """get_strategy(zeta) of one parameter vector -> [1, Z, D]."""
        base = torch.as_tensor(np.asarray(flat, np.float32), device=self._dev()).contiguous()
        if self.policy.KIND == "atari":
            return self._atari_strategies(base.view(1, -1))
        if self.carry_state:
            return self._carried(base)
        return self._strategies(lambda Z: engine.lanes_desc(base, 0), 1)

    def _strategies_of_flats(self, flats):
        """Strategies of the archived vectors -> [H, Z, D] (ImpalaPolicy: one launch, lane l reads flats[l])."""
        if self.policy.KIND == "impala" and not self.carry_state:
            base = torch.as_tensor(np.stack([np.asarray(f, np.float32) for f in flats]), device=self._dev())
            base = base.contiguous()
            return self._strategies(lambda Z: engine.lanes_desc(base, base.shape[1]), len(flats))
        return torch.cat([self._strategies_of_flat(f) for f in flats])

    def lane_strategies(self, table, idx, sign, sigma, pairs=False):
        """Strategies of the perturbed lanes theta + sign * sigma * table[idx:] -> [n, Z, D].  pairs: the lanes are
        antithetic pairs (same offset, signs +1 / -1), as the rollout that produced them was told."""
        p = self.policy
        if p.KIND == "atari":   # every lane over the zeta frames, batched (fdr_atari_strategies)
            bm, bv = p.bn_stats()
            zeta = torch.as_tensor(self.zeta, dtype=torch.float32, device=self._dev())
            return engine.atari_strategies(p.spec, engine.lanes_desc(p.flat, 0, table, idx, sign, sigma), idx.numel(),
                                           zeta, bm, bv)

        def lanes(Z):
            return engine.lanes_desc(p.flat, 0, table, idx.repeat_interleave(Z), sign.repeat_interleave(Z), sigma)
        return self._strategies(lanes, idx.numel(), pairs=pairs)

    @property
    def strategy_tensor(self):
        """The reference attribute (run_sequential.py:107,162): the archive as a host array."""
        return np.zeros(0) if self.archive is None else self.archive.cpu().numpy()

    def _ready(self):
        return self.zeta is not None and self.archive is not None and self.archive.shape[0] >= 2

    # ---- reference API -----------------------------------------------------------------------
    def set_zeta(self, zeta):
        """strategy_handler.py:19-24 -> evaluate_strategies + _construct_table (:33-71).  ImpalaPolicy: zeta
        is a list of obs dicts or one stacked dict {frame, reward, done} (impala.py:35-45)."""
        if zeta is None or len(zeta) == 0:
            return
        if self.policy.KIND == "impala":
            fr, rw, dn = self.policy._stack(zeta)
            self.zeta = (fr.to(self._dev()).contiguous(), rw.to(self._dev()).contiguous())
            self._zeta_done0 = bool(dn[0])
        else:
            z = torch.as_tensor(np.asarray(zeta, np.float32), device=self._dev())
            self.zeta = z.reshape(z.shape[0], -1).contiguous()
        if not self.points:
            return
        self.archive = self._strategies_of_flats(self.points).contiguous()
        self._construct_table()

    def _construct_table(self):
        H = self.archive.shape[0]
        _, _, d = engine.strategy_distances(self.archive, self.archive, self.kind, full=True)
        self.pair = d.cpu().numpy()
        self.pair[np.arange(H), np.arange(H)] = np.inf
        self._update_worst()

    def _update_worst(self):
        """_update_strategy_point_dists (:110-148): closest / second-closest per point, then the less
        novel member of the closest pair (first strict minimum in index order, as the reference)."""
        D = self.pair
        n = D.shape[0]
        if n < 2:
            self.worst_point_idx = 0
            return
        closest = np.argmin(D, axis=1)
        cd = D[np.arange(n), closest]
        second = np.sort(D, axis=1)[:, 1] if n > 2 else np.full(n, np.inf)
        worst, worst_dist = 0, np.inf
        for i in range(n):
            if cd[i] < worst_dist:
                j = closest[i]
                worst_dist = cd[i]
                worst = i if second[i] < second[j] else j
        self.worst_point_idx = int(worst)

    def add_policy(self, policy):
        """strategy_handler.py:16-17 -> submit_policy (:17-30) / _replace_point (:73-108)."""
        flat = np.asarray(policy.get_trainable_flat(), np.float32).copy()
        if len(self.points) < self.max_history_size or self.zeta is None or self.archive is None:
            self.points.append(flat)   # the archive is re-evaluated at the next set_zeta, as the reference
            return None
        s = self._strategies_of_flat(flat)
        mn, _, d = engine.strategy_distances(s, self.archive, self.kind, full=True)
        novelty, dists = float(mn.item()), d[0].cpu().numpy()
        idx = self.worst_point_idx
        current_worst = self.pair[idx].min()
        if novelty > current_worst or current_worst == np.inf:
            self.points[idx] = flat
            self.archive[idx] = s[0]
            others = np.arange(self.pair.shape[0]) != idx
            self.pair[idx, others] = dists[others]
            self.pair[others, idx] = dists[others]
            self._update_worst()
            return idx
        return -1

    def compute_novelty(self, policy):
        """strategy_handler.py:26-31: min distance of policy's strategy to the archive (0 if not ready)."""
        if not self._ready():
            return 0
        mn, _ = engine.strategy_distances(self._strategies_of_flat(policy.get_trainable_flat()), self.archive,
                                          self.kind)
        return float(mn.item())

    def lane_novelty(self, table, idx, sign, sigma, pairs=False):
        """Novelty of every perturbed lane (device f64 [n]); zeros if the archive is not ready."""
        if not self._ready():
            return torch.zeros(idx.numel(), dtype=torch.float64, device=self._dev())
        mn, _ = engine.strategy_distances(self.lane_strategies(table, idx, sign, sigma, pairs=pairs), self.archive,
                                          self.kind)
        return mn
