"""FiniteDifferences -- the reference learner's API (learner/finite_differences.py:6-114) on the GPU.

``step(batch, policy_reward, policy_novelty, policy_entropy)`` accepts either the reference's
list of FDReturn or an FDBatch (device SoA from Worker.evaluate) and runs, all on the device:

    fdr_fd_grad_fused  ONE launch: z = standardize(r - r_pol) over the batch, coef_d = sum_i z_i s_i sigma /
                       ||lambda_i||^2, g = sum_d coef_d * table[idx_d : idx_d + P] (f64, fixed order, chunk
                       partials combined in-launch)
    fdr_dsgd_step      ONE launch (P <= 65536): theta <- theta - lr*sqrt(P)*lr_scale * fl32(-g) / ||fl32(-g)||

Sharded over ranks (DESIGN.md "Multi-GPU") the z-score step needs ONE collective: every rank reduces its lanes
to the moments [A | B | n | r' slots] (A = sum r'_i v_i, B = sum v_i; its r' at its global lanes, 0 elsewhere),
one RCCL all-reduce sums them, and DSGD forms m, sd in two passes over all r' and g = (A - m B) / sd on the fly
(equal to the z-weighted sum in real arithmetic, B = 0 exactly for antithetic pairs).  One-sided
batches, and batches whose lane split is not known on every rank (a list of FDReturn), all-gather the returns
instead.
``weighting="centred_rank"`` (build extension named by the north star; the reference's weighting is the
z-score) ranks all returns, so it keeps the all-gather of the per-lane returns + the all-reduce of g.

Returns carry a current epoch in the synchronous engine; returns from an older epoch (the
reference's async server mode) add the parameter drift theta_epoch - theta_now to lambda
(finite_differences.py:66-92) -- fdr_fd_lambda_norms / fdr_fd_grad_lambda, single-process or sharded
(a list of FDReturn on every rank: counts + rewards all-gathered, one all-reduce of g).
"""
import numpy as np
import torch

from dsgd import DSGD
from fdr import dist as fdist
from fdr import engine
from utils import math_helpers
from utils.noise_sources import HostNoiseRows, is_host_noise, require_noise_source

from .fd_return import FDBatch

FUSED_STEP_MAX_P = 1 << 16   # fdr_fd_step fuses DSGD into the gradient launch up to this many parameters


class FiniteDifferences(object):
    def __init__(self, policy, gradient_optimizer, omega, noise_source, noise_std=0.1, batch_size=100,
                 ent_coef=0.0, max_delayed_return=10, process_group=None, weighting="zscore", one_collective=True):
        if weighting not in ("zscore", "centred_rank"):
            raise ValueError("weighting must be 'zscore' (the reference) or 'centred_rank'")
        self.weighting = weighting
        self.one_collective = one_collective
        self.max_delayed_return = max_delayed_return
        self.ent_coef = ent_coef
        self.noise_std = noise_std
        self.policy = policy
        self.gradient_optimizer = gradient_optimizer
        require_noise_source(noise_source, "FiniteDifferences")
        self.noise_source = noise_source
        self._host_noise = is_host_noise(noise_source)
        self.omega = omega
        self.batch_size = batch_size
        self.process_group = process_group
        self.epoch = 0
        self.discarded_returns = 0
        self.policy_history = [(policy.flat.detach().clone(), 0)]
        self.dist_map = {0: None}
        self.using_dsgd = isinstance(gradient_optimizer, DSGD)
        P = policy.num_params
        self.gradient_memory = torch.zeros(P, dtype=torch.float64, device=policy.flat.device)
        self._out = torch.zeros(2, dtype=torch.float64, device=policy.flat.device)
        # policy_history entries written by the DSGD launch itself (no per-step copy): a ring one longer than
        # the history, so a slot is rewritten only after its entry left the history
        self._hist_ring = None
        self._hist_next = 0

    # ------------------------------------------------------------------------------------------
    def _distributed(self):
        return fdist.active(self.process_group)

    def step(self, batch, policy_reward, policy_novelty, policy_entropy):
        """Reference signature; returns the update magnitude ||d theta|| as a float."""
        out = self.step_async(batch, policy_reward, policy_novelty, policy_entropy)
        if out is None:
            return 0
        upd, gnorm = out.tolist()
        assert gnorm > 0, "DSGD ENCOUNTERED GRADIENT WITH NORM OF ZERO"   # dynamic_sgd.py:28
        return upd

    def step_async(self, batch, policy_reward, policy_novelty, policy_entropy):
        """Same as step() but leaves (||d theta||, ||grad||) on the device: no host sync."""
        if policy_reward is None:
            policy_reward = 0
        if isinstance(batch, FDBatch):
            return self._step_batch(batch, float(policy_reward))
        return self._step_returns(list(batch), float(policy_reward))

    # ------------------------------------------------------------------------------------------
    def _table(self, b=None):
        """What lambda is gathered from: a host-noise batch's own fl32(noise) rows, else the shared table."""
        t = getattr(b, "noise_table", None) if b is not None else None
        if t is not None:
            return t
        if self._host_noise:
            raise ValueError("a host noise source's FDBatch carries its noise rows (Worker.evaluate sets noise_table)")
        return self.noise_source.device_table(self.policy.flat.device)

    def _step_batch(self, b, policy_reward):
        table = self._table(b)
        if not np.all(b.sign_host != 0):
            raise ValueError("FDBatch for the learner must not contain eval lanes (sign 0)")
        P = self.policy.num_params
        if not self._distributed():
            if P <= FUSED_STEP_MAX_P:   # the whole step in one launch: weights + gradient + DSGD
                lr, lr_scale = self._lr()
                slot = self._hist_slot()
                engine.fd_step(table, b.idx, b.reward, policy_reward, b.sign, b.norm2, b.lanes_per_dir, self.noise_std,
                               self.policy.flat, lr, lr_scale, mode=self.weighting, g=self.gradient_memory, out=self._out,
                               theta_hist=slot)
                return self._after_update(slot)
            g = engine.fd_grad_fused(table, b.idx, b.reward, policy_reward, 0, b.sign, b.norm2, b.lanes_per_dir,
                                     self.noise_std, P, mode=self.weighting, out=self.gradient_memory)
            return self._apply(g)
        sizes = getattr(b, "rank_lanes", None)
        if self.weighting == "zscore" and self.one_collective and sizes is not None and b.lanes_per_dir == 2:
            # the split is known on every rank (Worker.evaluate's lane_range): [A | B | n | r' slots], ONE all-reduce.
            # Antithetic only: there B = 0 exactly, so A - m B carries no cancellation; one-sided batches with
            # near-constant returns (|m| >> sd) would lose digits in it, and take the exact gather path below.
            ws, rank = fdist.world_rank(self.process_group)
            if len(sizes) != ws or int(sizes[rank]) != b.reward.numel():
                # the slots of [A | B | n | r'] would overlap or leave gaps: m, sd and g silently wrong
                raise ValueError("FDBatch.rank_lanes %s does not match the learner's process group (world %d, rank "
                                 "%d, %d local lanes)" % (list(sizes), ws, rank, b.reward.numel()))
            mom = engine.fd_grad_fused(table, b.idx, b.reward, policy_reward, int(sum(sizes[:rank])), b.sign, b.norm2,
                                       b.lanes_per_dir, self.noise_std, P, mode="moments", n_all=int(sum(sizes)))
            fdist.allreduce_grad(mom, self.process_group)            # the step's one collective
            return self._apply(mom, moments=True)
        rewards_all, lane_lo = fdist.gather_rewards(b.reward, self.process_group, getattr(b, "rank_lanes", None))
        g = engine.fd_grad_fused(table, b.idx, rewards_all, policy_reward, lane_lo, b.sign, b.norm2,
                                 b.lanes_per_dir, self.noise_std, P, mode=self.weighting, out=self.gradient_memory)
        fdist.allreduce_grad(g, self.process_group)
        return self._apply(g)

    def _lr(self):
        if self.using_dsgd:
            self.gradient_optimizer.adjust_lr(self.omega)
            return self.gradient_optimizer.lr, self.gradient_optimizer.lr_scale
        return self.gradient_optimizer.param_groups[0]["lr"], 1.0

    def _hist_slot(self):
        if self._hist_ring is None:
            n = max(1, self.max_delayed_return) + 1
            self._hist_ring = torch.empty((n, self.policy.num_params), dtype=torch.float32, device=self.policy.flat.device)
        slot = self._hist_ring[self._hist_next]
        self._hist_next = (self._hist_next + 1) % self._hist_ring.shape[0]
        return slot

    def _after_update(self, hist=None):
        self.gradient_optimizer.steps = getattr(self.gradient_optimizer, "steps", 0) + 1
        self.epoch += 1
        self._build_distance_map()
        self._update_policy_history(hist)
        return self._out

    def _apply(self, src, moments=False):
        lr, lr_scale = self._lr()
        engine.dsgd_step_ex(self.policy.flat, src, moments, lr, lr_scale, g_out=self.gradient_memory if moments else None,
                            out=self._out)
        return self._after_update()

    def _build_distance_map(self):
        # finite_differences.py:66-73: dist_map[ep] = theta_ep - theta_now for the recent epochs.  The
        # differences are formed on first use (only stale returns read them), not eagerly every step.
        self.dist_map = _LazyDistMap(self.epoch, self.policy_history, self.policy.flat.detach())

    def _update_policy_history(self, hist=None):
        # finite_differences.py:75-78; hist: theta already copied by the DSGD launch (fdr_fd_step theta_hist)
        self.policy_history.append((self.policy.flat.detach().clone() if hist is None else hist, self.epoch))
        while len(self.policy_history) > self.max_delayed_return:
            self.policy_history.pop(0)

    # ------------------------------------------------------------------------------------------
    def _step_returns(self, rets, policy_reward):
        """list[FDReturn] path (finite_differences.py:24-64, 80-114)."""
        keep = []
        for r in rets:
            if r.epoch not in self.dist_map:
                print("FINITE DIFFERENCE LEARNER RECEIVED RETURN THAT WAS TOO OLD")
                print("RECEIVED EPOCH:", r.epoch, "ACCEPTABLE EPOCHS:", list(self.dist_map.keys()))
                self.discarded_returns += 1
                continue
            keep.append(r)
        if self._distributed():
            # every rank joins the exchange, even with no (kept) returns of its own
            return self._step_returns_lambda(keep, policy_reward)
        if not keep:
            return None
        dev = self.policy.flat.device
        P = self.policy.num_params
        if self._host_noise:
            # finite_differences.py:94: decode() regenerates each return's noise vector on the host (f64); the device
            # gathers lambda_i = sign fl32(sigma fl32(noise_i)) (+ drift) from those rows
            return self._step_returns_lambda(keep, policy_reward)
        table = self.noise_source.device_table(dev)
        current = [r for r in keep if self.dist_map[r.epoch] is None]
        stale = [r for r in keep if self.dist_map[r.epoch] is not None]
        if stale:
            # finite_differences.py:88-114: lambda_i = sigma * eps_i + dist_map[epoch_i], v_i = lambda_i / ||lambda_i||^2
            return self._step_returns_lambda(keep, policy_reward)
        rewards = torch.as_tensor([r.reward for r in current], dtype=torch.float64, device=dev)
        idx = np.array([int(r.encoded_noise) for r in current], dtype=np.int64)
        sign = np.array([int(getattr(r, "sign", 1) or 1) for r in current], dtype=np.int8)
        idx_d = torch.as_tensor(idx, device=dev)
        sign_d = torch.as_tensor(sign, device=dev)
        if all(getattr(r, "norm2", None) is not None for r in current):
            n2 = torch.as_tensor([r.norm2 for r in current], dtype=torch.float64, device=dev)
        else:
            n2 = engine.fd_lambda_norms(table, idx_d, sign_d, None, self.noise_std, None, P)
        b = FDBatch(rewards, None, None, n2, idx_d, sign_d, idx, sign, self.epoch)
        return self._step_batch(b, policy_reward)


    def _step_returns_lambda(self, keep, policy_reward):
        """list[FDReturn] with the lambda kernels: delayed returns single-process, and every sharded list step (finite_differences.py:24-64, 80-114; the
        reference's server accepts returns up to max_delayed_return epochs old, networking/server.py:83-89).
        Sharded, each rank holds its own returns; the policy history -- hence dist_map -- is replicated (every rank applies
        the same DSGD step), so each rank forms its lambda_i = sign_i fl32(sigma eps_i) + dist_map[epoch_i] alone.
        Exchange: the per-rank return counts + an all-gather of the rewards (the z-score is global), then ONE
        all-reduce of g.  Every rank takes this path for every list step, stale returns or not, so the ranks'
        collectives always match."""
        dev = self.policy.flat.device
        P = self.policy.num_params
        n = len(keep)
        if self._host_noise:
            noises = np.stack([self.noise_source.decode(r.encoded_noise) for r in keep]) if n else np.zeros((0, P))
            rows = HostNoiseRows(np.zeros(P, np.float32), noises, np.arange(n), np.ones(n, np.int8), self.noise_std,
                                 dev, with_theta=False)
            table, idx_host = rows.table, rows.idx_host
        else:
            table = self.noise_source.device_table(dev)
            idx_host = np.array([int(r.encoded_noise) for r in keep], np.int64)
        sizes = fdist.exchange_counts(n, dev, self.process_group)
        if sum(sizes) == 0:
            return None
        epochs = sorted({r.epoch for r in keep if self.dist_map[r.epoch] is not None})
        drift = torch.stack([self.dist_map[e] for e in epochs]).contiguous() if epochs else None
        slot_of = {e: k for k, e in enumerate(epochs)}
        rewards = torch.as_tensor([r.reward for r in keep], dtype=torch.float64, device=dev)
        rewards_all, lane_lo = fdist.gather_rewards(rewards, self.process_group, sizes)
        g = self.gradient_memory
        if n:
            idx_d = torch.as_tensor(idx_host, device=dev)
            sign_d = torch.as_tensor(np.array([int(getattr(r, "sign", 1) or 1) for r in keep], np.int8), device=dev)
            slot_d = torch.as_tensor(np.array([slot_of.get(r.epoch, -1) for r in keep], np.int32), device=dev)
            n2 = engine.fd_lambda_norms(table, idx_d, sign_d, slot_d, self.noise_std, drift, P)
            if self.weighting == "centred_rank":   # ranks over all returns, v_i = lambda_i / ||lambda_i||^2
                coef = engine.rank_weights(rewards_all, lane_lo, n) / n2
            else:
                ones = torch.ones(n, dtype=torch.int8, device=dev)
                coef = engine.fd_weights(rewards_all, policy_reward, lane_lo, ones, n2, 1, 1.0)
            g = engine.fd_grad_lambda(table, idx_d, sign_d, slot_d, coef, self.noise_std, drift, P, g)
        else:
            g.zero_()
        fdist.allreduce_grad(g, self.process_group)
        return self._apply(g)


class _LazyDistMap(object):
    """The learner's epoch -> drift map (finite_differences.py:66-73) with the same keys and values as the
    reference's eager dict: None for the current epoch, theta_ep - theta_now (device f32) for the epochs
    in the policy history.  A difference is computed on first access and cached; theta_now is the
    learner's parameter tensor, which only changes in the next step, when the map is rebuilt."""

    def __init__(self, epoch, history, flat):
        self._cur = epoch
        self._hist = {ep: params for params, ep in history}
        self._flat = flat
        self._cache = {}

    def __contains__(self, ep):
        return ep == self._cur or ep in self._hist

    def __getitem__(self, ep):
        if ep in self._hist:
            if ep not in self._cache:
                self._cache[ep] = self._hist[ep] - self._flat
            return self._cache[ep]
        if ep == self._cur:
            return None
        raise KeyError(ep)

    def keys(self):
        return [self._cur] + [ep for ep in self._hist if ep != self._cur]

    def __len__(self):
        return len(self.keys())

