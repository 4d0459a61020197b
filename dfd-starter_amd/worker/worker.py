"""Worker -- worker/worker.py:7-57, batched: one rollout launch evaluates many perturbations.

``evaluate(n_dirs, antithetic)`` is the hot path (north star ``worker.worker.evaluate``): it draws
the noise-table indices on the host in the reference's order (utils/noise_sources.py:44-47), ships
them to the device and runs every (perturbation x env) lane for a whole episode in ONE
fdr_rollout launch.  theta' = theta + sign * fl32(sigma * eps) is formed inside the kernel
(bit-exact with worker.py:28) and never materialised.  The result is an FDBatch (device SoA).

``collect_returns(n)`` keeps the reference's list-of-FDReturn API: the eval coin flips
(worker.py:23) and index draws happen in the reference's order, then all n episodes run in one
launch (eval lanes: unperturbed theta, deterministic actions, worker.py:33-35).
"""
import os

import numpy as np
import torch

from fdr import engine
from learner.fd_return import FDBatch
from utils.math_helpers import WelfordRunningStat
from utils.noise_sources import HostNoiseRows, is_host_noise, require_noise_source


def obs_partials(res):
    """(mean [n, d], m2 [n, d], count [n]) device partials of a rollout run with obs statistics."""
    m = getattr(res, "obs_mean", None)
    return None if m is None else (res.obs_mean, res.obs_m2, res.obs_count)


class Worker(object):
    def __init__(self, policy, agent, noise_source, strategy_handler, sigma=0.02, eval_prob=0.1, random_seed=123):
        self.policy = policy
        self.agent = agent
        require_noise_source(noise_source, "Worker")
        self.noise_source = noise_source
        self._host_noise = is_host_noise(noise_source)   # RNGNoiseSource / SimpleNoiseSource: theta' rows per lane
        self.strategy_handler = strategy_handler
        self.sigma = sigma
        self.epoch = -1
        self.rng = np.random.RandomState(random_seed)
        self.eval_prob = eval_prob
        self.fixed_obs_stats = WelfordRunningStat(policy.input_shape)
        self._pinned = {}      # lane count -> ring of pinned upload slots
        self._copy_stream = None
        self._main_stream = None
        self._lane_consts = {}  # (n_dirs, antithetic, lane_range, world, rank) -> the constant parts of _lanes_of
        self._next = None      # (key, host lanes, device lanes) uploaded ahead by evaluate(prefetch=True)
        self._launch_pairs = False  # the last launch's lanes were antithetic pairs (lane_novelty takes the pair form)

    # ---- hot path ---------------------------------------------------------------------------
    _RING = 64  # upload slots per lane count: an FDBatch's device idx / sign stay valid for the next 63 uploads
    _GEN = 8    # one compute-stream event per 8 uploads bounds slot reuse (_RING >= 2 * _GEN)

    def _lanes_to_device(self, idx, sign, det, defer_wait=False):
        """The three per-lane descriptor arrays in ONE async host-to-device copy, [idx i64 | sign i8 | det i8], on a
        side copy stream: the copy runs as soon as it is enqueued (during the previous step's rollout, the host
        being ahead), and the compute stream waits on its event only if it has not completed (evaluate()).
        defer_wait=True returns (arrays, copy event) and leaves that wait to the consumer: a cross-stream wait
        enqueued behind a running kernel costs ~6-10 us of barrier processing when that kernel ends (rocprofv3 trace).
        r11: the slots (pinned source + device destination) form a ring of _RING -- a per-step device tensor freed
        after cross-stream use (record_stream) made the caching allocator record an event on the compute stream
        each step, which cost the GPU ~6 us of idle barrier processing before the learner (tools/worker_gaps.py).
        A slot's device block is released only after the compute-stream event recorded at most _RING - 1 uploads
        later has fired, i.e. after the rollout that read it."""
        n = len(idx)
        dev = self.policy.flat.device
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(dev)
            self._main_stream = torch.cuda.current_stream(dev)
        main = self._main_stream if torch.cuda.current_stream(dev) == self._main_stream \
            else torch.cuda.current_stream(dev)
        ring = self._pinned.get(n)
        if ring is None:
            ring = self._pinned[n] = {"slots": [], "count": 0, "gen": {}}
        u = ring["count"]
        ring["count"] = u + 1
        k = u % self._RING
        if k == len(ring["slots"]):
            ring["slots"].append({"buf": torch.empty(10 * n, dtype=torch.uint8).pin_memory(), "dev": None,
                                  "ev": torch.cuda.Event(), "used": False})
        slot = ring["slots"][k]
        if u >= self._RING:
            # the event recorded at upload v (v <= u - _GEN) follows the launch of every rollout of uploads < v,
            # which include upload u - _RING, the slot's previous reader
            v = self._GEN * ((u - self._GEN) // self._GEN)
            ring["gen"][v].synchronize()
            ring["gen"].pop(v - self._GEN, None)  # an older generation is no longer needed
        if slot["used"]:
            slot["ev"].synchronize()  # its previous copy has left the pinned buffer (long done)
        if u % self._GEN == 0:
            gev = torch.cuda.Event()
            gev.record(main)
            ring["gen"][u] = gev
        h = slot["buf"].numpy()
        h[:8 * n].view(np.int64)[:] = idx
        h[8 * n:9 * n].view(np.int8)[:] = sign
        h[9 * n:].view(np.int8)[:] = det
        # a fresh block of the copy stream's pool (torch's .to() from pinned memory: ~10 us of host time, where a
        # copy_ into a kept tensor or a direct hipMemcpyAsync cost ~100 us here); no record_stream -- the slot keeps
        # the block until the rollout that read it is proven done (above), so freeing it then records no event
        old = slot["dev"]
        if old is not None and torch._C._storage_Use_Count(old.untyped_storage()._cdata) > 2:
            # a view of the retiring block outlives the ring (an FDBatch kept > _RING - 1 uploads): tell the allocator
            # the compute stream may still read it, so the block is not handed out before that work is done
            old.record_stream(main)
        del old
        slot["dev"] = None
        with torch.cuda.stream(self._copy_stream):
            d = slot["buf"].to(dev, non_blocking=True)
        slot["dev"] = d
        ev = slot["ev"]
        ev.record(self._copy_stream)
        slot["used"] = True
        if not defer_wait:
            main.wait_event(ev)
        arrs = (d[:8 * n].view(torch.int64), d[8 * n:9 * n].view(torch.int8), d[9 * n:].view(torch.int8))
        return (arrs, ev) if defer_wait else arrs

    def launch(self, idx, sign, det, seed=None, out=None, jiggle=True, lane_offset=0, lanes_dev=None, pairs=False,
               timing=None, rows=None):
        """Run one rollout over explicit lanes (host arrays) -> FDBatch (asynchronous).  lanes_dev: the same lanes
        already on the device (idx, sign, det), e.g. uploaded ahead by evaluate(prefetch=True).  pairs: lanes 2p,
        2p+1 are antithetic pairs (checked here) -- an Impala rollout then streams each pair's sigma-eps once
        (fdr_impala_desc.pairs).  timing: a (start, end) pair of torch.cuda.Event recorded on the stream right
        around the rollout launch(es), nothing else inside (bench.py's kernel-time pass)."""
        p = self.policy
        n = len(idx)
        idx_d, sign_d, det_d = lanes_dev if lanes_dev is not None else self._lanes_to_device(idx, sign, det)
        if rows is not None:
            # a host noise source: each lane runs its materialised theta' row, unperturbed in the kernel
            # (fdr_lanes_desc.base_stride = P, no table); norm2 comes from the rows afterwards (_launch_host)
            lanes = engine.lanes_desc(rows.theta, p.num_params, None, idx_d, sign_d, self.sigma, det_d, lane_offset)
            pairs = False
        else:
            table = self.noise_source.device_table(p.flat.device)
            lanes = engine.lanes_desc(p.flat, 0, table, idx_d, sign_d, self.sigma, det_d, lane_offset)
        bm, bv = p.bn_stats()
        if seed is None:
            seed = self.agent.next_seed(n)
        if p.KIND in ("impala", "atari"):
            # E envs per lane: returns are per (lane, env), lane-major; idx / sign / norm2 repeat per env
            E = self.agent.env.envs_per_lane
            roll = engine.impala_rollout if p.KIND == "impala" else engine.atari_rollout
            spec = self.agent.env.spec()
            self._launch_pairs = False
            if pairs and p.KIND == "impala":
                ii, ss, dd = np.asarray(idx), np.asarray(sign).astype(np.int32), np.asarray(det)
                # +eps / -eps training batches only (the pair cores also take sign-0 lanes, include/fdr.h; eval
                # batches keep the per-lane form they were measured in)
                spec.pairs = bool(n % 2 == 0 and np.array_equal(ii[0::2], ii[1::2]) and np.all(ss[0::2] == 1)
                                  and np.all(ss[1::2] == -1) and not np.any(dd))
                self._launch_pairs = spec.pairs
            if timing is not None:
                timing[0].record()
            res = roll(spec, lanes, n, seed, jiggle=jiggle, bn_mean=bm, bn_var=bv, device=p.flat.device)
            if timing is not None:
                timing[1].record()
            if E > 1:
                res.norm2 = res.norm2.repeat_interleave(E)
                idx_d, sign_d = idx_d.repeat_interleave(E), sign_d.repeat_interleave(E)
            return res, idx_d, sign_d
        om, osd = self.agent.obs_norm_tensors(self.fixed_obs_stats.mean, self.fixed_obs_stats.std)
        # agent.py:37-39: with normalize_obs every episode also samples raw obs into its Welford stats
        chance = self.agent.obs_stats_update_chance if self.agent.normalize_obs else None
        if timing is not None:
            timing[0].record()
        self._launch_pairs = False
        res = engine.rollout(p.spec, self.agent.env, lanes, n, seed, jiggle=jiggle, obs_mean=om, obs_std=osd,
                             bn_mean=bm, bn_var=bv, out=out, device=p.flat.device, obs_stats=chance)
        if timing is not None:
            timing[1].record()
        return res, idx_d, sign_d

    def _launch_host(self, noises, row_of_lane, sign, det, lane_offset=0, jiggle=True, seed=None, out=None,
                     timing=None):
        """One rollout over lanes whose perturbations come from a host noise source (RNGNoiseSource /
        SimpleNoiseSource): noises [n_rows, P] f64 in the source's draw order, lane l runs
        theta + sign_l * sigma * noises[row_of_lane[l]] (HostNoiseRows: the reference's f64 formula, rounded to f32).
        -> (res, idx_d, sign_d, rows); res.norm2 = ||sign fl32(sigma fl32(noise))||^2 per lane, idx_d the lanes' row
        offsets into rows.table (what the learner and the lane strategies gather from)."""
        p = self.policy
        rows = HostNoiseRows(p.get_trainable_flat(), noises, row_of_lane, sign, self.sigma, p.flat.device)
        res, idx_d, sign_d = self.launch(rows.idx_host, sign, det, seed=seed, out=out, jiggle=jiggle,
                                         lane_offset=lane_offset, timing=timing, rows=rows)
        E = getattr(self.agent.env, "envs_per_lane", 1)
        li, ls = (idx_d[::E].contiguous(), sign_d[::E].contiguous()) if E > 1 else (idx_d, sign_d)
        if rows.table.numel() >= p.num_params:
            # fd_lambda_norms reads a sign-0 (eval) lane as +1; the rollout reports 0 for it, as here
            n2 = engine.fd_lambda_norms(rows.table, li, ls, None, self.sigma, None, p.num_params) * (ls != 0)
        else:                               # eval lanes only: nothing was drawn
            n2 = torch.zeros(li.numel(), dtype=torch.float64, device=p.flat.device)
        res.norm2 = n2.repeat_interleave(E) if E > 1 else n2
        return res, idx_d, sign_d, rows

    def _lanes_of(self, idx, n_dirs, antithetic, lane_range):
        """Host lane arrays of one evaluate() call from its direction indices: (lidx, sign, det, lane_range,
        rank_lanes).  Everything but lidx depends only on the call's shape and the process group: computed once
        (sign / det are shared read-only arrays)."""
        lpd = 2 if antithetic else 1
        world, rank = (1, 0)
        if lane_range is not None:
            from fdr import dist as fdist
            world, rank = fdist.world_rank()
        ckey = (int(n_dirs), bool(antithetic), lane_range if lane_range is None or lane_range == "auto"
                else tuple(lane_range), world, rank)
        c = self._lane_consts.get(ckey)
        if c is None:
            rank_lanes = None
            d_lo, d_hi = 0, n_dirs
            if lane_range is not None:
                from fdr import dist as fdist
                std = fdist.lane_range(n_dirs, lpd, world, rank)
                if lane_range == "auto":
                    lane_range = std
                if tuple(lane_range) == std:  # the standard split: every rank's lane count is known
                    rank_lanes = [hi - lo for lo, hi in (fdist.lane_range(n_dirs, lpd, world, k) for k in range(world))]
                lo, hi = lane_range
                if lo % lpd or hi % lpd:
                    raise ValueError("lane_range must not split antithetic pairs")
                d_lo, d_hi = lo // lpd, hi // lpd
            nd = d_hi - d_lo
            sign = np.tile(np.array([1, -1], np.int8), nd) if antithetic else np.ones(nd, np.int8)
            det = np.zeros(nd * lpd, np.int8)
            sign.setflags(write=False)
            det.setflags(write=False)
            c = self._lane_consts[ckey] = (d_lo, d_hi, sign, det, lane_range, rank_lanes)
        d_lo, d_hi, sign, det, lane_range, rank_lanes = c
        # only this rank's directions are expanded to lanes (at N = 8 one eighth of the stream)
        lidx = np.repeat(idx[d_lo:d_hi], lpd)
        return lidx, sign, det, lane_range, rank_lanes

    def evaluate(self, n_dirs, antithetic=True, seed=None, lane_range=None, out=None, novelty=False, prefetch=False,
                 timing=None):
        """n_dirs perturbation directions (x2 lanes if antithetic) -> FDBatch on the device.
        novelty=True also scores every lane against the strategy archive (FDBatch.novelty, device f64).

        lane_range=(lo, hi) evaluates only that slice of the lanes (multi-GPU sharding: every rank
        draws the full index list, in order, and keeps its contiguous share).
        prefetch=True: after launching this rollout, the NEXT call's indices are drawn ahead
        (SharedNoiseTable.peek_batch: the index stream is unchanged) and uploaded on the copy stream, so the
        next rollout does not wait for its host-to-device copy; a next call with other arguments ignores it.
        timing: (start, end) events around the rollout launch (Worker.launch)."""
        if self._host_noise:
            return self._evaluate_host(n_dirs, antithetic, seed, lane_range, out, novelty, timing)
        pre, self._next = self._next, None
        idx = self.noise_source.sample_batch(n_dirs)
        lidx, sign, det, lane_range, rank_lanes = self._lanes_of(idx, n_dirs, antithetic, lane_range)
        # the key holds the RESOLVED lane range ("auto" -> this rank's (lo, hi))
        key = (int(n_dirs), bool(antithetic), None if lane_range is None else tuple(lane_range))
        lanes_dev = None
        if pre is not None and pre[0] == key and np.array_equal(pre[1], lidx):
            lanes_dev, ev = pre[2]
            # the upload was enqueued a step ago and has normally completed: then the rollout needs no device-side
            # wait at all (a cross-stream wait costs ~10 us of barrier processing before the rollout starts, every
            # step -- rocprofv3 trace); only a copy still in flight is waited for on the compute stream
            if os.environ.get("FDR_PREFETCH_WAIT") == "always" or not ev.query():
                torch.cuda.current_stream(self.policy.flat.device).wait_event(ev)
        lpd = 2 if antithetic else 1
        lo = 0 if lane_range is None else lane_range[0]
        res, idx_d, sign_d = self.launch(lidx, sign, det, seed=seed, out=out, lane_offset=lo, lanes_dev=lanes_dev,
                                         pairs=antithetic, timing=timing)
        if prefetch and hasattr(self.noise_source, "peek_batch"):
            nidx = self.noise_source.peek_batch(n_dirs)
            nl, ns, nd, _, _ = self._lanes_of(nidx, n_dirs, antithetic, key[2])
            self._next = (key, nl, self._lanes_to_device(nl, ns, nd, defer_wait=True))
        E = getattr(self.agent.env, "envs_per_lane", 1)
        if E > 1:
            lidx, sign = np.repeat(lidx, E), np.repeat(sign, E)
        if getattr(self.agent.env, "terminates", False):   # episodes end before T: count the steps taken
            self.agent.add_timesteps(res.timesteps)
        else:
            self.agent.cumulative_timesteps += int(len(lidx)) * self.agent.env.episode_len
        nov = self.lane_novelty(idx_d, sign_d) if novelty else None
        b = FDBatch(res.reward, res.entropy, res.timesteps, res.norm2, idx_d, sign_d, lidx, sign, self.epoch,
                    lanes_per_dir=lpd * E, novelty=nov)
        b.obs_stats = obs_partials(res)
        b.rank_lanes = None if rank_lanes is None else [k * E for k in rank_lanes]
        return b

    def _evaluate_host(self, n_dirs, antithetic, seed, lane_range, out, novelty, timing):
        """evaluate() with a host noise source: every rank draws all n_dirs vectors in the source's order (the
        stream has no skip-ahead) and materialises the theta' rows of its own directions."""
        draws = [self.noise_source.sample() for _ in range(int(n_dirs))]
        lpd = 2 if antithetic else 1
        _, sign, det, lane_range, rank_lanes = self._lanes_of(np.zeros(int(n_dirs), np.int64), n_dirs, antithetic,
                                                              lane_range)
        lo = 0 if lane_range is None else lane_range[0]
        d_lo = lo // lpd
        nd = len(sign) // lpd
        noises = np.stack([draws[d_lo + d][1] for d in range(nd)]) if nd else np.zeros((0, self.policy.num_params))
        row = np.repeat(np.arange(nd, dtype=np.int64), lpd)
        res, idx_d, sign_d, rows = self._launch_host(noises, row, sign, det, lane_offset=lo, seed=seed, out=out,
                                                     timing=timing)
        lidx = rows.idx_host
        enc = [str(draws[d_lo + d][0]) if not isinstance(draws[d_lo + d][0], np.ndarray) else draws[d_lo + d][0]
               for d in range(nd) for _ in range(lpd)]
        E = getattr(self.agent.env, "envs_per_lane", 1)
        if E > 1:
            lidx, sign = np.repeat(lidx, E), np.repeat(sign, E)
            enc = [e for e in enc for _ in range(E)]
        if getattr(self.agent.env, "terminates", False):
            self.agent.add_timesteps(res.timesteps)
        else:
            self.agent.cumulative_timesteps += int(len(lidx)) * self.agent.env.episode_len
        nov = self.lane_novelty(idx_d, sign_d, table=rows.table) if novelty else None
        b = FDBatch(res.reward, res.entropy, res.timesteps, res.norm2, idx_d, sign_d, lidx, sign, self.epoch,
                    lanes_per_dir=lpd * E, novelty=nov)
        b.noise_table, b.encoded = rows.table, enc
        b.obs_stats = obs_partials(res)
        b.rank_lanes = None if rank_lanes is None else [k * E for k in rank_lanes]
        return b

    # ---- reference API ----------------------------------------------------------------------
    @torch.no_grad()
    def collect_returns(self, n=1):
        is_eval = np.array([self.rng.uniform(0, 1) < self.eval_prob for _ in range(n)])
        idx = np.zeros(n, np.int64)
        k = int((~is_eval).sum())
        sign = np.where(is_eval, 0, 1).astype(np.int8)
        host_rows, enc = None, None
        if self._host_noise:        # worker.py:27-28 per training lane: sample() in order, theta' materialised
            draws = [self.noise_source.sample() for _ in range(k)]
            row = np.cumsum(~is_eval) - 1
            noises = np.stack([d[1] for d in draws]) if k else np.zeros((0, self.policy.num_params))
            res, idx_d, sign_d, host_rows = self._launch_host(noises, np.maximum(row, 0), sign,
                                                              is_eval.astype(np.int8), jiggle=False)
            idx = host_rows.idx_host
            it = iter(draws)
            enc = ["0" if e else next(it)[0] for e in is_eval]
        else:
            if k:
                idx[~is_eval] = self.noise_source.sample_batch(k)
            res, idx_d, sign_d = self.launch(idx, sign, is_eval.astype(np.int8), jiggle=False)
        nov = self.lane_novelty(idx_d, sign_d, table=None if host_rows is None else host_rows.table)
        E = getattr(self.agent.env, "envs_per_lane", 1)
        if E > 1:
            idx, sign, is_eval = np.repeat(idx, E), np.repeat(sign, E), np.repeat(is_eval, E)
        eval_states = self.eval_states() if is_eval.any() else None
        if isinstance(eval_states, dict):   # ImpalaPolicy: the stacked obs dict -> the reference's list of dicts
            eval_states = [{k: v[i:i + 1] for k, v in eval_states.items()} for i in range(len(eval_states["frame"]))]
        b = FDBatch(res.reward, res.entropy, res.timesteps, res.norm2, idx_d, sign_d, idx, sign, self.epoch,
                    is_eval=is_eval)
        if enc is not None:
            b.encoded = [e for e in enc for _ in range(E)] if E > 1 else enc
            b.noise_table = host_rows.table
        b.novelty = None if nov is None else nov.cpu().numpy()
        b.obs_stats = obs_partials(res)
        rets = b.to_returns()
        for r in rets:
            r.reward += self.agent.rng.choice((-1e-12, 1e-12))     # agent.py:69
            self.agent.cumulative_timesteps += r.timesteps
            if r.is_eval and eval_states is not None:
                r.eval_states = list(eval_states)                   # worker.py:35 (agent.saved_states)
            if r.obs_stats_update is None or len(r.obs_stats_update) == 0:
                r.obs_stats_update = self.agent.obs_stats.serialize()
        return rets

    # ---- novelty path -----------------------------------------------------------
    def lane_novelty(self, idx_d, sign_d, table=None):
        """compute_novelty of every lane's (perturbed) policy, worker.py:53, batched on the device
        (f64 [n]); None without a strategy handler.  With E envs per lane (ImpalaPolicy / AtariPolicy)
        idx_d / sign_d repeat per env: one strategy per lane, its novelty repeated for the lane's envs."""
        h = self.strategy_handler
        if h is None:
            return None
        E = getattr(self.agent.env, "envs_per_lane", 1)
        if E > 1:
            idx_d, sign_d = idx_d[::E].contiguous(), sign_d[::E].contiguous()
        if table is None:      # the shared table; a host noise source passes its launch's rows (HostNoiseRows)
            table = self.noise_source.device_table(self.policy.flat.device)
        nov = h.lane_novelty(table, idx_d, sign_d, self.sigma, pairs=self._launch_pairs)
        return nov.repeat_interleave(E) if E > 1 else nov

    def eval_states(self, max_states=None):
        """Visited observations of the deterministic unperturbed episode (agent.py:36,58-59 with
        save_states=True).  Every eval episode of an epoch starts from reset with theta and deterministic
        actions, so one recorded lane serves all of them.
          MLP policies: raw observations, host f32 [T, n_in] (fdr_rollout_states).
          ImpalaPolicy: the obs dicts stacked (impala.py:35-45) -- {frame [n, 3, 64, 64], reward [n] (the
          reward each obs carries: that of the previous step), done [n]} device tensors, n = min(T,
          max_states) -- of env instance 0 (fdr_impala_env_frames over the recorded actions).
          AtariPolicy: frames [n, 4, 84, 84] (host f32) of env instance 0 (fdr_atari_env_frames)."""
        p = self.policy
        dev = p.flat.device
        T = self.agent.env.episode_len
        det = torch.ones(1, dtype=torch.int8, device=dev)
        bm, bv = p.bn_stats()
        if p.KIND == "impala":
            env = self.agent.env
            n = T if max_states is None else min(T, int(max_states))
            spec = engine.ImpalaSpec(p.output_shape, 1, T, entropy=False, env_seed=env.env_seed, fp16=env.fp16)
            res = engine.impala_rollout(spec, engine.lanes_desc(p.flat, 0, deterministic=det), 1, 0, jiggle=False,
                                        bn_mean=bm, bn_var=bv, record=True, device=dev)
            frames, r = engine.impala_env_frames(env.env_seed, p.output_shape, 0, 0, n, res.actions[0, :n], device=dev)
            carried = torch.cat([torch.zeros(1, dtype=torch.float32, device=dev), r[:-1]])
            return {"frame": frames, "reward": carried, "done": torch.zeros(n, dtype=torch.bool, device=dev)}
        if p.KIND == "atari":
            # the stacked-frame env's frames do not depend on the actions: env 0's first n observations
            n = T if max_states is None else min(T, int(max_states))
            return engine.atari_env_frames(self.agent.env.env_seed, 0, 0, n, device=dev).cpu().numpy()
        if p.KIND != "discrete" and p.KIND != "mujoco":
            return None
        states = torch.empty((1, T, p.input_shape), dtype=torch.float32, device=dev)
        om, osd = self.agent.obs_norm_tensors(self.fixed_obs_stats.mean, self.fixed_obs_stats.std)
        res = engine.rollout(p.spec, self.agent.env, engine.lanes_desc(p.flat, 0, deterministic=det), 1, 0,
                             jiggle=False, obs_mean=om, obs_std=osd, bn_mean=bm, bn_var=bv, device=dev, states=states)
        # a terminating env's episode visits only `steps` states (agent.py:36,58: saved_states holds visited obs);
        # the rows after the done step are never written
        steps = int(res.timesteps[0].item())
        out = states[0, :steps].cpu().numpy()
        return out if max_states is None else out[:int(max_states)]

    def update(self, state):
        # worker.py:40-43, with SURVEY finding 1 fixed: policy_params is the trainable flat vector
        params = np.asarray(state.policy_params)
        if params.size == self.policy.num_params:
            self.policy.set_trainable_flat(params)
        else:
            self.policy.deserialize(list(params))
        self.epoch = state.epoch
        if state.obs_stats is not None:
            self.fixed_obs_stats.deserialize(state.obs_stats)
