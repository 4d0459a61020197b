"""SequentialRunner -- run_sequential.py:17-213 on one MI355X.

Same constructor keywords and train(n_epochs) loop as the reference, with its three crash /
silent-NaN bugs fixed (Worker.update takes the parameter vector, noise_std is
passed by keyword, SharedNoiseTable instead of the numpy-2-broken RNGNoiseSource) and with the
per-episode host loop replaced by ONE batched rollout launch per epoch:

  1. eval coin flips (Worker.rng) until ``batch_size`` training returns are scheduled, exactly as
     run_sequential.py:134-147 consumes them; noise indices in the reference's order;
  2. one fdr_rollout over all those lanes (eval lanes: theta, deterministic actions);
  3. eval EMA / omega update on the host (run_sequential.py:137-151);
  4. FiniteDifferences.step on the device (fd weights -> gradient reduce -> DSGD);
  5. optional BN refresh (compute_vbn), report.

``antithetic=True`` evaluates +eps/-eps pairs (build extension; batch_size then counts directions).
Environments are GPU-resident (envs/): the trap env exactly, MuJoCo / CartPole ids map to the
build's synthetic fixed-length envs of the same shapes (no simulator exists on this platform).
``procgen`` ids (the reference's ImpalaPolicy route, run_sequential.py:68-71) and Atari ``NoFrameskip``
ids (BASELINE configs 4/5: the Impala conv stack on Atari-shaped frames) run ImpalaPolicy on the
synthetic frame env (``envs_per_lane`` envs per perturbation, ``fp16`` rollouts for config 5), with the
categorical-TVD novelty archive (utils/init_helper.py:9-12) and AdaptiveOmega stepped on every epoch that
had an eval episode (run_sequential.py:149-151); ``policy="atari"`` routes NoFrameskip ids to AtariPolicy
as utils/init_helper.py:13-18 does.
"""
import time

import numpy as np
import torch

from dsgd import DSGD
from fdr import engine
from envs import FrameEnv, StackedFrameEnv, SyntheticEnv, TrapEnv
from learner import FDBatch, FDState, FiniteDifferences
from policies import AtariPolicy, DiscretePolicy, ImpalaPolicy, MujocoPolicy
from strategy import StrategyHandler
from utils import AdaptiveOmega, SharedNoiseTable, math_helpers
from utils.noise_sources import RNGNoiseSource, SimpleNoiseSource
from worker import Agent, Worker


# action counts of the frame envs' namesakes (procgen: 15; gym Atari minimal action sets)
FRAME_ACTIONS = {"Pong": 6, "Breakout": 4, "SpaceInvaders": 6}


def frame_env_id(env_id):
    return "procgen" in env_id or "NoFrameskip" in env_id


def make_env(env_id, device=None, episode_len=None, env_seed=0, n_act=None, envs_per_lane=1, fp16=False,
             policy=None):
    if env_id.startswith("SimpleTrapEnv"):
        return TrapEnv(device=device)
    if frame_env_id(env_id):
        if n_act is None:
            n_act = 15 if "procgen" in env_id else next((a for k, a in FRAME_ACTIONS.items() if k in env_id), 6)
        T = 1000 if episode_len is None else episode_len
        if policy == "atari":
            return StackedFrameEnv(n_act, episode_len=T, envs_per_lane=envs_per_lane, env_seed=env_seed)
        return FrameEnv(n_act, episode_len=T, envs_per_lane=envs_per_lane, env_seed=env_seed, fp16=fp16)
    name = "cartpole" if env_id.startswith("CartPole") else "halfcheetah"
    kw = {} if episode_len is None else {"episode_len": episode_len}
    return SyntheticEnv.named(name, device=device, env_seed=env_seed, **kw)


def eval_lane_means(values, n_train, E):
    """Per-(lane, env) values of a launch -> one value per EVAL lane: the mean over its E envs (lanes past n_train
    are eval lanes, lane-major).  Deliberate divergence: the reference's single env makes one eval
    return per episode and moves the 0.9 / 0.1 EMAs and zeta once per eval return (run_sequential.py:136-143); an
    eval lane with E frame envs is that one evaluation, so its E envs are averaged first and the EMAs / zeta draw
    count do not depend on E.  E == 1 is the reference's update exactly."""
    return [np.asarray(a[n_train:], dtype=np.float64).reshape(-1, E).mean(1) for a in values]


class SequentialRunner(object):
    def __init__(self, opt_fn=DSGD, env_id="Walker2d-v2", normalize_obs=False, learning_rate=0.01,
                 noise_std=0.02, batch_size=40, ent_coef=0.0, random_seed=123, max_delayed_return=10,
                 vbn_buffer_size=0, zeta_size=200, max_strategy_history_size=200, eval_prob=0.05,
                 omega_default_value=0, omega_improvement_threshold=1.035, omega_reward_history_size=20,
                 omega_min_value=0, omega_max_value=1, omega_steps_to_min=25, omega_steps_to_max=75,
                 log_to_wandb=False, wandb_project="fd-starter", wandb_group=None, wandb_run_name=None,
                 noise_table_size=25_000_000, antithetic=False, episode_len=None, device=None, verbose=True,
                 envs_per_lane=1, fp16=False, policy=None, noise_source="table"):
        if log_to_wandb:
            raise NotImplementedError("wandb logging is not part of the MI355X engine (no network)")
        self.verbose = verbose
        self.rng = np.random.RandomState(random_seed)
        self.omega = AdaptiveOmega(default_value=omega_default_value, improvement_threshold=omega_improvement_threshold,
                                   reward_history_size=omega_reward_history_size, min_value=omega_min_value,
                                   max_value=omega_max_value, steps_to_min=omega_steps_to_min,
                                   steps_to_max=omega_steps_to_max)
        self.batch_size = batch_size
        self.zeta_size = zeta_size
        self.antithetic = antithetic
        torch.manual_seed(random_seed)
        np.random.seed(random_seed)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.env = make_env(env_id, self.device, episode_len, envs_per_lane=envs_per_lane, fp16=fp16, policy=policy)
        self.frames = isinstance(self.env, FrameEnv)
        if isinstance(self.env, StackedFrameEnv):      # utils/init_helper.py:13-18
            self.policy = AtariPolicy(self.env.obs_shape, self.env.act_dim, seed=random_seed, device=self.device)
            dist_fn = math_helpers.categorical_tvd
        elif self.frames:                              # run_sequential.py:68-71
            self.policy = ImpalaPolicy(self.env.obs_shape, self.env.act_dim, seed=random_seed, device=self.device)
            dist_fn = math_helpers.categorical_tvd
        elif self.env.discrete:
            self.policy = DiscretePolicy(self.env.obs_dim, self.env.act_dim, seed=random_seed, device=self.device)
            dist_fn = math_helpers.categorical_tvd
        else:
            self.policy = MujocoPolicy(self.env.obs_dim, self.env.act_dim, seed=random_seed, device=self.device)
            dist_fn = math_helpers.gaussian_wasserstein_dist_from_strategies   # SURVEY finding 6 fixed
        opt = opt_fn(self.policy.parameters(), lr=learning_rate)
        # noise_source: "table" (SharedNoiseTable, the GPU fast path: offsets into an HBM-resident table) or the
        # reference runner's default "rng" (run_sequential.py:89, RNGNoiseSource) / "simple": host noise sources,
        # theta' rows materialised per lane (slow, correct; utils/noise_sources.py HostNoiseRows)
        if noise_source == "table":
            self.noise_source = SharedNoiseTable(noise_table_size, self.policy.num_params, random_seed=random_seed)
        elif noise_source in ("rng", "simple"):
            cls = RNGNoiseSource if noise_source == "rng" else SimpleNoiseSource
            self.noise_source = cls(self.policy.num_params, random_seed=random_seed)
        else:
            raise ValueError("noise_source must be 'table', 'rng' or 'simple'")
        self.strategy_handler = StrategyHandler(self.policy, dist_fn, max_history_size=max_strategy_history_size,
                                                fp16=getattr(self.env, "fp16", False))
        self.agent = Agent(self.policy, self.env, random_seed, normalize_obs=normalize_obs)
        self.worker = Worker(self.policy, self.agent, self.noise_source, self.strategy_handler, sigma=noise_std,
                             random_seed=random_seed, eval_prob=eval_prob)
        self.learner = FiniteDifferences(self.policy, opt, self.omega, self.noise_source, noise_std=noise_std,
                                         batch_size=batch_size, ent_coef=ent_coef,
                                         max_delayed_return=max_delayed_return)
        self.policy_reward = 0
        self.policy_entropy = 0
        self.policy_novelty = 0
        self.zeta = np.zeros((0, self.policy.input_shape), np.float32) if not self.frames else None
        # run_server.py:94,143,196: every return's obs-stat update is merged into one global Welford
        # accumulator that the workers normalise with next epoch (device, fdr_obs_stats_merge)
        self.global_obs = None
        if normalize_obs and not self.frames:
            d = self.policy.input_shape
            self.global_obs = (torch.zeros(d, dtype=torch.float32, device=self.device),
                               torch.zeros(d, dtype=torch.float32, device=self.device),
                               torch.zeros(1, dtype=torch.int64, device=self.device))
        self.zeta_idxs = []
        self.vbn_buffer = None
        if self.frames and self.policy.KIND == "impala":
            # run_sequential.py:198-213: zeta (and the VBN buffer) are the first obs of random-action env steps
            n = max(vbn_buffer_size, zeta_size)
            obs = self._random_action_obs(n)
            self.zeta = {k: v[:zeta_size].clone() for k, v in obs.items()}
            self.zeta_idxs = list(range(len(self.zeta["frame"])))
            if vbn_buffer_size > 0:
                self.vbn_buffer = {k: v[:vbn_buffer_size] for k, v in obs.items()}
        elif self.frames:
            # AtariPolicy: the stacked-frame env's observations do not depend on the actions, so the random-action
            # steps of run_sequential.py:198-213 are env 0's first frames (host f32 [n, 4, 84, 84])
            n = max(vbn_buffer_size, zeta_size)
            obs = engine.atari_env_frames(self.env.env_seed, 0, 0, n, device=self.device).cpu().numpy()
            self.zeta = obs[:zeta_size].copy()
            self.zeta_idxs = list(range(len(self.zeta)))
            if vbn_buffer_size > 0:
                self.vbn_buffer = obs[:vbn_buffer_size]
        elif vbn_buffer_size > 0 and not self.frames:
            # run_sequential.py:198-213 samples the buffer from env steps; the GPU envs expose no host
            # stepping, so the buffer is drawn around the reset state (documented deviation)
            s0 = getattr(self.env, "s0_host", np.zeros(self.env.obs_dim, np.float32))
            self.vbn_buffer = (s0 + 0.1 * self.rng.randn(vbn_buffer_size, self.env.obs_dim)).astype(np.float32)
        self.current_state = FDState()
        self.current_state.policy_params = self.policy.get_trainable_flat()
        self.current_state.epoch = 0
        self.history = []

    def _random_action_obs(self, n):
        """The first n obs of env instance 0 under uniformly random actions (env.action_space.sample() in
        run_sequential.py:207; here self.rng), stacked {frame, reward, done}; the env resets every T steps."""
        env = self.env
        A, T = env.act_dim, env.episode_len
        fr, rw = [], []
        for t0 in range(0, n, T):
            k = min(T, n - t0)
            acts = torch.as_tensor(self.rng.randint(0, A, size=k).astype(np.int32), device=self.device)
            f, r = engine.impala_env_frames(env.env_seed, A, 0, 0, k, acts, device=self.device)
            fr.append(f)
            rw.append(torch.cat([torch.zeros(1, dtype=torch.float32, device=self.device), r[:-1]]))
        return {"frame": torch.cat(fr), "reward": torch.cat(rw), "done": torch.zeros(n, dtype=torch.bool,
                                                                                       device=self.device)}

    def _update_zeta(self, eval_states):
        """run_sequential.py:142-143: shuffled slots of the probe set zeta take an eval episode's states.
        The reference starts from zeta = [] (so the fancy-index assignment raises); here the first eval
        episode seeds zeta with its first zeta_size states.  ImpalaPolicy: zeta and the eval states are
        stacked obs dicts of device tensors, seeded from random-action steps as the reference's
        _sample_initial_buffers (run_sequential.py:198-213)."""
        if eval_states is None or len(eval_states) == 0:
            return
        if isinstance(eval_states, dict):
            self.rng.shuffle(self.zeta_idxs)
            k = min(len(eval_states["frame"]), self.zeta_size, len(self.zeta_idxs))
            slots = torch.as_tensor(np.asarray(self.zeta_idxs[:k], np.int64), device=self.device)
            for key in self.zeta:
                self.zeta[key][slots] = eval_states[key][:k].to(self.zeta[key].dtype)
            return
        if len(self.zeta) == 0:
            self.zeta = np.array(eval_states[:self.zeta_size], np.float32)
            self.zeta_idxs = list(range(len(self.zeta)))
            return
        self.rng.shuffle(self.zeta_idxs)
        new = np.asarray(eval_states[:self.zeta_size], np.float32)
        self.zeta[self.zeta_idxs[:len(new)]] = new[:len(self.zeta_idxs)]

    def _schedule(self):
        """Eval coins in the reference's order until batch_size training returns (run_sequential.py:134)."""
        evals = []
        n_train = 0
        while n_train < self.batch_size:
            e = self.worker.rng.uniform(0, 1) < self.worker.eval_prob
            evals.append(e)
            n_train += 0 if e else 1
        return np.array(evals)

    @torch.no_grad()
    def train(self, n_epochs):
        self.strategy_handler.add_policy(self.policy)
        self.worker.update(self.current_state)
        E = getattr(self.env, "envs_per_lane", 1)
        if self.frames and self.zeta is not None:
            self.strategy_handler.set_zeta(self.zeta)
        for _ in range(n_epochs):
            t1 = time.perf_counter()
            is_eval = self._schedule()
            n_dirs = int((~is_eval).sum())
            lpd = 2 if self.antithetic else 1
            sign = np.concatenate([np.tile(np.array([1, -1], np.int8), n_dirs) if self.antithetic
                                   else np.ones(n_dirs, np.int8), np.zeros(int(is_eval.sum()), np.int8)])
            det = (sign == 0).astype(np.int8)
            rows = None
            if self.worker._host_noise:      # worker.py:27-28: one sample() per direction, theta' rows materialised
                draws = [self.noise_source.sample() for _ in range(n_dirs)]
                idx_dirs = [d[0] for d in draws]
                noises = np.stack([d[1] for d in draws]) if n_dirs else np.zeros((0, self.policy.num_params))
                row = np.concatenate([np.repeat(np.arange(n_dirs), lpd), np.zeros(int(is_eval.sum()), np.int64)])
                res, idx_d, sign_d, rows = self.worker._launch_host(noises, row, sign, det, jiggle=False)
                lidx = rows.idx_host
            else:
                idx_dirs = self.noise_source.sample_batch(n_dirs)
                # lane layout: training lanes first (lanes of a direction contiguous), eval lanes last
                lidx = np.concatenate([np.repeat(idx_dirs, lpd), np.zeros(int(is_eval.sum()), np.int64)])
                res, idx_d, sign_d = self.worker.launch(lidx, sign, det, jiggle=False)
            # E envs per lane (frame envs): one return per (lane, env), lane-major; idx_d / sign_d repeat per env
            lidx, sign = np.repeat(lidx, E), np.repeat(sign, E)
            if self.global_obs is not None and getattr(res, "obs_mean", None) is not None:
                engine.obs_stats_merge(res.obs_mean, res.obs_m2, res.obs_count, *self.global_obs)
            nov = self.worker.lane_novelty(idx_d, sign_d, table=None if rows is None else rows.table)  # worker.py:53
            nov = np.zeros(len(lidx)) if nov is None else nov.cpu().numpy()
            rew = res.reward.cpu().numpy() + np.array([self.agent.rng.choice((-1e-12, 1e-12)) for _ in lidx])
            ent = res.entropy.cpu().numpy()
            steps = int(res.timesteps.sum().item())
            self.agent.cumulative_timesteps += steps
            n_train = n_dirs * lpd * E
            eval_states = self.worker.eval_states(self.zeta_size) if is_eval.any() else None
            # run_sequential.py:142-151 runs once per eval EPISODE of the reference's single env; an eval lane with
            # E envs is one such evaluation, so its E returns are averaged and the EMAs / zeta move once per lane
            # (per-env updates would make the 0.9 time constants and the zeta churn depend on E)
            for r, e, nv in zip(*eval_lane_means((rew, ent, nov), n_train, E)):
                self.policy_reward = self.policy_reward * 0.9 + r * 0.1
                self.policy_entropy = self.policy_entropy * 0.9 + e * 0.1
                self.policy_novelty = self.policy_novelty * 0.9 + nv * 0.1
                self._update_zeta(eval_states)
            if is_eval.any():
                self.strategy_handler.set_zeta(self.zeta)
                self.omega.step(float(np.mean(rew[:n_train])))
            dev = self.policy.flat.device
            batch = FDBatch(torch.as_tensor(rew[:n_train], device=dev), res.entropy[:n_train],
                            res.timesteps[:n_train], res.norm2[:n_train], idx_d[:n_train], sign_d[:n_train],
                            lidx[:n_train], sign[:n_train], self.learner.epoch, lanes_per_dir=lpd * E)
            if rows is not None:
                batch.noise_table = rows.table
            update_magnitude = self.learner.step(batch, self.policy_reward, self.policy_novelty, self.policy_entropy)
            if self.vbn_buffer is not None:
                self.policy.compute_vbn(self.vbn_buffer)
            if update_magnitude > 0:
                self.strategy_handler.add_policy(self.policy)                   # run_sequential.py:160
                self.current_state.strategy_frames = self.zeta
                self.current_state.strategy_history = self.strategy_handler.strategy_tensor
                self.current_state.policy_params = self.policy.get_trainable_flat()
                if self.global_obs is not None:
                    m, v, c = (t.cpu().numpy() for t in self.global_obs)
                    self.current_state.obs_stats = m.tolist() + v.tolist() + [int(c[0])]
                self.current_state.epoch = self.learner.epoch
                self.worker.update(self.current_state)
                report = {"Epoch": self.learner.epoch,
                          "Epoch Time": time.perf_counter() - t1,
                          "Cumulative Timesteps": self.agent.cumulative_timesteps,
                          "Policy Reward": self.policy_reward,
                          "Policy Entropy": self.policy_entropy,
                          "Policy Novelty": self.policy_novelty,
                          "Noisy Reward": float(np.mean(rew[:n_train])),
                          "Noisy Novelty": float(np.mean(nov[:n_train])),
                          "Update Magnitude": update_magnitude,
                          "Omega": self.omega.omega}
                self.history.append(dict(report, idx=idx_dirs, rewards=rew[:n_train]))
                self._report_epoch(report)

    def _report_epoch(self, report):
        if not self.verbose:
            return
        print("\n***********Begin Epoch Report***********")
        for k, v in report.items():
            print("{} {:7.4f}".format(k, v) if isinstance(v, (float, np.floating)) else "{} {}".format(k, v))
        print("***********End Epoch Report***********")
