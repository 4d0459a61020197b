"""SequentialRunner.train restated (bug-fixed harness form) -- trap env, injected action noise.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows run_sequential.py:113-179 with the three harness fixes of SURVEY.md section 8c
(Worker.update takes the parameter vector, learner.noise_std = noise_std, SharedNoiseTable
instead of the numpy-2-broken RNGNoiseSource).  RNG streams, in the reference's order:
  * torch.manual_seed / np.random.seed (run_sequential.py:64-66) -> policy default init + normc
  * Worker.rng = RandomState(seed): one uniform per collect_returns call, eval if < eval_prob
    (worker/worker.py:15,23)
  * Agent.rng  = RandomState(seed): one choice((-1e-12, 1e-12)) per episode (worker/agent.py:9,69)
  * noise table RandomState(seed): table then indices (utils/noise_sources.py:39-47)
  * injected action uniforms: one per non-deterministic step, in order
  * initial zeta sampling steps the env ``zeta_size`` times with random actions AFTER the Agent
    captured its reset observation (run_sequential.py:92-103,198-213) -- reproduced.
Novelty / strategy archive is computed by the reference but unused by the objective
(learner/finite_differences.py:48), so it is not restated.
"""
import numpy as np
import torch

from .agent import collect_return
from .envs import TrapEnv
from .learner import FDLearner
from .noise import NoiseTable
from .policies import TorchPolicy


class _AdaptiveOmega(object):
    """utils/adaptive_omega.py:5-53."""

    def __init__(self, default_value=0, improvement_threshold=1.035, reward_history_size=20,
                 min_value=0, max_value=1, steps_to_min=25, steps_to_max=75):
        self.omega = default_value
        self.improvement_threshold = improvement_threshold
        self.size = reward_history_size
        self.min_omega, self.max_omega = min_value, max_value
        self.increase, self.decrease = 1 / steps_to_max, 1 / steps_to_min
        self.history = []

    def step(self, reward):
        if reward is None:
            return
        self.history.append(reward)
        if len(self.history) > self.size:
            self.history.pop(0)
        mean = round(float(np.mean(self.history)), 5)
        reward = round(reward, 5)
        mean = mean / self.improvement_threshold if mean < 0 else mean * self.improvement_threshold
        if reward > mean:
            self.omega = max(self.omega - self.decrease, self.min_omega)
        else:
            self.omega = min(self.omega + self.increase, self.max_omega)


def run_trap(n_epochs, batch_size=16, seed=124, noise_std=0.02, lr=0.01, eval_prob=0.05,
             zeta_size=4, action_seed=777, table_size=2 ** 22):
    torch.manual_seed(seed)
    np.random.seed(seed)
    omega = _AdaptiveOmega()
    env = TrapEnv()
    policy = TorchPolicy("discrete", 2, 9, seed=seed)
    P = policy.num_params
    table = NoiseTable(table_size, P, seed)
    agent_rng = np.random.RandomState(seed)
    worker_rng = np.random.RandomState(seed)
    action_rng = np.random.RandomState(action_seed)
    last_obs = env.reset()                                   # Agent.__init__ (agent.py:10)
    space_rng = np.random.RandomState(seed)                  # action_space.seed(seed)
    for _ in range(zeta_size):                               # _sample_initial_buffers
        _, _, done, _ = env.step(int(space_rng.randint(9)))
        if done:
            env.reset()
    learner = FDLearner(policy.get_flat(), table.table, P, noise_std, lr)
    policy_reward, cum_steps, log = 0.0, 0, []

    def noise_fn(t):
        return np.float32(action_rng.uniform())

    for _ in range(n_epochs):
        theta = learner.theta
        rets, any_eval = [], False
        while len(rets) < batch_size:
            is_eval = worker_rng.uniform(0, 1) < eval_prob
            if not is_eval:
                idx = int(table.sample_indices(1)[0])
                policy.set_flat(theta + np.float32(noise_std) * table.decode(idx))
            else:
                idx = 0
                policy.set_flat(theta)
            r, e, steps, last_obs = collect_return(
                policy, env, last_obs, is_eval, noise_fn,
                lambda: agent_rng.choice((-1e-12, 1e-12)))
            policy.set_flat(theta)
            cum_steps += steps
            if is_eval:
                any_eval = True
                policy_reward = policy_reward * 0.9 + r * 0.1
            else:
                rets.append((learner.epoch, idx, r))
        rewards = [r for _, _, r in rets]
        if any_eval:
            omega.step(np.mean(rewards))
        upd, _ = learner.step([e for e, _, _ in rets], [i for _, i, _ in rets], [1] * len(rets), rewards,
                              policy_reward, omega.omega, omega.min_omega, omega.max_omega)
        log.append(dict(rewards=np.array(rewards), idx=np.array([i for _, i, _ in rets]),
                        policy_reward=policy_reward, update=upd))
    return dict(theta=learner.theta, log=log, cum_steps=cum_steps, policy_reward=policy_reward)
