"""utils/adaptive_omega.py:5-53 -- scalar novelty-weight controller (host, O(1) per epoch)."""
import numpy as np


class AdaptiveOmega(object):
    def __init__(self, default_value=0, improvement_threshold=1.025, reward_history_size=10,
                 min_value=0, max_value=1, steps_to_min=15, steps_to_max=200):
        self.omega = default_value
        self.improvement_threshold = improvement_threshold
        self.reward_history_size = reward_history_size
        self.min_omega, self.max_omega = min_value, max_value
        self.reward_history = []
        self.steps_to_max, self.steps_to_min = steps_to_max, steps_to_min
        self.increase, self.decrease = 1 / steps_to_max, 1 / steps_to_min

    def step(self, theta_reward):
        if theta_reward is None:
            return
        self.reward_history.append(theta_reward)
        if len(self.reward_history) > self.reward_history_size:
            self.reward_history.pop(0)
        self.adapt_omega(theta_reward)

    def adapt_omega(self, theta_reward):
        if not self.reward_history:
            return
        mean = round(float(np.mean(self.reward_history)), 5)
        theta_reward = round(theta_reward, 5)
        mean = mean / self.improvement_threshold if mean < 0 else mean * self.improvement_threshold
        if theta_reward > mean:
            self.omega = max(self.omega - self.decrease, self.min_omega)
        else:
            self.omega = min(self.omega + self.increase, self.max_omega)
