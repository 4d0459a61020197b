"""MujocoPolicy -- policies/mujoco.py:8-41 on the HIP policy kernel."""
import numpy as np
import torch
import torch.nn as nn
from torch.distributions import Normal

from .policy import Policy


class MapContinuousToAction(nn.Module):
    """utils/torch_helpers.py:15-25: tanh, mean = first half, std = 0.55 + 0.45 * second half."""

    def __init__(self):
        super().__init__()
        self.tanh = nn.Tanh()

    def forward(self, x):
        x = self.tanh(x)
        n = x.shape[-1] // 2
        return x[..., :n], 0.55 + 0.45 * x[..., n:]


class MujocoPolicy(Policy):
    KIND = "mujoco"

    def __init__(self, n_inputs, n_actions, seed=124, device=None):
        super().__init__(n_inputs, n_actions, seed=seed, device=device)
        self._build_model()
        self._finalize()

    @torch.no_grad()
    def get_action(self, x, deterministic=False):
        mean, std = self.forward(x)
        if deterministic:
            return mean.flatten().tolist()                             # mujoco.py:17-18
        return Normal(mean.cpu(), std.cpu()).sample().flatten().tolist()  # mujoco.py:20-22

    @torch.no_grad()
    def get_entropy(self, x):
        mean, std = self.forward(np.asarray(x))
        return Normal(mean, std).entropy().sum(dim=-1).mean().item()    # mujoco.py:24-26

    @torch.no_grad()
    def get_strategy(self, x):
        mean, std = self.forward(np.asarray(x))
        return torch.cat([mean, std], dim=-1).cpu().numpy()             # mujoco.py:29-30

    def _build_model(self):
        h1 = h2 = 64                                                    # mujoco.py:32-41
        self.model = nn.Sequential(
            nn.Linear(self.input_shape, h1), nn.Tanh(),
            nn.Linear(h1, h2), nn.Tanh(),
            nn.Linear(h2, self.output_shape * 2), MapContinuousToAction())
