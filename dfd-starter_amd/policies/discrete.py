"""DiscretePolicy -- policies/discrete.py:8-48 on the HIP policy kernel."""
import numpy as np
import torch
import torch.nn as nn
from torch.distributions import Categorical

from fdr import engine
from .policy import Policy


class DiscretePolicy(Policy):
    KIND = "discrete"

    def __init__(self, n_inputs, n_actions, seed=124, device=None):
        super().__init__(n_inputs, n_actions, seed=seed, device=device)
        self._build_model()
        self._finalize()

    @torch.no_grad()
    def get_action(self, x, deterministic=False):
        probs = self.forward(x)
        if deterministic:
            return int(probs[0].argmax().item())                        # discrete.py:18-19
        return int(Categorical(probs=probs[0].cpu()).sample().item())   # discrete.py:21-24

    @torch.no_grad()
    def get_entropy(self, x):
        probs = self.forward(np.asarray(x))
        return Categorical(probs=probs).entropy().mean().item()         # discrete.py:26-29

    @torch.no_grad()
    def get_strategy(self, x):
        return self.forward(np.asarray(x)).cpu().numpy()                # discrete.py:31-32

    @torch.no_grad()
    def compute_vbn(self, buffer):
        """policies/policy.py:31-34 on the device: fdr_bn_refresh runs the train-mode pass (batch-stat
        normalisation + running-stat update of the 3 BatchNorm1d) -- no torch compute."""
        x = torch.as_tensor(np.asarray(buffer), dtype=torch.float32).reshape(-1, self.input_shape)
        bns = [m for m in self.model if isinstance(m, nn.BatchNorm1d)]
        bm, bv = self.bn_stats()
        engine.bn_refresh(self.spec, self.flat, x.to(self.flat.device), bm, bv, momentum=bns[0].momentum)
        off = 0
        for m in bns:
            n = m.num_features
            if m.running_mean.data_ptr() != bm[off:off + n].data_ptr():   # (no-op when they alias, Policy._bn_flat)
                m.running_mean.copy_(bm[off:off + n])
                m.running_var.copy_(bv[off:off + n])
            m.num_batches_tracked += 1
            off += n

    def _build_model(self):
        h1 = h2 = 64                                                    # discrete.py:34-48
        self.model = nn.Sequential(
            nn.BatchNorm1d(self.input_shape), nn.Linear(self.input_shape, h1), nn.ReLU(),
            nn.BatchNorm1d(h1), nn.Linear(h1, h2), nn.ReLU(),
            nn.BatchNorm1d(h2), nn.Linear(h2, self.output_shape), nn.Softmax(dim=-1))
