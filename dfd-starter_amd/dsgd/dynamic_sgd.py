"""DSGD -- dsgd/dynamic_sgd.py:7-51: normalised-gradient SGD with an omega-scaled learning rate.

    theta <- theta - lr * sqrt(d) * lr_scale * grad / ||grad||,
    lr_scale = affine(omega, [omega_min, omega_max] -> [min_scale, max_scale])

``step()`` keeps the torch.optim API (gradients in p.grad).  When the parameters are the views of
a Policy's flat device buffer the update is the fused fdr_dsgd_step kernel; the learner calls that
kernel directly with its f64 gradient (no p.grad round trip).
"""
import numpy as np
import torch
from torch.optim import Optimizer

from fdr import engine
from utils import math_helpers


class DSGD(Optimizer):
    def __init__(self, params, lr, min_scale=0.23, max_scale=1.0):
        super().__init__(params, {"lr": lr})
        self.lr = lr
        self.min_scale = min_scale
        self.max_scale = max_scale
        self.lr_scale = 1
        self.steps = 0
        d = sum(p.numel() for g in self.param_groups for p in g["params"])
        self.coef = np.sqrt(d)

    def _flat_view(self):
        """The single contiguous buffer the params view, if they tile one (Policy.flat)."""
        ps = [p for g in self.param_groups for p in g["params"]]
        base = ps[0].data
        if not base.is_cuda:
            return None
        start = base.data_ptr()
        off = 0
        for p in ps:
            if p.data.data_ptr() != start + 4 * off or not p.data.is_contiguous():
                return None
            off += p.numel()
        return torch.as_strided(base, (off,), (1,))

    @torch.no_grad()
    def step(self, closure=None):
        ps = [p for g in self.param_groups for p in g["params"] if p.grad is not None]
        flat_grad = torch.cat([p.grad.reshape(-1) for p in ps])
        flat = self._flat_view()
        if flat is not None and len(ps) == sum(len(g["params"]) for g in self.param_groups):
            out = engine.dsgd_step(flat, -flat_grad.double(), self.lr, self.lr_scale)
            assert out[1].item() > 0, "DSGD ENCOUNTERED GRADIENT WITH NORM OF ZERO"
        else:   # foreign (non-policy) parameters: same update with torch ops
            norm = flat_grad.norm().item()
            assert norm > 0, "DSGD ENCOUNTERED GRADIENT WITH NORM OF ZERO"
            coef = self.lr * self.coef * self.lr_scale / norm
            idx = 0
            for p in ps:
                n = p.numel()
                p.sub_(coef * flat_grad[idx:idx + n].view_as(p))
                idx += n
        self.steps += 1

    def adjust_lr(self, omega):
        self.lr_scale = math_helpers.affine_transform(omega.omega, omega.min_omega, omega.max_omega,
                                                      self.min_scale, self.max_scale)
