"""AtariPolicy -- policies/atari.py:7-51 on the HIP AtariPolicy kernels (fdr_atari_*).

Same API as the reference (get_action / get_entropy / get_strategy / compute_vbn + the Policy flat
methods).  theta lives in ``self.flat`` in parameters() order; normc initialisation touches every
layer with a weight (both convs, both BatchNorm2d, the BatchNorm1d and both linears), bit-exact with
the reference.  Observations are [4, 84, 84] stacks (raw pixel values, as the reference feeds them).
Deviation: the reference's Policy.forward views non-tensor input with a tuple input_shape
(policies/policy.py:27-28), which torch rejects; here any array-like of 4*84*84 values per frame works.
"""
import numpy as np
import torch
import torch.nn as nn
from torch.distributions import Categorical

from fdr import engine
from .policy import Policy


class AtariPolicy(Policy):
    KIND = "atari"

    def __init__(self, n_inputs, n_actions, seed=124, device=None):
        super().__init__(n_inputs, n_actions, seed=seed, device=device)
        self.input_shape = (4, int(n_inputs[0]), int(n_inputs[1]))      # atari.py:11-12
        if self.input_shape[1:] != (84, 84):
            raise ValueError("AtariPolicy's Linear(2592, .) fixes 84 x 84 frames (policies/atari.py:47)")
        self.model = nn.Sequential(
            nn.Conv2d(4, 16, kernel_size=[8, 8], stride=[4, 4]), nn.BatchNorm2d(16), nn.ReLU(),
            nn.Conv2d(16, 32, kernel_size=[4, 4], stride=[2, 2]), nn.BatchNorm2d(32), nn.ReLU(),
            nn.Flatten(), nn.Linear(2592, 256), nn.BatchNorm1d(256), nn.ReLU(),
            nn.Linear(256, self.output_shape), nn.Softmax(dim=-1))
        self._finalize()
        self.spec = engine.AtariSpec(self.output_shape)
        assert self.spec.n_params == self.num_params

    def bn_stats(self):
        bns = [m for m in self.model if isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d))]
        return (torch.cat([m.running_mean for m in bns]).float().contiguous(),
                torch.cat([m.running_var for m in bns]).float().contiguous())

    @torch.no_grad()
    def forward(self, x):
        fr = torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x, dtype=torch.float32)
        bm, bv = self.bn_stats()
        return engine.atari_forward(self.spec, self.flat, fr.reshape(-1, 4 * 84 * 84).to(self.flat.device),
                                    bn_mean=bm, bn_var=bv)

    @torch.no_grad()
    def get_action(self, x, deterministic=False):
        probs = self.forward(x)
        if deterministic:
            return int(probs.argmax().item())                            # atari.py:17-20
        return int(Categorical(probs=probs.cpu()).sample().item())      # atari.py:22-24

    @torch.no_grad()
    def get_entropy(self, x):
        return Categorical(probs=self.forward(x)).entropy().mean().item()   # atari.py:25-28

    @torch.no_grad()
    def get_strategy(self, x):
        return self.forward(x).cpu().numpy()                             # atari.py:30-31

    @torch.no_grad()
    def compute_vbn(self, buffer):
        """policy.py:31-34 on the device (fdr_atari_bn_refresh): one train-mode pass of the buffer -- each BN
        normalises with its batch statistics and folds them into its running stats; the policy stays in eval mode."""
        x = torch.as_tensor(np.asarray(buffer) if not torch.is_tensor(buffer) else buffer, dtype=torch.float32)
        x = x.reshape(-1, 4 * 84 * 84).to(self.flat.device)
        bns = [m for m in self.model if isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d))]
        bm, bv = self.bn_stats()
        engine.atari_bn_refresh(self.spec, self.flat, x, bm, bv, momentum=bns[0].momentum)
        off = 0
        for m in bns:
            k = m.num_features
            m.running_mean.copy_(bm[off:off + k])
            m.running_var.copy_(bv[off:off + k])
            m.num_batches_tracked += 1
            off += k
        self.eval()
