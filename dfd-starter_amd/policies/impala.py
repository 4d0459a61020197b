"""ImpalaPolicy -- policies/impala.py:8-186 on the HIP Impala kernels (fdr_impala_*).

Same API as the reference: ``forward(obs)`` / ``get_action`` / ``get_entropy`` / ``get_strategy`` /
``reset`` / ``compute_vbn`` and the flat-parameter methods of Policy.  ``obs`` is the reference's
ImpalaEnvWrapper dict (utils/impala_env_wrapper.py:25-28): frame [B, T, 3, 64, 64] (0..255),
reward [B, T], done [B, T]; a list of such dicts is the stacked form get_entropy takes.

* theta lives in ``self.flat`` (HBM), in the reference's parameters() order (feat_convs, resnet1,
  resnet2, fc, core, policy -- impala.py:60-119); the module below is its parameter container and
  is initialised with torch's default init, like the reference (ImpalaPolicy has no normc layer).
* the LSTM state ``self.state`` = (h, c) device tensors [B, 256]; ``reset`` zeroes it (impala.py:29-30).
* Deviation, documented in DESIGN.md: with B > 1 the reference masks every env's state with env 0's
  done flag (its zip over ``notdone.unbind()`` iterates the batch dim); here each env uses its own.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Categorical

from fdr import engine
from .policy import Policy

STAGES = (16, 32, 32)


def _res_block(c):
    return nn.Sequential(nn.BatchNorm2d(c), nn.ReLU(), nn.Conv2d(c, c, 3, 1, 1),
                         nn.BatchNorm2d(c), nn.ReLU(), nn.Conv2d(c, c, 3, 1, 1))


class ImpalaNet(nn.Module):
    """Parameter container with the reference ImpalaCNN's registration order (impala.py:48-123)."""

    def __init__(self, n_act):
        super().__init__()
        feats, r1, r2 = [], [], []
        cin = 3
        for c in STAGES:
            feats.append(nn.Sequential(nn.BatchNorm2d(cin), nn.Conv2d(cin, c, 3, 1, 1),
                                       nn.MaxPool2d(3, 2, 1)))
            r1.append(_res_block(c))
            r2.append(_res_block(c))
            cin = c
        self.feat_convs, self.resnet1, self.resnet2 = nn.ModuleList(feats), nn.ModuleList(r1), nn.ModuleList(r2)
        self.fc = nn.Sequential(nn.BatchNorm1d(2048), nn.Linear(2048, 256))
        self.core = nn.LSTM(257, 256, num_layers=1, batch_first=True)
        self.policy = nn.Sequential(nn.BatchNorm1d(256), nn.Linear(256, n_act))

    def bn_layers(self):
        return [m for m in self.modules() if isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d))]


class ImpalaPolicy(Policy):
    KIND = "impala"

    def __init__(self, n_inputs, n_actions, seed=124, device=None):
        super().__init__(n_inputs, n_actions, seed=seed, device=device)
        self.model = ImpalaNet(self.output_shape)
        self._finalize()
        self.spec = engine.ImpalaSpec(self.output_shape)
        assert self.spec.n_params == self.num_params, (self.spec.n_params, self.num_params)
        self.state = None
        self.reset()

    def _init_params(self):
        pass  # impala.py: the Sequential(ImpalaCNN, Softmax) has no .weight, so normc does nothing

    def reset(self, batch_size=1):
        dev = self.flat.device
        self.state = (torch.zeros(batch_size, 256, device=dev), torch.zeros(batch_size, 256, device=dev))

    @staticmethod
    def _stack(x):
        """dict or list of dicts (impala.py:35-45) -> frames [N,3,64,64], reward [N], done [N]."""
        if isinstance(x, dict):
            x = [x]
        fr = torch.cat([torch.as_tensor(o["frame"], dtype=torch.float32).reshape(-1, 3, 64, 64) for o in x])
        rw = torch.cat([torch.as_tensor(o["reward"], dtype=torch.float32).reshape(-1) for o in x])
        dn = torch.cat([torch.as_tensor(o["done"]).reshape(-1).bool() for o in x])
        return fr, rw, dn

    @torch.no_grad()
    def _step(self, frames, reward, done):
        dev = self.flat.device
        n = frames.shape[0]
        if self.state[0].shape[0] != n:
            self.state = tuple(s[:1].expand(n, 256).contiguous() for s in self.state)
        bm, bv = self.bn_stats()
        notdone = (~done).float().to(dev)
        return engine.impala_forward(self.spec, self.flat, frames.to(dev), self.state[0], self.state[1],
                                     reward=reward.to(dev), notdone=notdone, bn_mean=bm, bn_var=bv)

    def forward(self, x):
        """impala.py:18-19 + Softmax: probs [T=1, B, A] for one obs dict (B envs)."""
        fr, rw, dn = self._stack(x)
        return self._step(fr, rw, dn).view(1, -1, self.output_shape)

    @torch.no_grad()
    def get_action(self, x, deterministic=False):
        probs = self.forward(x)
        if deterministic:
            return int(probs.argmax().item())                            # discrete.py:18-19
        return int(Categorical(probs=probs.cpu()).sample().item())      # discrete.py:21-24

    @torch.no_grad()
    def _sequence(self, x):
        """The reference's stacked obs (impala.py:35-45: B = n, T = 1) through ImpalaCNN.forward: the
        batch_first LSTM reads them as ONE sequence of length n (B = 1) from self.state, and only the first
        obs' done flag masks the incoming state (the zip over notdone.unbind() yields one pair,
        impala.py:165-176).  self.state becomes the end-of-sequence state (impala.py:184).  -> probs [n, A]."""
        fr, rw, dn = self._stack(list(x) if not isinstance(x, dict) else x)
        dev = self.flat.device
        h, c = (s[:1].reshape(1, 256).clone().contiguous() for s in self.state)
        if bool(dn[0]):
            h.zero_()
            c.zero_()
        bm, bv = self.bn_stats()
        probs = engine.impala_strategies(self.spec, engine.lanes_desc(self.flat, 0), 1, fr.to(dev), rw.to(dev),
                                         h, c, bm, bv)
        self.state = (h, c)
        return probs[0]

    @torch.no_grad()
    def get_entropy(self, x):
        """impala.py:21-22 -> discrete.py:26-29: mean Categorical entropy of the stacked obs' sequence."""
        return Categorical(probs=self._sequence(x)).entropy().mean().item()

    @torch.no_grad()
    def get_strategy(self, x):
        """impala.py:24-27: the probabilities of the stacked obs' sequence, [n, A] (host)."""
        return self._sequence(x).cpu().numpy()

    @torch.no_grad()
    def compute_vbn(self, buffer):
        """impala.py:12-16 on the device (fdr_impala_bn_refresh): the stacked buffer (B = n, T = 1) in train mode --
        every BatchNorm normalises with its batch statistics and folds them into its running stats (updated in
        place: they are views of the flat stat buffers), and the batch_first LSTM reads the n obs as ONE sequence
        from self.state, zeroed iff the first obs is done (impala.py:165-176); self.state becomes the sequence's
        end state (impala.py:184)."""
        fr, rw, dn = self._stack(list(buffer) if not isinstance(buffer, dict) else buffer)
        dev = self.flat.device
        h, c = (s[:1].reshape(256).clone().contiguous() for s in self.state)
        bns = self._bn_layers
        bm, bv = self.bn_stats()
        engine.impala_bn_refresh(self.spec, self.flat, fr.to(dev), bm, bv, reward=rw.to(dev), first_done=bool(dn[0]),
                                 h=h, c=c, momentum=bns[0].momentum)
        if not self._bn_views_intact(bns):   # a user replaced a buffer: write the refreshed stats back
            off = 0
            for m in bns:
                k = m.num_features
                m.running_mean.copy_(bm[off:off + k])
                m.running_var.copy_(bv[off:off + k])
                off += k
        for m in bns:
            m.num_batches_tracked += 1
        self.state = (h.view(1, 256), c.view(1, 256))
