"""FDReturn record (learner/fd_return.py:5-56) and FDBatch, its struct-of-arrays device form.

The hot path never builds per-return Python objects: ``Worker.evaluate`` returns an FDBatch whose
fields are device tensors written by the rollout kernel, and ``FiniteDifferences.step`` consumes
it directly.  ``FDBatch.to_returns()`` / ``FDBatch.from_returns()`` adapt to the reference's
list-of-FDReturn API.
"""
import numpy as np
import torch


class FDReturn(object):
    def __init__(self):
        self.epoch = -1
        self.encoded_noise = "-1"
        self.perturbation = None
        self.reward = 0
        self.novelty = 0
        self.entropy = 0
        self.timesteps = 0
        self.is_eval = False
        self.eval_states = []
        self.obs_stats_update = []
        self.sign = 1          # build extension: -1 for the antithetic partner
        self.norm2 = None      # build extension: ||lambda||^2 from the rollout kernel

    def serialize(self):
        return (self.reward, self.novelty, self.entropy, self.timesteps, self.encoded_noise, self.perturbation,
                self.epoch, self.is_eval, self.eval_states, self.obs_stats_update)

    def deserialize(self, other):
        (self.reward, self.novelty, self.entropy, self.timesteps, self.encoded_noise, self.perturbation,
         self.epoch, self.is_eval, self.eval_states, self.obs_stats_update) = other


class FDBatch(object):
    """One batched evaluation.  Lanes of one direction are contiguous (lanes_per_dir = 2 when
    antithetic: +eps then -eps).  All tensors live on ``device``; ``idx_host`` mirrors idx.

    ``idx`` / ``sign`` of a Worker.evaluate batch are views of the Worker's upload ring (64 slots per lane count):
    a batch kept past the next 63 uploads of its shape stays valid -- the ring then hands the block to the
    allocator with the compute stream recorded on it (Worker._lanes_to_device) -- so the views never alias a
    newer upload."""

    def __init__(self, reward, entropy, timesteps, norm2, idx, sign, idx_host, sign_host, epoch,
                 lanes_per_dir=1, is_eval=None, novelty=None):
        self.reward, self.entropy, self.timesteps, self.norm2 = reward, entropy, timesteps, norm2
        self.idx, self.sign = idx, sign
        self.idx_host, self.sign_host = np.asarray(idx_host), np.asarray(sign_host)
        self.epoch = epoch
        self.lanes_per_dir = lanes_per_dir
        self.is_eval = np.zeros(len(self.sign_host), bool) if is_eval is None else np.asarray(is_eval)
        self.novelty = novelty
        self.obs_stats = None   # (mean [n, d], m2 [n, d], count [n]) device Welford partials, or None
        self.noise_table = None  # host noise sources: the batch's fl32(noise) rows (idx = row offsets into them)
        self.encoded = None      # host noise sources: each lane's encoded perturbation

    def __len__(self):
        return len(self.sign_host)

    @property
    def n_dirs(self):
        return len(self) // self.lanes_per_dir

    def dir_idx(self):
        """Device int64 [n_dirs]: table offset of each direction."""
        if self.lanes_per_dir == 1:
            return self.idx
        return self.idx[::self.lanes_per_dir].contiguous()

    def to_returns(self):
        rew = self.reward.double().cpu().numpy()
        ent = self.entropy.double().cpu().numpy()
        ts = self.timesteps.cpu().numpy()
        n2 = self.norm2.cpu().numpy() if self.norm2 is not None else [None] * len(rew)
        nov = np.zeros(len(rew)) if self.novelty is None else \
            (self.novelty.double().cpu().numpy() if torch.is_tensor(self.novelty) else np.asarray(self.novelty))
        os_host = None if self.obs_stats is None else tuple(t.cpu().numpy() for t in self.obs_stats)
        out = []
        for i in range(len(rew)):
            r = FDReturn()
            r.epoch = self.epoch
            r.is_eval = bool(self.is_eval[i])
            enc = getattr(self, "encoded", None)    # a host noise source's encoded draws (RNGNoiseSource states)
            r.encoded_noise = enc[i] if enc is not None else ("0" if r.is_eval else "{}".format(int(self.idx_host[i])))
            r.sign = int(self.sign_host[i])
            r.reward, r.entropy, r.timesteps = float(rew[i]), float(ent[i]), int(ts[i])
            r.novelty = float(nov[i])
            if os_host is not None:     # WelfordRunningStat.serialize() of this episode (worker.py:56)
                r.obs_stats_update = os_host[0][i].tolist() + os_host[1][i].tolist() + [int(os_host[2][i])]
            r.norm2 = None if n2[i] is None else float(n2[i])
            out.append(r)
        return out
