"""Shared noise table, index stream and the theta +/- sigma*eps perturbation.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

  table   utils/noise_sources.py:37-42   RandomState(seed).randn(size).astype(float32)
  indices utils/noise_sources.py:44-47   randint(0, size - P) from the SAME RandomState, continuing
                                         after the table draw.  A vectorised randint(size=n) gives
                                         the identical stream as n scalar calls (checked against the
                                         reference's own sample() in tests/test_oracle_golden.py).
  decode  utils/noise_sources.py:49-51   table[idx : idx + P]
  perturb worker/worker.py:26-30         new_flat = flat + sigma * noise in numpy f32:
                                         fl32(theta + fl32(fl32(sigma) * eps)); antithetic lanes
                                         (build-defined) use fl32(theta - fl32(fl32(sigma) * eps)).
"""
import numpy as np


class NoiseTable(object):
    def __init__(self, size, n_params, seed=123):
        assert size > n_params
        self.rng = np.random.RandomState(seed)
        self.table = self.rng.randn(size).astype(np.float32)
        self.n_params = n_params
        self.max_idx = size - n_params

    def sample_indices(self, n):
        return self.rng.randint(0, self.max_idx, size=n).astype(np.int64)

    def decode(self, idx):
        return self.table[int(idx):int(idx) + self.n_params]


def perturb(theta, table, idx, sign, sigma):
    """theta [P] f32, idx [L] int64, sign [L] in {-1, 0, +1} -> theta' [L, P] f32 (bit-exact form)."""
    theta = np.asarray(theta, dtype=np.float32)
    P = theta.shape[0]
    out = np.empty((len(idx), P), dtype=np.float32)
    s32 = np.float32(sigma)
    for i, (ix, sg) in enumerate(zip(idx, sign)):
        if sg == 0:
            out[i] = theta
            continue
        step = (s32 * table[int(ix):int(ix) + P]).astype(np.float32)
        out[i] = (theta + step) if sg > 0 else (theta - step)
    return out
