"""Noise sources -- the API of utils/noise_sources.py:4-51, with a GPU-resident shared table.

``SharedNoiseTable`` is the hot-path source:
  * table = RandomState(seed).randn(size).astype(float32)       (noise_sources.py:39-40)
  * indices drawn from the SAME RandomState, continuing after the table draw
    (noise_sources.py:45): sample() draws one, ``sample_batch(n)`` draws n at once -- numpy's
    vectorised randint yields the identical MT19937 stream (pinned in tests/test_oracle_golden.py);
  * the table is uploaded once per device and stays resident in HBM (100 MB at 25M entries);
    the HIP kernels gather table[idx : idx + P] directly, theta' is never materialised;
  * ``peek_batch(n)`` draws ahead without consuming: the next sample / sample_batch calls return those
    indices first, so the stream is unchanged (a batch of n draws is n single draws) -- the worker uses it
    to upload the next FD step's lane descriptors while the current rollout runs.
"""
import ctypes

import numpy as np
import torch


class SharedNoiseTable(object):
    def __init__(self, size, n_params, random_seed=123):
        assert size > n_params, "!ATTEMPTED TO MAKE NOISE TABLE WITH SIZE {} FOR {} PARAMETERS!".format(size, n_params)
        rng = np.random.RandomState(random_seed)
        self._table = rng.randn(size).astype(np.float32)
        self._n_params = n_params
        self._max_sample_idx = size - n_params
        self._device_tables = {}
        self._ahead = np.empty(0, np.int64)     # drawn by peek_batch, not yet consumed
        # the index stream continues the table's MT19937 state (noise_sources.py:45); the draws advance this copy of
        # it natively (fdr_noise_draw_indices), and rng_state() / _rng hand it back in numpy's format
        name, key, pos, has_gauss, cached = rng.get_state()
        self._mt_key = np.array(key, dtype=np.uint32)
        self._mt_pos = ctypes.c_int32(int(pos))
        self._mt_extra = (name, has_gauss, cached)

    def rng_state(self):
        """The index stream's generator state as numpy's RandomState.get_state() tuple."""
        name, has_gauss, cached = self._mt_extra
        return (name, self._mt_key.copy(), int(self._mt_pos.value), has_gauss, cached)

    @property
    def _rng(self):
        """A RandomState at the index stream's current position (the reference's attribute; a snapshot)."""
        rs = np.random.RandomState()
        rs.set_state(self.rng_state())
        return rs

    @property
    def size(self):
        return self._table.size

    def sample(self):
        idx = int(self.sample_batch(1)[0])
        return "{}".format(idx), self._table[idx:idx + self._n_params]

    def _draw(self, n):
        """n randint(0, max_idx) draws continuing the table's RandomState stream: fdr_noise_draw_indices advances the
        MT19937 state natively -- bit-identical to RandomState.randint (tests/test_noise_ahead.py), ~4x faster
        than numpy's per-word loop at the sizes one step draws (16,384 indices per rank at N = 8)."""
        n = int(n)
        out = np.empty(n, np.int64)
        if n == 0:
            return out
        try:
            from fdr import _lib                # loaded on first draw: utils stays importable without libfdr.so
        except ImportError:
            _lib = None
        rc = 2 if _lib is None else _lib.lib.fdr_noise_draw_indices(self._mt_key.ctypes.data, ctypes.byref(self._mt_pos), self._max_sample_idx,
                                             n, out.ctypes.data)
        if rc == 2:   # FDR_ERR_UNSUPPORTED (a table wider than 2^32 entries) or no libfdr.so: numpy's own draw
            rs = self._rng
            out = rs.randint(0, self._max_sample_idx, size=n).astype(np.int64)
            _, key, pos, _, _ = rs.get_state()
            self._mt_key[:] = key
            self._mt_pos.value = int(pos)
            return out
        _lib.check(rc, "fdr_noise_draw_indices")
        return out

    def peek_batch(self, n):
        """The next n indices, drawn ahead but not consumed."""
        n = int(n)
        if self._ahead.size < n:
            self._ahead = np.concatenate([self._ahead, self._draw(n - self._ahead.size)])
        return self._ahead[:n].copy()

    def sample_batch(self, n):
        """n indices in the order n sample() calls would draw them (int64 numpy array)."""
        n = int(n)
        if self._ahead.size == 0:
            return self._draw(n)
        out = self.peek_batch(n)
        self._ahead = self._ahead[n:]
        return out

    def decode(self, noise_idx):
        noise_idx = int(noise_idx)
        return self._table[noise_idx:noise_idx + self._n_params]

    def device_table(self, device=None):
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        t = self._device_tables.get(dev)
        if t is None:
            t = torch.from_numpy(self._table).to(dev)
            self._device_tables[dev] = t
        return t


class RNGNoiseSource(object):
    """noise_sources.py:4-20 (the reference runner's default source, run_sequential.py:89): every perturbation is a
    fresh standard_normal(P) draw (f64) of one PCG64 stream, encoded as that stream's state string.  Uses
    bit_generator.state: Generator.__getstate__ returns None on numpy >= 2, which breaks the reference (SURVEY.md
    finding 3).  decode() regenerates from a fresh bit generator instead of rewinding self.rng (the reference
    restores the state into its shared rng: in its synchronous loop that leaves the stream where the worker's
    last draw left it, which is where this stream stays).

    A host noise source: the GPU path materialises each lane's theta' = fl32(theta + sigma * noise) on the host,
    exactly the reference's f64 arithmetic (worker.py:28), and hands the rows to the kernels through
    fdr_lanes_desc.base_stride; the learner gathers lambda from the fl32(noise) rows (Worker / FiniteDifferences,
    HostNoiseRows).  Correct, and slow: numpy draws P normals per perturbation on one core."""

    host_noise = True

    def __init__(self, n_params, random_seed=123):
        self.rng = np.random.default_rng(np.random.SeedSequence(random_seed))
        self.n_params = n_params

    def sample(self):
        st = self.rng.bit_generator.state["state"]
        enc = "{},{}".format(st["state"], st["inc"])
        return enc, self.rng.standard_normal(size=self.n_params)

    def decode(self, state):
        s, inc = (int(v) for v in state.split(","))
        bg = np.random.PCG64()
        st = bg.state
        st["state"]["state"], st["state"]["inc"] = s, inc
        st["has_uint32"], st["uinteger"] = 0, 0
        bg.state = st
        return np.random.Generator(bg).standard_normal(size=self.n_params)


class SimpleNoiseSource(object):
    """noise_sources.py:23-33: ships the raw noise vector (RandomState.randn, f64).  A host noise source like
    RNGNoiseSource: its encoded perturbation IS the vector."""

    host_noise = True

    def __init__(self, n_params, random_seed=123):
        self.rng = np.random.RandomState(random_seed)
        self.n_params = n_params

    def sample(self):
        noise = self.rng.randn(self.n_params)
        return noise, noise

    def decode(self, noise):
        return noise


def is_device_table(noise_source):
    """A table source the kernels gather from by offset (SharedNoiseTable's device_table / sample_batch interface)."""
    return hasattr(noise_source, "device_table") and hasattr(noise_source, "sample_batch")


def is_host_noise(noise_source):
    """A host source with the reference interface sample() -> (encoded, noise) / decode(encoded) -> noise."""
    return (not is_device_table(noise_source) and hasattr(noise_source, "sample") and
            hasattr(noise_source, "decode"))


def require_noise_source(noise_source, who):
    """Worker / FiniteDifferences take a SharedNoiseTable (the fast path: offsets into an HBM-resident table, theta'
    never materialised) or a host source with the reference's sample / decode interface (RNGNoiseSource,
    SimpleNoiseSource: theta' rows materialised per lane).  Anything else is refused at construction with a clear
    error rather than an AttributeError in the middle of a step."""
    if not (is_device_table(noise_source) or is_host_noise(noise_source)):
        raise TypeError("%s needs a noise source with the reference interface (SharedNoiseTable, RNGNoiseSource or "
                        "SimpleNoiseSource); got %s" % (who, type(noise_source).__name__))


class HostNoiseRows(object):
    """Device rows of a host noise source's perturbations for one launch / learner step.
      theta   [n_lanes, P] f32: theta'_l = fl32(theta + s_l * sigma * noise_l) in f64 as worker.py:28 forms it
              (set_trainable_flat rounds to f32), theta for eval lanes (s = 0); fdr_lanes_desc base / base_stride P
      table   [n_rows * P] f32: fl32(noise_r), the "table" the norms / gradient / lane strategies gather from
      idx     [n_lanes] int64 offsets row * P into table (0 for eval lanes)"""

    def __init__(self, flat_host, noises, row_of_lane, sign, sigma, device, with_theta=True):
        P = flat_host.size
        noises = np.asarray(noises, dtype=np.float64).reshape(-1, P)
        row_of_lane = np.asarray(row_of_lane, np.int64)
        sign = np.asarray(sign)
        self.table = torch.as_tensor(noises.astype(np.float32).reshape(-1), device=device)
        self.idx_host = np.where(sign != 0, row_of_lane * P, 0).astype(np.int64)
        self.theta = None
        if with_theta:
            f64 = flat_host.astype(np.float64)
            th = np.empty((len(sign), P), np.float32)
            for l in range(len(sign)):
                if sign[l] == 0:
                    th[l] = flat_host
                else:
                    th[l] = (f64 + float(sigma) * noises[row_of_lane[l]]) if sign[l] > 0 else \
                        (f64 - float(sigma) * noises[row_of_lane[l]])
            self.theta = torch.as_tensor(th, device=device)
