"""SharedNoiseTable draw-ahead (peek_batch): consuming pre-drawn indices leaves the index stream exactly the
reference's (utils/noise_sources.py:44-47: one randint per sample from the table's RandomState)."""
import numpy as np


def test_peek_then_sample_is_the_sequential_stream():
    from utils.noise_sources import SharedNoiseTable
    a = SharedNoiseTable(1 << 16, 1000, random_seed=7)
    b = SharedNoiseTable(1 << 16, 1000, random_seed=7)
    seq = [int(b.sample()[0]) for _ in range(40)]
    got = []
    pk = a.peek_batch(10)
    assert np.array_equal(a.peek_batch(10), pk)            # peeking twice draws nothing new
    got += list(a.sample_batch(4))                          # part of the peeked batch
    got.append(int(a.sample()[0]))                          # a single draw from the queue
    got += list(a.sample_batch(12))                         # the rest of the queue + fresh draws
    assert np.array_equal(a.peek_batch(3), seq[17:20])
    got += list(a.sample_batch(23))
    assert got == seq
    assert list(pk) == seq[:10]


def test_noise_source_kinds_and_refusal():
    """the reference's default RNGNoiseSource (run_sequential.py:89) and SimpleNoiseSource are
    accepted as host noise sources (theta' rows materialised per lane); an object with neither the table nor the
    sample / decode interface is refused with a TypeError at construction, not an AttributeError mid-step.  The
    host sources keep the reference's streams: RNGNoiseSource.decode(sample()[0]) regenerates the sampled vector."""
    import pytest
    from learner.finite_differences import FiniteDifferences
    from utils.noise_sources import (RNGNoiseSource, SharedNoiseTable, SimpleNoiseSource, is_device_table,
                                     is_host_noise, require_noise_source)
    from worker.worker import Worker
    assert is_device_table(SharedNoiseTable(1 << 12, 100, 1)) and not is_host_noise(SharedNoiseTable(1 << 12, 100, 1))
    for src in (RNGNoiseSource(100, 1), SimpleNoiseSource(100, 1)):
        assert is_host_noise(src) and not is_device_table(src)
        require_noise_source(src, "Worker")
        enc, noise = src.sample()
        np.testing.assert_array_equal(src.decode(enc), noise)
        assert noise.dtype == np.float64 and noise.shape == (100,)
    with pytest.raises(TypeError, match="noise source"):
        Worker(object(), object(), object(), None)
    with pytest.raises(TypeError, match="noise source"):
        FiniteDifferences(object(), None, 0.0, object())
    r = RNGNoiseSource(50, 5)
    ref = np.random.default_rng(np.random.SeedSequence(5))
    for _ in range(3):
        enc, noise = r.sample()
        st = ref.bit_generator.state["state"]
        assert enc == "{},{}".format(st["state"], st["inc"])
        np.testing.assert_array_equal(noise, ref.standard_normal(size=50))


def test_native_index_draw_is_numpy_randint():
    """fdr_noise_draw_indices (the product's host draw) == RandomState.randint, the reference's draw
    (utils/noise_sources.py:45), word for word: the same indices and the same generator state afterwards --
    including the cached Gaussian of the table's randn, across 624-word refills and for masks of every width."""
    from utils.noise_sources import SharedNoiseTable
    for size, P, seed in ((1 << 16, 1000, 7), (25_000_000, 6092, 124), (6093, 6092, 3), (6094, 6092, 9),
                          ((1 << 20) + 1, 1, 11)):
        t = SharedNoiseTable(size, P, seed)
        ref = np.random.RandomState(seed)
        ref.randn(size)
        for n in (1, 5, 700, 16384, 3):
            got = t._draw(n)
            exp = ref.randint(0, size - P, size=n).astype(np.int64)
            assert np.array_equal(got, exp), (size, n)
        a, b = t.rng_state(), ref.get_state()
        assert np.array_equal(a[1], b[1]) and a[2:] == b[2:]
        assert t._rng.randn() == ref.randn()     # the cached Gaussian of the table's randn is carried


def test_host_draw_of_an_eight_rank_step_is_short():
    """at N = 8 every rank draws the whole 16,384-index stream of a config-3 step (2048
    directions x 8), then builds its lane slice and the packed upload.  It runs under the rollout it overlaps
    (Worker.evaluate(prefetch=True) draws the next step while this one runs): < 10 % of the ~1 ms step."""
    import time
    from utils.noise_sources import SharedNoiseTable
    from fdr import dist as fdist
    t = SharedNoiseTable(25_000_000, 6092, 124)
    ts = []
    for _ in range(30):
        t0 = time.perf_counter()
        idx = t.sample_batch(16384)
        lo, hi = fdist.lane_range(16384, 2, 8, 3)
        lidx = np.repeat(idx[lo // 2:hi // 2], 2)
        sign = np.tile(np.array([1, -1], np.int8), (hi - lo) // 2)
        m = hi - lo
        packed = np.empty(10 * m, np.uint8)
        packed[:8 * m] = lidx.view(np.uint8)
        packed[8 * m:9 * m] = sign.view(np.uint8)
        packed[9 * m:] = 0
        ts.append(time.perf_counter() - t0)
    med = float(np.median(ts))
    print("host draw + lane slice + pack, 16384 indices: %.1f us" % (med * 1e6))
    assert med < 100e-6 * 2   # 2x margin over the < 0.1 ms target for a loaded CI host
