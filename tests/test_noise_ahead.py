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
