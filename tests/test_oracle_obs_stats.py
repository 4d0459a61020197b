"""CPU: oracle/obs_stats.py pinned to the reference WelfordRunningStat (G10, utils/math_helpers.py:7-124)."""
import numpy as np

from oracle import obs_stats as oo


def test_welford_updates_and_merge_match_reference(golden):
    g = golden("g10_welford.npz")
    d = int(g["d"])
    acc = oo.Welford(d)
    i = 0
    while "x%d" % i in g:
        w = oo.Welford(d)
        for x in g["x%d" % i]:
            w.update(x)
        ser = np.asarray(w.serialize(), np.float64)
        np.testing.assert_array_equal(ser, g["ser%d" % i])          # bit-exact f32 arithmetic
        acc.merge(w.mean_, w.m2, w.count)
        i += 1
    np.testing.assert_array_equal(np.asarray(acc.serialize(), np.float64), g["acc_ser"])
    np.testing.assert_array_equal(acc.mean, g["acc_mean"])
    np.testing.assert_array_equal(acc.std, g["acc_std"])
