"""CPU: oracle/novelty.py pinned to the reference's own distance functions (G9, utils/math_helpers.py:147-222)."""
import numpy as np

from oracle import novelty as on


def test_distances_match_reference(golden):
    g = golden("g9_novelty.npz")
    np.testing.assert_allclose(on.categorical_tvd(g["cat_a"], g["cat_b"]), g["tvd"], rtol=1e-6)
    np.testing.assert_allclose(on.l2_dist(g["cat_a"], g["cat_b"]), g["l2"], rtol=1e-6)
    np.testing.assert_allclose(on.gaussian_w2(g["gau_a"], g["gau_b"]), g["w2"], rtol=1e-6)
    assert abs(on.novelty(g["cat_a"], g["cat_b"], "tvd") - float(g["nov_tvd"])) < 1e-7
    assert abs(on.novelty(g["cat_a"], g["cat_b"], "l2") - float(g["nov_l2"])) < 1e-7
    assert abs(on.novelty(g["gau_a"], g["gau_b"], "w2") - float(g["nov_w2"])) < 1e-6
    P = g["cat_b"]
    pair = np.array([[on.categorical_tvd(P[i], P[j][None])[0] for j in range(len(P))] for i in range(len(P))])
    np.testing.assert_allclose(pair, g["pair_tvd"], rtol=1e-6, atol=1e-7)
