"""Strategy distances and novelty (utils/math_helpers.py:147-222) -- numpy restatement.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py); pinned by tests/golden/g9_novelty.npz, which the
reference's own math_helpers produced.  a: [Z, D] (one strategy = get_strategy over the probe states
zeta), b: [H, Z, D] (the archive) -> [H].
"""
import numpy as np


def l2_dist(a, b):
    """math_helpers.py:166-170: mean_z || b - a ||_2."""
    return np.linalg.norm(np.asarray(b) - np.asarray(a), axis=-1).mean(axis=-1)


def categorical_tvd(a, b):
    """math_helpers.py:216-219: mean_z sum_d |a - b| (no 1/2 factor)."""
    return np.abs(np.subtract(a, b)).sum(axis=-1).mean(axis=-1)


def gaussian_w2(a, b):
    """math_helpers.py:202-213 (gaussian_wasserstein_dist_from_strategies): D = 2k = [mean | std];
    mean_z ( ||m1 - m2||^2 + sum(s1 + s2 - 2 sqrt(s1 s2)) )."""
    a, b = np.asarray(a), np.asarray(b)
    k = a.shape[-1] // 2
    m1, s1, m2, s2 = a[..., :k], a[..., k:], b[..., :k], b[..., k:]
    inside = s1 + s2 - 2 * np.sqrt(s1 * s2)
    return (np.square(np.linalg.norm(m1 - m2, axis=-1)) + inside.sum(axis=-1)).mean(axis=-1)


DISTANCES = {"l2": l2_dist, "tvd": categorical_tvd, "w2": gaussian_w2}


def novelty(a, b, kind):
    """compute_strategy_novelty (math_helpers.py:147-155): min over the archive."""
    return float(np.min(DISTANCES[kind](a, b)))
