"""CPU: the eval-lane convention of SequentialRunner with E > 1 frame envs per lane:
an eval lane's E returns / entropies / novelties are averaged into ONE evaluation before the reference's
0.9 / 0.1 EMA (run_sequential.py:136-143), so the EMAs and the zeta update count do not depend on E."""
import numpy as np

from run_sequential import eval_lane_means


def _ema(values, start=0.0):
    x = start
    for v in values:
        x = x * 0.9 + v * 0.1
    return x


def test_eval_lanes_with_four_envs_are_one_evaluation_each():
    E, n_train = 4, 8
    rew = np.concatenate([np.full(n_train, 100.0), np.arange(1.0, 9.0)])        # 2 eval lanes x 4 envs
    ent = np.concatenate([np.zeros(n_train), np.full(8, 0.5)])
    nov = np.concatenate([np.zeros(n_train), [0, 0, 0, 4, 1, 1, 1, 1]])
    r, e, nv = eval_lane_means((rew, ent, nov), n_train, E)
    np.testing.assert_array_equal(r, [2.5, 6.5])
    np.testing.assert_array_equal(e, [0.5, 0.5])
    np.testing.assert_array_equal(nv, [1.0, 1.0])
    # the runner's EMA after these two evaluations (2 updates, not 8; training lanes never enter it)
    assert abs(_ema(r) - 0.875) < 1e-15
    assert len(r) == 2


def test_one_env_is_the_reference_update():
    rew = np.array([5.0, -1.0, 3.0, 7.0])
    (r,) = eval_lane_means((rew,), 2, 1)
    np.testing.assert_array_equal(r, [3.0, 7.0])
    assert abs(_ema(r) - (0.3 * 0.9 + 0.7)) < 1e-15
