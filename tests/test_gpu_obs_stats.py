"""GPU: obs-normalisation statistics -- per-lane Welford partials sampled inside the rollout
(worker/agent.py:37-39, utils/math_helpers.py:29-38) and the in-order merge (:68-87, run_server.py:143).
Counts are exact (integer coins of the counter stream); per-lane mean / m2 rel 1e-4 (the GPU env state
differs from numpy's by ~1e-7 per step); the merge of given partials is bit-exact."""
import numpy as np
import pytest
import torch

from oracle import agent as oagent
from oracle import envs as oenvs
from oracle import noise as onoise
from oracle import obs_stats as oo
from oracle import policies as opol

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fdr import engine
    return engine


def dev(a):
    return torch.as_tensor(np.asarray(a)).to("cuda").contiguous()


@pytest.mark.parametrize("normalize", [False, True])
def test_lane_welford_vs_oracle(eng, normalize):
    from envs import SyntheticEnv
    torch.manual_seed(124)
    pol = opol.TorchPolicy("mujoco", 17, 6, seed=124)
    theta = pol.get_flat()
    t = onoise.NoiseTable(1 << 20, theta.size, 124)
    L, T, chance = 8, 200, 0.3
    idx = t.sample_indices(L)
    sign = np.ones(L, np.int8)
    om = np.linspace(-0.2, 0.2, 17).astype(np.float32) if normalize else None
    osd = np.linspace(0.5, 1.5, 17).astype(np.float32) if normalize else None
    spec = eng.PolicySpec("mujoco", 17, 6, theta.size)
    lanes = eng.lanes_desc(dev(theta), 0, dev(t.table), dev(idx), dev(sign), 0.02)
    res = eng.rollout(spec, SyntheticEnv(17, 6, False, T), lanes, L, 31, obs_mean=None if om is None else dev(om),
                      obs_std=None if osd is None else dev(osd), obs_stats=chance)
    torch.cuda.synchronize()
    ref = oagent.evaluate_lanes("mujoco", 17, 6, theta, t.table, idx, sign, 0.02, oenvs.BatchedSyntheticEnv(17, 6, False, T, L),
                                31, obs_mean=om, obs_std=osd, obs_chance=chance)
    stats = ref[4]
    cnt = res.obs_count.cpu().numpy()
    np.testing.assert_array_equal(cnt, [s.count for s in stats])
    assert 0.2 * T < cnt.mean() < 0.4 * T
    np.testing.assert_allclose(res.obs_mean.cpu().numpy(), np.stack([s.mean_ for s in stats]), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(res.obs_m2.cpu().numpy(), np.stack([s.m2 for s in stats]), rtol=1e-4, atol=1e-4)
    # the merge of these partials is bit-exact against the restated reference merge
    acc = (torch.zeros(17, device="cuda"), torch.zeros(17, device="cuda"), torch.zeros(1, dtype=torch.int64,
                                                                                     device="cuda"))
    eng.obs_stats_merge(res.obs_mean, res.obs_m2, res.obs_count, *acc)
    w = oo.Welford(17)
    for m, v, c in zip(res.obs_mean.cpu().numpy(), res.obs_m2.cpu().numpy(), cnt):
        w.merge(m, v, c)
    np.testing.assert_array_equal(acc[0].cpu().numpy(), w.mean_)
    np.testing.assert_array_equal(acc[1].cpu().numpy(), w.m2)
    assert int(acc[2].item()) == w.count


def test_runner_normalize_obs_accumulates_global_stats(eng):
    from run_sequential import SequentialRunner
    r = SequentialRunner(env_id="HalfCheetah-v4", batch_size=16, normalize_obs=True, episode_len=100,
                         noise_table_size=1 << 20, random_seed=5, eval_prob=0.2, verbose=False)
    r.agent.obs_stats_update_chance = 0.05
    r.train(2)
    c = int(r.global_obs[2].item())
    assert c > 0
    assert r.worker.fixed_obs_stats.count == c
    assert np.all(np.isfinite(r.worker.fixed_obs_stats.std)) and np.any(r.worker.fixed_obs_stats.std != 1.0)
    assert len(r.zeta) > 0 and r.strategy_handler.archive is not None
