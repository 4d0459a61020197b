"""GPU: AtariPolicy novelty (VERDICT r3 missing 4) -- the reference's StrategyHandler.compute_novelty calls
get_strategy on any policy (strategy/strategy_handler.py:25-30); AtariPolicy's is its forward over zeta
(policies/atari.py:30-31, stateless).  The device handler's lane novelty, archive and the env's eval-state frames
against the oracle: frames bit-exact, novelty <= 1e-5."""
import numpy as np
import pytest
import torch

from oracle import atari as oa
from oracle import noise as onoise
from oracle import novelty as onov

pytestmark = pytest.mark.gpu


def test_env_frames_match_oracle():
    from fdr import engine
    fr = engine.atari_env_frames(9, 7, 3, 4).cpu().numpy()
    ref = np.stack([oa.frames(9, [7], t)[0] for t in range(3, 7)]).astype(np.float32)
    np.testing.assert_array_equal(fr, ref)


def test_atari_lane_novelty_matches_oracle():
    from fdr import engine
    from policies import AtariPolicy
    from strategy import StrategyHandler
    from utils import math_helpers
    A = 6
    dev = torch.device("cuda", 0)
    pol = AtariPolicy((84, 84, 4), A, seed=124, device=dev)
    theta = pol.get_trainable_flat().copy()
    P = theta.size
    g = np.random.RandomState(3)
    nb = 16 + 32 + 256
    rm, rv = (g.randn(nb) * 0.1).astype(np.float32), (0.5 + g.rand(nb)).astype(np.float32)
    bns = [m for m in pol.model if isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d))]
    o = 0
    with torch.no_grad():
        for m in bns:
            n = m.num_features
            m.running_mean.copy_(torch.as_tensor(rm[o:o + n]))
            m.running_var.copy_(torch.as_tensor(rv[o:o + n]))
            o += n
    Z = 5
    zeta = engine.atari_env_frames(5, 0, 0, Z).cpu().numpy()
    h = StrategyHandler(pol, math_helpers.categorical_tvd, max_history_size=4)
    pts = [theta] + [(theta + np.float32(0.05) * g.randn(P).astype(np.float32)).astype(np.float32) for _ in range(2)]
    for f in pts:
        pol.set_trainable_flat(f)
        h.add_policy(pol)
    pol.set_trainable_flat(theta)
    h.set_zeta(zeta)
    bn = oa.split_bn(rm, rv)
    arch = np.stack([oa.forward(oa.unflatten(f, A), bn, zeta)[0].numpy() for f in pts])
    np.testing.assert_allclose(h.archive.cpu().numpy(), arch, rtol=1e-5, atol=1e-6)
    t = onoise.NoiseTable(1 << 21, P, 124)
    idx = np.repeat(t.sample_indices(3), 2)
    sign = np.tile(np.array([1, -1], np.int8), 3)
    tab = torch.as_tensor(t.table, device=dev)
    nov = h.lane_novelty(tab, torch.as_tensor(idx, device=dev), torch.as_tensor(sign, device=dev), 0.02)
    nov = nov.cpu().numpy()
    thetas = onoise.perturb(theta, t.table, idx, sign, 0.02)
    ref = [onov.novelty(oa.forward(oa.unflatten(th, A), bn, zeta)[0].numpy(), arch, "tvd") for th in thetas]
    np.testing.assert_allclose(nov, ref, rtol=1e-5, atol=1e-6)
    assert np.all(nov > 0)
    # compute_novelty of one policy (strategy_handler.py:26-31) = that lane's novelty
    pol.set_trainable_flat(thetas[0])
    assert abs(h.compute_novelty(pol) - ref[0]) <= 1e-5 * max(1.0, ref[0])


def test_sequential_runner_atari_novelty():
    """SequentialRunner(policy="atari") with the novelty archive: eval epochs refresh zeta from the env's frames,
    every lane is scored, the archive fills and replaces."""
    from run_sequential import SequentialRunner
    r = SequentialRunner(env_id="PongNoFrameskip-v4", policy="atari", antithetic=True, batch_size=2, episode_len=6,
                         zeta_size=4, eval_prob=0.5, max_strategy_history_size=2, random_seed=3,
                         noise_table_size=1 << 22, device="cuda", verbose=False)
    assert r.policy.KIND == "atari" and r.zeta.shape == (4, 4, 84, 84)
    r.train(4)
    assert len(r.history) == 4
    for rep in r.history:
        assert np.isfinite(rep["Noisy Reward"]) and np.isfinite(rep["Noisy Novelty"])
    assert r.strategy_handler.archive is not None and r.strategy_handler.archive.shape[1:] == (4, 6)
    assert any(rep["Noisy Novelty"] > 0 for rep in r.history[1:])


def test_batched_atari_strategies_equal_per_lane_forwards():
    """fdr_atari_strategies (every lane's theta' over the Z shared frames, one prep / conv / core
    launch per 256 lanes) is bitwise the per-lane path it replaced (fdr_perturb, then fdr_atari_forward over zeta
    for each lane) -- 300 lanes, so two chunks, with out-of-order offsets and a sign-0 lane."""
    from fdr import engine
    from policies import AtariPolicy
    A, Z, n = 5, 3, 300
    dev = torch.device("cuda", 0)
    pol = AtariPolicy((84, 84, 4), A, seed=124, device=dev)
    P = pol.num_params
    t = onoise.NoiseTable(1 << 21, P, 124)
    g = np.random.RandomState(4)
    idx = g.randint(0, t.table.size - P, size=n).astype(np.int64)
    sign = np.where(g.rand(n) < 0.5, 1, -1).astype(np.int8)
    sign[7] = 0
    tab = torch.as_tensor(t.table, device=dev)
    idx_d, sign_d = torch.as_tensor(idx, device=dev), torch.as_tensor(sign, device=dev)
    zeta = engine.atari_env_frames(5, 0, 0, Z)
    bm, bv = pol.bn_stats()
    got = engine.atari_strategies(pol.spec, engine.lanes_desc(pol.flat, 0, tab, idx_d, sign_d, 0.02), n, zeta, bm, bv)
    thetas = engine.perturb(pol.flat, tab, idx_d, sign_d, 0.02)
    want = torch.stack([engine.atari_forward(pol.spec, thetas[l].contiguous(), zeta, bm, bv) for l in range(n)])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), want.cpu().numpy())
