"""GPU: the novelty path -- fdr_strategy_distances vs the reference's distances (G9),
batched lane strategies vs the oracle forward, the device StrategyHandler, recorded eval states.
Tolerances: distances rel 1e-5 (f64 accumulation vs the reference's f32 numpy); strategies 1e-5 abs."""
import numpy as np
import pytest
import torch

from oracle import envs as oe
from oracle import noise as onz
from oracle import novelty as on
from oracle import policies as op

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fdr import engine
    return engine


def _t(a):
    return torch.as_tensor(np.asarray(a), device="cuda")


def test_distances_match_reference_golden(engine, golden):
    g = golden("g9_novelty.npz")
    for kind, a, b in (("tvd", "cat_a", "cat_b"), ("l2", "cat_a", "cat_b"), ("w2", "gau_a", "gau_b")):
        mn, am, d = engine.strategy_distances(_t(g[a])[None], _t(g[b]), kind, full=True)
        np.testing.assert_allclose(d.cpu().numpy()[0], g[kind], rtol=1e-5)
        assert abs(mn.item() - float(g["nov_" + kind])) <= 1e-5 * abs(float(g["nov_" + kind]))
        assert am.item() == int(np.argmin(g[kind]))
    _, _, pair = engine.strategy_distances(_t(g["cat_b"]), _t(g["cat_b"]), "tvd", full=True)
    np.testing.assert_allclose(pair.cpu().numpy(), g["pair_tvd"], rtol=1e-5, atol=1e-7)


def test_distances_many_lanes_vs_oracle(engine):
    rs = np.random.RandomState(1)
    S = rs.rand(300, 50, 4).astype(np.float32)
    B = rs.rand(37, 50, 4).astype(np.float32)
    mn, am, d = engine.strategy_distances(_t(S), _t(B), "l2", full=True)
    ref = np.stack([on.l2_dist(S[i], B) for i in range(len(S))])
    np.testing.assert_allclose(d.cpu().numpy(), ref, rtol=1e-5)
    np.testing.assert_array_equal(am.cpu().numpy(), ref.argmin(1))


@pytest.mark.parametrize("kind,n_in,n_act", [("discrete", 4, 2), ("mujoco", 17, 6)])
def test_lane_strategies_and_novelty(engine, kind, n_in, n_act):
    from policies import DiscretePolicy, MujocoPolicy
    from strategy import StrategyHandler
    from utils import math_helpers
    torch.manual_seed(124)
    pol = (DiscretePolicy if kind == "discrete" else MujocoPolicy)(n_in, n_act, seed=124)
    P = pol.num_params
    table = np.random.RandomState(124).randn(1 << 20).astype(np.float32)
    tt = _t(table)
    rs = np.random.RandomState(2)
    zeta = rs.randn(20, n_in).astype(np.float32)
    dist = math_helpers.categorical_tvd if kind == "discrete" else math_helpers.gaussian_wasserstein_dist_from_strategies
    h = StrategyHandler(pol, dist, max_history_size=4)
    theta = pol.get_trainable_flat().copy()
    arch_idx = [100, 2000, 30000]
    for i in arch_idx:                                   # archive: three perturbed policies
        pol.set_trainable_flat(onz.perturb(theta, table, [i], [1], 0.02)[0])
        h.add_policy(pol)
    pol.set_trainable_flat(theta)
    h.set_zeta(zeta)

    def oracle_strategy(flat):
        out = op.lanes_forward(kind, n_in, n_act, np.repeat(flat[None], len(zeta), 0), zeta)
        return out if kind == "discrete" else np.concatenate(out, -1)
    arch = np.stack([oracle_strategy(onz.perturb(theta, table, [i], [1], 0.02)[0]) for i in arch_idx])
    np.testing.assert_allclose(h.strategy_tensor, arch, atol=1e-5)
    okind = "tvd" if kind == "discrete" else "w2"
    idx = np.array([5, 700, 9000, 123456, 5, 77], np.int64)
    sign = np.array([1, -1, 1, 1, -1, 0], np.int8)
    nov = h.lane_novelty(tt, _t(idx), _t(sign), 0.02).cpu().numpy()
    ref = [on.novelty(oracle_strategy(onz.perturb(theta, table, [i], [s], 0.02)[0]), arch, okind)
           for i, s in zip(idx, sign)]
    np.testing.assert_allclose(nov, ref, rtol=1e-4, atol=1e-6)
    assert abs(h.compute_novelty(pol) - on.novelty(oracle_strategy(theta), arch, okind)) < 1e-4 * max(1, ref[-1])
    # full archive: a point more novel than the closest pair replaces its less novel member
    h.add_policy(pol)
    assert len(h.points) == 4
    pol.set_trainable_flat(onz.perturb(theta, table, [400000], [1], 0.5)[0])
    h.set_zeta(zeta)
    r = h.add_policy(pol)
    assert r is not None and r >= -1


def test_rollout_records_visited_states(engine):
    from envs import SyntheticEnv
    from policies import MujocoPolicy
    torch.manual_seed(124)
    pol = MujocoPolicy(17, 6, seed=124)
    env = SyntheticEnv.named("halfcheetah", episode_len=50)
    states = torch.empty((2, 50, 17), dtype=torch.float32, device="cuda")
    det = torch.ones(2, dtype=torch.int8, device="cuda")
    res = engine.rollout(pol.spec, env, engine.lanes_desc(pol.flat, 0, deterministic=det), 2, 0, jiggle=False,
                         states=states)
    torch.cuda.synchronize()
    S = states.cpu().numpy()
    oenv = oe.SyntheticEnv(17, 6, False, 50, env_seed=0)
    np.testing.assert_array_equal(S[0, 0], oenv.reset())
    theta = pol.get_trainable_flat()
    mean, _ = op.lanes_forward("mujoco", 17, 6, np.repeat(theta[None], 49, 0), S[0, :-1])
    nxt = np.tanh(S[0, :-1] @ oenv.M.T + mean @ oenv.K.T)
    np.testing.assert_allclose(S[0, 1:], nxt, atol=2e-5)
    np.testing.assert_array_equal(S[0], S[1])
    np.testing.assert_allclose(res.reward.cpu().numpy()[0], S[0, 1:, 0].sum() + np.tanh(S[0, -1] @ oenv.M.T
                               + op.lanes_forward("mujoco", 17, 6, theta[None], S[0, -1:])[0] @ oenv.K.T)[0, 0],
                               rtol=1e-4)


@pytest.mark.parametrize("tag,kind,n_in,n_act,fn", [("disc", "discrete", 4, 2, "categorical_tvd"),
                                                    ("mj", "mujoco", 17, 6, "gaussian_wasserstein_dist_from_strategies")])
def test_archive_replacement_matches_reference(engine, golden, tag, kind, n_in, n_act, fn):
    """StrategyHandler.add_policy on the device archive == the reference SparseHistoryManager (G12): every
    submit's return (replaced index / -1), the worst_point_idx trace, the final archive and distance table."""
    from policies import DiscretePolicy, MujocoPolicy
    from strategy import StrategyHandler
    from utils import math_helpers
    z = golden("g12_history.npz")
    H = int(z[tag + "_H"])
    flats, zeta = z[tag + "_flats"], z[tag + "_zeta"]
    torch.manual_seed(124)
    pol = (DiscretePolicy if kind == "discrete" else MujocoPolicy)(n_in, n_act, seed=124, device="cuda")
    h = StrategyHandler(pol, getattr(math_helpers, fn), max_history_size=H)
    for k in range(H):
        pol.set_trainable_flat(flats[k])
        assert h.add_policy(pol) is None
    h.set_zeta(zeta)
    worst, rets = [h.worst_point_idx], []
    for k in range(H, len(flats)):
        pol.set_trainable_flat(flats[k])
        r = h.add_policy(pol)
        rets.append(-2 if r is None else r)
        worst.append(h.worst_point_idx)
    np.testing.assert_array_equal(rets, z[tag + "_returns"])
    np.testing.assert_array_equal(worst, z[tag + "_worst"])
    np.testing.assert_allclose(h.archive.cpu().numpy(), z[tag + "_strategies"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(h.pair, z[tag + "_dists"], rtol=1e-5)


@pytest.mark.parametrize("carry", [False, True])
def test_impala_archive_replacement_matches_reference(engine, golden, carry):
    """the device StrategyHandler over an ImpalaPolicy (fdr_impala_strategies: conv stack on
    the shared zeta frames, the zeta obs as ONE LSTM sequence from the reset state) against G12-impala, made by
    the reference's StrategyHandler / SparseHistoryManager with get_strategy from reset (the build's documented
    zero-state rule): every submit's return and worst_point_idx, the archive (f32, 1e-5), the distance table
    and compute_novelty.  carry=True (VERDICT r4 missing 4): StrategyHandler(carry_state=True) chains the LSTM
    state through the policy object as the unpatched reference does, against G12-impala-unpatched."""
    from policies import ImpalaPolicy
    from strategy import StrategyHandler
    from utils import math_helpers
    z = golden("g12_impala_unpatched.npz" if carry else "g12_impala.npz")
    A, H, P = int(z["A"]), int(z["H"]), int(z["P"])
    table = np.random.RandomState(int(z["table_seed"])).randn(2 ** 22).astype(np.float32)
    off = int(z["param_offset"])
    theta = (table[off:off + P] * np.float32(0.1)).astype(np.float32)
    flats = [(theta + s * table[o:o + P]).astype(np.float32) for s, o in zip(z["scales"], z["offs"])]
    pol = ImpalaPolicy((64, 64, 3), A, seed=124)
    assert pol.num_params == P
    o = 0
    for m in pol.model.bn_layers():
        n = m.num_features
        m.running_mean.copy_(torch.as_tensor(z["rm"][o:o + n]))
        m.running_var.copy_(torch.as_tensor(z["rv"][o:o + n]))
        o += n
    Z = z["zeta_frames"].shape[0]
    zeta = {"frame": torch.as_tensor(z["zeta_frames"].astype(np.float32)).view(Z, 1, 3, 64, 64),
            "reward": torch.as_tensor(z["zeta_rewards"]).view(Z, 1),
            "done": torch.zeros(Z, 1, dtype=torch.bool)}
    h = StrategyHandler(pol, math_helpers.categorical_tvd, max_history_size=H, carry_state=carry)
    for k in range(H):
        pol.set_trainable_flat(flats[k])
        assert h.add_policy(pol) is None
    h.set_zeta(zeta)
    worst, rets = [h.worst_point_idx], []
    for k in range(H, len(flats)):
        pol.set_trainable_flat(flats[k])
        r = h.add_policy(pol)
        rets.append(-2 if r is None else r)
        worst.append(h.worst_point_idx)
    np.testing.assert_array_equal(rets, z["returns"])
    np.testing.assert_array_equal(worst, z["worst"])
    np.testing.assert_allclose(h.archive.cpu().numpy(), z["strategies"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(h.pair, z["dists"], rtol=1e-5)
    for k, want in zip((0, len(flats) - 1), z["novelty"]):
        pol.set_trainable_flat((theta - z["scales"][k] * table[z["offs"][k]:z["offs"][k] + P]).astype(np.float32))
        assert abs(h.compute_novelty(pol) - want) <= 1e-5 * max(1.0, want)
