"""Pin the CPU oracle against fixtures produced by the reference itself (tests/golden/make_golden.py)."""
import hashlib

import numpy as np
import pytest
import torch

from oracle import agent as oagent
from oracle import envs as oenvs
from oracle import learner as olearn
from oracle import noise as onoise
from oracle import policies as opol
from oracle import runner as orunner

SHAPES = {"trap": ("discrete", 2, 9), "cartpole": ("discrete", 4, 2), "cheetah": ("mujoco", 17, 6)}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("seed,P", [(124, 5197), (124, 4874), (124, 6092), (7, 5197), (7, 6092)])
def test_noise_table_and_indices(golden, seed, P):
    g = golden("g1_noise.npz")
    key = "s%d_p%d" % (seed, P)
    t = onoise.NoiseTable(2 ** 22, P, seed)
    assert sha(t.table) == str(g[key + "_sha"])
    np.testing.assert_array_equal(t.table[[0, 1, 2, 1000, 2 ** 21, 2 ** 22 - 1]], g[key + "_spot"])
    np.testing.assert_array_equal(t.sample_indices(64), g[key + "_idx"])


def test_noise_indices_bench_size(golden):
    g = golden("g1_noise.npz")
    t = onoise.NoiseTable(25_000_000, 6092, 124)
    assert sha(t.table) == str(g["big_sha"])
    # vectorised draw in two chunks == 256 scalar reference draws
    idx = np.concatenate([t.sample_indices(100), t.sample_indices(156)])
    np.testing.assert_array_equal(idx, g["big_idx"])


def _policy(kind, n_in, n_act, seed):
    torch.manual_seed(seed)
    return opol.TorchPolicy(kind, n_in, n_act, seed=seed)


@pytest.mark.parametrize("name", list(SHAPES))
def test_init_and_perturb_bit_exact(golden, name):
    g = golden("g2_perturb.npz")
    kind, n_in, n_act = SHAPES[name]
    for seed in (124, 123):
        np.testing.assert_array_equal(_policy(kind, n_in, n_act, seed).get_flat(), g["%s_s%d_theta" % (name, seed)])
    theta = g["%s_s124_theta" % name]
    t = onoise.NoiseTable(2 ** 22, theta.size, 124)
    idx = t.sample_indices(4)
    np.testing.assert_array_equal(idx, g[name + "_idx"])
    out = onoise.perturb(theta, t.table, idx, [1, 1, 1, 1], 0.02)
    np.testing.assert_array_equal(out, g[name + "_perturbed"])


@pytest.mark.parametrize("name", list(SHAPES))
def test_forward(golden, name):
    g = golden("g3_forward.npz")
    kind, n_in, n_act = SHAPES[name]
    P = opol.num_params(kind, n_in, n_act)
    t = onoise.NoiseTable(2 ** 22, P, 124)
    params = (t.decode(int(g[name + "_idx"])) * 0.1).astype(np.float32)
    x = g[name + "_x"]
    pol = _policy(kind, n_in, n_act, 124)
    pol.set_flat(params)
    lanes = np.repeat(params[None], len(x), axis=0)
    if kind == "discrete":
        with torch.no_grad():
            np.testing.assert_allclose(pol.forward(x).numpy(), g[name + "_probs"], atol=1e-7)
        np.testing.assert_allclose(opol.lanes_forward(kind, n_in, n_act, lanes, x), g[name + "_probs"], atol=1e-6)
        assert abs(pol.entropy(x) - float(g[name + "_entropy"])) < 1e-6
        ent = opol.categorical_entropy(opol.lanes_forward(kind, n_in, n_act, lanes, x)).mean()
        assert abs(ent - float(g[name + "_entropy"])) < 1e-5
        assert [pol.act(x[i], True, None) for i in range(8)] == list(g[name + "_argmax"])
        stats = [(g["%s_vbn_rm%d" % (name, i)], g["%s_vbn_rv%d" % (name, i)]) for i in range(3)]
        np.testing.assert_allclose(opol.lanes_forward(kind, n_in, n_act, lanes, x, stats),
                                   g[name + "_vbn_probs"], atol=1e-6)
    else:
        m, s = opol.lanes_forward(kind, n_in, n_act, lanes, x)
        np.testing.assert_allclose(m, g[name + "_mean"], atol=1e-6)
        np.testing.assert_allclose(s, g[name + "_std"], atol=1e-6)
        assert abs(opol.normal_entropy(s).mean() - float(g[name + "_entropy"])) < 1e-5
        np.testing.assert_allclose(np.stack([pol.act(x[i], True, None) for i in range(8)]),
                                   g[name + "_det_action"], atol=1e-7)


@pytest.mark.parametrize("case", ["cheetah_n16", "cheetah_n64", "trap_n16"])
def test_fd_step(golden, case):
    g = golden("g4_fd_step.npz")
    name = case.split("_")[0]
    kind, n_in, n_act = SHAPES[name]
    theta0 = g[case + "_theta0"]
    P = theta0.size
    t = onoise.NoiseTable(2 ** 22, P, 124)
    N = len(g[case + "_idx"])
    idx = t.sample_indices(N)
    np.testing.assert_array_equal(idx, g[case + "_idx"])
    L = olearn.FDLearner(theta0, t.table, P, 0.02, 0.01)
    om = float(g[case + "_omega"])
    upd, gr = L.step([0] * N, idx, [1] * N, g[case + "_rewards"], 0.25, omega=om)
    rel = np.linalg.norm(gr - g[case + "_g"]) / np.linalg.norm(g[case + "_g"])
    assert rel < 1e-5
    np.testing.assert_allclose(L.theta, g[case + "_theta1"], rtol=0, atol=1e-6)
    assert abs(upd - float(g[case + "_update"])) < 1e-5
    # second step with one-epoch-stale returns (lambda drift)
    idx2 = t.sample_indices(N)
    np.testing.assert_array_equal(idx2, g[case + "_idx2"])
    upd2, gr2 = L.step(list(g[case + "_ep2"]), idx2, [1] * N, g[case + "_rewards2"], -0.5, omega=om)
    rel = np.linalg.norm(gr2 - g[case + "_g2"]) / np.linalg.norm(g[case + "_g2"])
    assert rel < 1e-5
    np.testing.assert_allclose(L.theta, g[case + "_theta2"], rtol=0, atol=1e-6)


def test_trap_env_known_answers(golden):
    g = golden("g5_trap.npz")
    env = oenvs.TrapEnv()
    np.testing.assert_array_equal(env.walkable, g["walkable"])
    np.testing.assert_array_equal(env.reset(), g["start_obs"])
    for a in range(9):
        env.reset()
        tot, done, steps = 0, False, 0
        while not done:
            _, r, done, _ = env.step(a)
            tot += r
            steps += 1
        assert steps == 201
        assert tot == g["const_return"][a]
        assert (env.col, env.row) == (g["const_col"][a], g["const_row"][a])


@pytest.mark.parametrize("seed", [124, 1, 2])
def test_trap_deterministic_episode(golden, seed):
    g = golden("g5_trap.npz")
    pol = _policy("discrete", 2, 9, seed)
    np.testing.assert_array_equal(pol.get_flat(), g["det_s%d_theta" % seed])
    env = oenvs.TrapEnv()
    rng = np.random.RandomState(seed)
    r, e, steps, _ = oagent.collect_return(pol, env, env.reset(), True, None,
                                           lambda: rng.choice((-1e-12, 1e-12)))
    ref = g["det_s%d" % seed]
    assert r == ref[0] and steps == ref[2]
    assert abs(e - ref[1]) < 1e-6


def test_sequential_runner_trap(golden):
    g = golden("g6_runner_trap.npz")
    out = orunner.run_trap(2)
    for e, rec in enumerate(out["log"]):
        np.testing.assert_array_equal(rec["idx"], g["e%d_idx" % e])
        np.testing.assert_array_equal(rec["rewards"], g["e%d_rewards" % e])
        assert rec["policy_reward"] == float(g["e%d_policy_reward" % e])
        assert abs(rec["update"] - g["update_magnitude_printed"][e]) < 1e-4
    assert out["cum_steps"] == int(g["cum_steps"])
    np.testing.assert_allclose(out["theta"], g["theta_final"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("name", ["cheetah", "cartpole"])
def test_worker_synthetic_episodes(golden, name):
    """Episode loop (agent.py:20-71) + worker perturbation (worker.py:20-38) vs the reference."""
    g = golden("g7_worker_synthetic.npz")
    kind, n_in, n_act = SHAPES[name]
    T = int(g[name + "_T"])
    pol = _policy(kind, n_in, n_act, 124)
    theta = pol.get_flat()
    np.testing.assert_array_equal(theta, g[name + "_theta"])
    env = oenvs.SyntheticEnv(n_in, n_act, kind == "discrete", T)
    t = onoise.NoiseTable(2 ** 22, theta.size, 124)
    worker_rng, agent_rng, inj = (np.random.RandomState(3), np.random.RandomState(11), np.random.RandomState(31))
    obs = env.reset()
    for i in range(8):
        is_eval = worker_rng.uniform(0, 1) < 0.25
        assert is_eval == g[name + "_is_eval"][i]
        if not is_eval:
            idx = int(t.sample_indices(1)[0])
            assert idx == g[name + "_idx"][i]
            pol.set_flat(theta + np.float32(0.02) * t.decode(idx))
        else:
            pol.set_flat(theta)
        noise_fn = (lambda s: np.float32(inj.uniform())) if kind == "discrete" else \
                   (lambda s: inj.randn(n_act).astype(np.float32))
        r, e, steps, obs = oagent.collect_return(pol, env, obs, is_eval, noise_fn,
                                                 lambda: agent_rng.choice((-1e-12, 1e-12)))
        pol.set_flat(theta)
        assert steps == g[name + "_timesteps"][i]
        assert abs(r - g[name + "_reward"][i]) <= 1e-9 * max(1.0, abs(r))
        assert abs(e - g[name + "_entropy"][i]) < 1e-6


def test_history_replacement_matches_reference(golden):
    """oracle.history (SparseHistoryManager restated) reproduces the reference's submit_policy returns,
    worst_point_idx trace, final strategies and distance table (G12), from strategies computed by the
    oracle's policy forward."""
    from oracle import history, policies
    z = golden("g12_history.npz")
    for tag, kind, n_in, n_act, dist in (("disc", "discrete", 4, 2, "tvd"), ("mj", "mujoco", 17, 6, "w2")):
        pol = policies.TorchPolicy(kind, n_in, n_act, seed=124)
        H = int(z[tag + "_H"])
        flats, zeta = z[tag + "_flats"], z[tag + "_zeta"]

        def strat(f):
            pol.set_flat(f)
            out = pol.forward(zeta)
            return (torch.cat(out, -1) if isinstance(out, tuple) else out).detach().numpy()
        hist = history.History(dist, H)
        for k in range(H):
            hist.submit(None, False)
        hist.evaluate([strat(f) for f in flats[:H]])
        worst, rets = [hist.worst_point_idx], []
        for k in range(H, len(flats)):
            r = hist.submit(strat(flats[k]), True)
            rets.append(-2 if r is None else r)
            worst.append(hist.worst_point_idx)
        np.testing.assert_array_equal(rets, z[tag + "_returns"])
        np.testing.assert_array_equal(worst, z[tag + "_worst"])
        np.testing.assert_allclose(np.stack(hist.strategies), z[tag + "_strategies"], rtol=0, atol=1e-6)
        D = np.full((H, H), np.inf)
        for (i, j), d in hist.known.items():
            D[i, j] = D[j, i] = d
        np.testing.assert_allclose(D, z[tag + "_dists"], rtol=1e-6)


def _g12i_flats(z):
    """The G12-impala parameter vectors, regenerated from the committed seeds (4.6 MB each, not committed)."""
    P = int(z["P"])
    table = np.random.RandomState(int(z["table_seed"])).randn(2 ** 22).astype(np.float32)
    off = int(z["param_offset"])
    theta = (table[off:off + P] * np.float32(0.1)).astype(np.float32)
    return theta, table, [(theta + s * table[o:o + P]).astype(np.float32) for s, o in zip(z["scales"], z["offs"])]


def test_impala_history_replacement_matches_reference(golden):
    """G12-impala: oracle.history over ImpalaPolicy strategies (oracle.impala.strategy from the reset state:
    the zeta obs as ONE LSTM sequence, policies/impala.py:24-27) reproduces the reference StrategyHandler /
    SparseHistoryManager run with get_strategy from reset -- returns, worst_point_idx trace, archive, distances
    and compute_novelty."""
    from oracle import history
    from oracle import impala as oi
    from oracle import novelty as onov
    z = golden("g12_impala.npz")
    A, H = int(z["A"]), int(z["H"])
    _, _, flats = _g12i_flats(z)
    bn = oi.split_bn(z["rm"], z["rv"])
    fr = z["zeta_frames"].astype(np.float32)

    def strat(f):
        return oi.strategy(oi.unflatten(f, A), bn, fr, z["zeta_rewards"])[0]
    hist = history.History("tvd", H)
    for k in range(H):
        hist.submit(None, False)
    hist.evaluate([strat(f) for f in flats[:H]])
    worst, rets = [hist.worst_point_idx], []
    for k in range(H, len(flats)):
        r = hist.submit(strat(flats[k]), True)
        rets.append(-2 if r is None else r)
        worst.append(hist.worst_point_idx)
    np.testing.assert_array_equal(rets, z["returns"])
    np.testing.assert_array_equal(worst, z["worst"])
    np.testing.assert_allclose(np.stack(hist.strategies), z["strategies"], rtol=0, atol=1e-5)
    D = np.full((H, H), np.inf)
    for (i, j), d in hist.known.items():
        D[i, j] = D[j, i] = d
    np.testing.assert_allclose(D, z["dists"], rtol=1e-5)
    theta, table, _ = _g12i_flats(z)
    P = int(z["P"])
    for k, want in zip((0, len(flats) - 1), z["novelty"]):
        f = (theta - z["scales"][k] * table[z["offs"][k]:z["offs"][k] + P]).astype(np.float32)
        assert abs(onov.novelty(strat(f), np.stack(hist.strategies), "tvd") - want) <= 1e-5 * max(1.0, want)


def test_impala_history_unpatched_reference_carried_state(golden):
    """G12-impala-unpatched: the same archive run with the reference's get_strategy as it is, where
    every StrategyPoint.evaluate_strategy continues the LSTM state the previous call left in the shared policy
    object (policies/impala.py:24-27; strategy_point.py:17-25).  The oracle reproduces it by carrying (h, c) through
    the reference's call order -- set_zeta evaluates points 0..H-1, every _replace_point one candidate,
    compute_novelty one policy -- which pins the reference's behaviour and the size of the build's documented
    divergence (the zero-state rule): the two fixtures' archives differ by up to ~0.65 in a probability."""
    from oracle import history
    from oracle import impala as oi
    from oracle import novelty as onov
    z = golden("g12_impala_unpatched.npz")
    zp = golden("g12_impala.npz")
    A, H = int(z["A"]), int(z["H"])
    _, _, flats = _g12i_flats(z)
    bn = oi.split_bn(z["rm"], z["rv"])
    fr = z["zeta_frames"].astype(np.float32)
    state = [None, None]

    def strat(f):
        pr, h, c = oi.strategy(oi.unflatten(f, A), bn, fr, z["zeta_rewards"], state[0], state[1])
        state[0], state[1] = h, c
        return pr
    hist = history.History("tvd", H)
    for k in range(H):
        hist.submit(None, False)
    hist.evaluate([strat(f) for f in flats[:H]])
    worst, rets = [hist.worst_point_idx], []
    for k in range(H, len(flats)):
        r = hist.submit(strat(flats[k]), True)
        rets.append(-2 if r is None else r)
        worst.append(hist.worst_point_idx)
    np.testing.assert_array_equal(rets, z["returns"])
    np.testing.assert_array_equal(worst, z["worst"])
    np.testing.assert_allclose(np.stack(hist.strategies), z["strategies"], rtol=0, atol=1e-5)
    theta, table, _ = _g12i_flats(z)
    P = int(z["P"])
    for k, want in zip((0, len(flats) - 1), z["novelty"]):
        f = (theta - z["scales"][k] * table[z["offs"][k]:z["offs"][k] + P]).astype(np.float32)
        assert abs(onov.novelty(strat(f), np.stack(hist.strategies), "tvd") - want) <= 1e-5 * max(1.0, want)
    # the recorded divergence of the zero-state rule from the unpatched reference
    d = float(np.abs(zp["strategies"] - z["strategies"]).max())
    assert 0.1 < d < 1.0, d
