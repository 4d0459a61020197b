"""GPU: episodes that end before T (worker/agent.py:35-52: done -> reset, break).

The terminating synthetic envs (fdr_env_desc.done_threshold, fdr 0.4) end a lane's episode after the step whose next
state has |s'[done_dim]| > done_threshold, or at T.  Only the terminating kernel instances (FEAT bit 4) carry the
per-lane done test, in all three synthetic-env rollout kernels:
  * G13 (tests/golden/make_golden.py g13_worker_terminating): the REFERENCE's Worker.collect_returns(12) on the
    CartPole- and Hopper-shaped terminating envs with injected draws -- replayed through u_inject (each training
    episode consumes exactly its steps' draws of the injected stream): steps exact, rewards / entropies <= 1e-4 rel;
  * the counter-stream lanes of rollout_kernel, its WIDE variant and rollout_pair_kernel against the oracle
    (oracle/agent.py evaluate_lanes with the env's failure test): steps exact, rewards / entropies as the
    fixed-length parity tests, odd lane counts included (a pair wave with an idle half);
  * visited-state recording stops at the done step; the Welford obs statistics only sample visited states;
  * Worker.evaluate counts the true steps in cumulative_timesteps.
"""
import numpy as np
import pytest
import torch

from oracle import agent as oagent
from oracle import envs as oenvs
from oracle import noise as onoise
from oracle import policies as opol

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
TERM = {"cartpole_term": ("discrete", 4, 2, 500, 0.4, 1), "hopper_term": ("mujoco", 11, 3, 1000, 0.5, 1)}
IMPLS = ("single", "pair", "wide")


@pytest.fixture(scope="module")
def eng():
    from fdr import engine
    return engine


def _dev(a, dtype=None):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device=DEV)


@pytest.mark.parametrize("name", sorted(TERM))
def test_injected_draws_replay_reference_terminating_episodes(golden, name):
    from envs import SyntheticEnv
    from fdr import engine
    from utils import SharedNoiseTable
    g = golden("g13_worker_terminating.npz")
    kind, n_in, n_act, T, thr, dim = TERM[name]
    assert int(g[name + "_T"]) == T and tuple(g[name + "_done"]) == (thr, dim)
    theta = g[name + "_theta"]
    P = theta.size
    steps_ref = g[name + "_timesteps"]
    n = len(steps_ref)
    assert steps_ref.min() < T and len(set(steps_ref.tolist())) > 3     # the fixture really terminates early
    tab = SharedNoiseTable(2 ** 22, P, random_seed=124)
    worker_rng, agent_rng, inj = np.random.RandomState(3), np.random.RandomState(11), np.random.RandomState(31)
    k = 1 if kind == "discrete" else n_act
    u = np.zeros((n, T, k), np.float32)
    idx = np.zeros(n, np.int64)
    sign = np.zeros(n, np.int8)
    jig = np.zeros(n)
    for i in range(n):
        is_eval = worker_rng.uniform(0, 1) < 0.25                          # worker.py:23
        assert is_eval == bool(g[name + "_is_eval"][i])
        if not is_eval:
            idx[i] = int(tab.sample_batch(1)[0])                             # worker.py:27
            assert idx[i] == g[name + "_idx"][i]
            sign[i] = 1
            for t in range(int(steps_ref[i])):       # agent.py:43: one draw per step actually taken
                u[i, t] = np.float32(inj.uniform()) if kind == "discrete" else inj.randn(n_act).astype(np.float32)
        jig[i] = agent_rng.choice((-1e-12, 1e-12))                           # agent.py:69
    env = SyntheticEnv(n_in, n_act, kind == "discrete", T, env_seed=0, device=DEV, done_threshold=thr, done_dim=dim)
    spec = engine.PolicySpec(kind, n_in, n_act, P)
    lanes = engine.lanes_desc(_dev(theta), 0, tab.device_table(DEV), _dev(idx), _dev(sign), 0.02,
                              _dev((sign == 0).astype(np.int8)))
    res = engine.rollout(spec, env, lanes, n, 99, jiggle=False, u_inject=_dev(u))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(res.timesteps.cpu().numpy(), steps_ref)
    assert int(res.timesteps.sum()) == int(g[name + "_cumulative_timesteps"])     # agent.py:55
    np.testing.assert_allclose(res.reward.cpu().numpy() + jig, g[name + "_reward"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(res.entropy.cpu().numpy(), g[name + "_entropy"], rtol=1e-4, atol=1e-6)


def _case(name, L, seed=21, idx_seed=5, det_lanes=2):
    kind, n_in, n_act, T, thr, dim = TERM[name]
    pol = opol.TorchPolicy(kind, n_in, n_act, seed=124)
    theta = pol.get_flat()
    P = theta.size
    t = onoise.NoiseTable(1 << 22, P, 124)
    idx = np.random.RandomState(idx_seed).randint(0, t.max_idx, size=L).astype(np.int64)
    sign = np.ones(L, np.int8)
    sign[:L // 2 * 2:2] = -1
    sign[-det_lanes:] = 0
    det = (sign == 0).astype(np.int8)
    return kind, n_in, n_act, T, thr, dim, theta, t, idx, sign, det, seed


@pytest.mark.parametrize("name,L", [("cartpole_term", 64), ("cartpole_term", 13), ("hopper_term", 48),
                                    ("hopper_term", 9)])
def test_terminating_rollout_kernels_vs_oracle(eng, name, L):
    from envs import SyntheticEnv
    kind, n_in, n_act, T, thr, dim, theta, t, idx, sign, det, seed = _case(name, L)
    oenv = oenvs.BatchedSyntheticEnv(n_in, n_act, kind == "discrete", T, L, done_threshold=thr, done_dim=dim)
    r_ret, r_ent, r_steps, r_n2 = oagent.evaluate_lanes(kind, n_in, n_act, theta, t.table, idx, sign, 0.02, oenv, seed,
                                                        deterministic=det.astype(bool))
    assert r_steps.min() < T and len(set(r_steps.tolist())) > 3
    env = SyntheticEnv(n_in, n_act, kind == "discrete", T, env_seed=0, device=DEV, done_threshold=thr, done_dim=dim)
    spec = eng.PolicySpec(kind, n_in, n_act, theta.size)
    lanes = eng.lanes_desc(_dev(theta), 0, _dev(t.table), _dev(idx), _dev(sign), 0.02, _dev(det))
    got = {}
    try:
        for impl in IMPLS:
            eng.context().set_rollout_impl(impl)
            res = eng.rollout(spec, env, lanes, L, seed)
            torch.cuda.synchronize()
            got[impl] = res
            np.testing.assert_array_equal(res.timesteps.cpu().numpy(), r_steps, err_msg=impl)
            np.testing.assert_allclose(res.reward.cpu().numpy(), r_ret, rtol=1e-4, atol=1e-4, err_msg=impl)
            np.testing.assert_allclose(res.entropy.cpu().numpy(), r_ent, rtol=1e-5, atol=1e-5, err_msg=impl)
            np.testing.assert_allclose(res.norm2.cpu().numpy(), r_n2, rtol=1e-9, atol=0, err_msg=impl)
    finally:
        eng.context().set_rollout_impl("auto")
    # the same env without termination runs every lane to T (the fixed-length instances are untouched)
    env_fixed = SyntheticEnv(n_in, n_act, kind == "discrete", T, env_seed=0, device=DEV)
    res = eng.rollout(spec, env_fixed, lanes, L, seed)
    assert np.all(res.timesteps.cpu().numpy() == T)


@pytest.mark.parametrize("impl", IMPLS)
def test_terminating_states_stop_at_done(eng, impl):
    """save_states of a terminating episode (agent.py:36,58-59) holds exactly the visited observations."""
    from envs import SyntheticEnv
    name, L = "cartpole_term", 12
    kind, n_in, n_act, T, thr, dim, theta, t, idx, sign, det, seed = _case(name, L)
    oenv = oenvs.BatchedSyntheticEnv(n_in, n_act, True, T, L, done_threshold=thr, done_dim=dim)
    ref = oagent.evaluate_lanes(kind, n_in, n_act, theta, t.table, idx, sign, 0.02, oenv, seed,
                                deterministic=det.astype(bool), record_states=True)
    r_steps, r_states = ref[2], ref[-1]
    env = SyntheticEnv(n_in, n_act, True, T, env_seed=0, device=DEV, done_threshold=thr, done_dim=dim)
    spec = eng.PolicySpec(kind, n_in, n_act, theta.size)
    lanes = eng.lanes_desc(_dev(theta), 0, _dev(t.table), _dev(idx), _dev(sign), 0.02, _dev(det))
    states = torch.full((L, T, n_in), float("nan"), dtype=torch.float32, device=DEV)
    try:
        eng.context().set_rollout_impl(impl)
        res = eng.rollout(spec, env, lanes, L, seed, states=states)
        torch.cuda.synchronize()
    finally:
        eng.context().set_rollout_impl("auto")
    S = states.cpu().numpy()
    np.testing.assert_array_equal(res.timesteps.cpu().numpy(), r_steps)
    for l in range(L):
        n = int(r_steps[l])
        np.testing.assert_allclose(S[l, :n], r_states[l, :n], atol=1e-4)
        assert np.all(np.isnan(S[l, n:])), "state written after the done step (lane %d)" % l


def test_terminating_welford_samples_only_visited_states(eng):
    from envs import SyntheticEnv
    name, L = "hopper_term", 16
    kind, n_in, n_act, T, thr, dim, theta, t, idx, sign, det, seed = _case(name, L)
    chance = 0.25
    oenv = oenvs.BatchedSyntheticEnv(n_in, n_act, False, T, L, done_threshold=thr, done_dim=dim)
    ref = oagent.evaluate_lanes(kind, n_in, n_act, theta, t.table, idx, sign, 0.02, oenv, seed,
                                deterministic=det.astype(bool), obs_chance=chance)
    r_steps, stats = ref[2], ref[4]
    env = SyntheticEnv(n_in, n_act, False, T, env_seed=0, device=DEV, done_threshold=thr, done_dim=dim)
    spec = eng.PolicySpec(kind, n_in, n_act, theta.size)
    lanes = eng.lanes_desc(_dev(theta), 0, _dev(t.table), _dev(idx), _dev(sign), 0.02, _dev(det))
    res = eng.rollout(spec, env, lanes, L, seed, obs_stats=chance)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(res.timesteps.cpu().numpy(), r_steps)
    cnt = res.obs_count.cpu().numpy()
    np.testing.assert_array_equal(cnt, [s.count for s in stats])
    assert np.all(cnt <= r_steps) and cnt.sum() < chance * 2 * T * L
    for l in range(L):
        if stats[l].count:
            np.testing.assert_allclose(res.obs_mean.cpu().numpy()[l], stats[l].mean_, rtol=1e-5, atol=1e-5)


def test_worker_counts_true_steps(eng):
    """Worker.evaluate on a terminating env: cumulative_timesteps = the steps taken (agent.py:55), not lanes x T."""
    from envs import SyntheticEnv
    from policies import DiscretePolicy
    from utils import SharedNoiseTable
    from worker import Agent, Worker
    torch.manual_seed(124)
    pol = DiscretePolicy(4, 2, seed=124, device=DEV)
    env = SyntheticEnv.named("cartpole_term", device=DEV)
    agent = Agent(pol, env, random_seed=7)
    w = Worker(pol, agent, SharedNoiseTable(1 << 22, pol.num_params, 124), None, sigma=0.02)
    b1 = w.evaluate(64, antithetic=True, seed=3)
    b2 = w.evaluate(64, antithetic=True, seed=4)
    torch.cuda.synchronize()
    steps = int(b1.timesteps.sum()) + int(b2.timesteps.sum())
    assert steps < 2 * 128 * env.episode_len
    assert agent.cumulative_timesteps == steps
    assert agent.cumulative_timesteps == steps          # reading twice does not double count


def test_worker_eval_states_hold_only_visited_states(eng):
    """Worker.eval_states / collect_returns on a terminating env return exactly the visited
    observations of the eval episode (agent.py:36,58 saved_states), never the unwritten rows after the done step."""
    from envs import SyntheticEnv
    from policies import DiscretePolicy
    from utils import SharedNoiseTable
    from worker import Agent, Worker
    torch.manual_seed(124)
    pol = DiscretePolicy(4, 2, seed=124, device=DEV)
    env = SyntheticEnv.named("cartpole_term", device=DEV)
    agent = Agent(pol, env, random_seed=7)
    w = Worker(pol, agent, SharedNoiseTable(1 << 22, pol.num_params, 124), None, sigma=0.02, eval_prob=1.0)
    # the eval episode's own length: one deterministic unperturbed lane
    det = torch.ones(1, dtype=torch.int8, device=DEV)
    res = eng.rollout(pol.spec, env, eng.lanes_desc(pol.flat, 0, deterministic=det), 1, 0, jiggle=False)
    steps = int(res.timesteps[0].item())
    assert steps < env.episode_len, "pick a case whose eval episode terminates"
    st = w.eval_states()
    assert st.shape == (steps, 4) and np.all(np.isfinite(st))
    assert w.eval_states(max_states=3).shape == (min(3, steps), 4)
    rets = w.collect_returns(2)
    for r in rets:
        assert r.is_eval and len(r.eval_states) == steps
        assert np.all(np.isfinite(np.asarray(r.eval_states)))
