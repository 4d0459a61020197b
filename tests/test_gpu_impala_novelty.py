"""ImpalaPolicy strategies and novelty (BASELINE config 5: strategy.sparse_history_manager over an Impala
policy) on the GPU -- fdr_impala_strategies against the reference's own stacked-obs pass (G8 ent_probs) and
the oracle's restatement of get_strategy (oracle/impala.py strategy: ONE batch_first LSTM sequence over
the stacked zeta obs, policies/impala.py:24-27, from the reset state worker/agent.py:66 leaves).
Tolerances: f32 1e-5 abs on the reference fixture; 2e-5 abs over a 66-step sequence (crosses the 64-step
chunk of the input-projection GEMM); fp16 mode 2e-2 abs (SURVEY 8c fp16 tolerance)."""
import numpy as np
import pytest
import torch

from oracle import impala as oi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mods():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fdr import engine
    from policies import ImpalaPolicy
    from strategy import StrategyHandler
    from utils import math_helpers
    return engine, ImpalaPolicy, StrategyHandler, math_helpers


def _g8_policy(ImpalaPolicy, g8):
    A, P = int(g8["A"]), int(g8["P"])
    tab = np.random.RandomState(int(g8["table_seed"])).randn(2 ** 22).astype(np.float32)
    off = int(g8["param_offset"])
    pol = ImpalaPolicy((64, 64, 3), A, device="cuda")
    pol.set_trainable_flat((tab[off:off + P] * np.float32(0.1)).astype(np.float32))
    o = 0
    for m in pol.model.bn_layers():
        n = m.num_features
        m.running_mean.copy_(torch.as_tensor(g8["rm"][o:o + n]))
        m.running_var.copy_(torch.as_tensor(g8["rv"][o:o + n]))
        o += n
    return pol


def _obs(g8, q, t, done=None):
    return {"frame": g8["frames"][q, t].astype(np.float32).reshape(1, 1, 3, 64, 64),
            "reward": np.array([[g8["rewards"][q, t]]], np.float32),
            "done": np.array([[bool(g8["dones"][q, t]) if done is None else done]])}


def test_get_strategy_matches_reference(mods, golden):
    """ImpalaPolicy.get_strategy over the visited obs from the end-of-sequence state == the reference's
    stacked-obs forward (tests/golden/g8_impala.npz ent_probs, made by policies/impala.py itself)."""
    engine, ImpalaPolicy, _, _ = mods
    g8 = golden("g8_impala.npz")
    pol = _g8_policy(ImpalaPolicy, g8)
    T = g8["frames"].shape[1]
    for q in range(g8["frames"].shape[0]):
        pol.reset()
        for t in range(T):
            pol.forward(_obs(g8, q, t))
        h0, c0 = (s.clone() for s in pol.state)
        got = pol.get_strategy([_obs(g8, q, t, done=False) for t in range(T)])
        np.testing.assert_allclose(got, g8["ent_probs"][q], rtol=0, atol=1e-5)
        # the state advances to the end of the sequence (impala.py:184); entropy is the same sequence's
        assert not torch.equal(pol.state[0], h0)
        pol.state = (h0, c0)
        ent = pol.get_entropy([_obs(g8, q, t, done=False) for t in range(T)])
        ref = float(oi.categorical_entropy(g8["ent_probs"][q]).mean())
        assert abs(ent - ref) < 1e-5
        # fp16 mode (config 5) from the same state: within the fp16 tolerance of the f32 reference
        h, c = h0[:1].clone().contiguous(), c0[:1].clone().contiguous()
        bm, bv = pol.bn_stats()
        fr = torch.as_tensor(g8["frames"][q].astype(np.float32), device="cuda")
        rw = torch.as_tensor(g8["rewards"][q], device="cuda")
        ph = engine.impala_strategies(engine.ImpalaSpec(int(g8["A"]), fp16=True), engine.lanes_desc(pol.flat, 0), 1,
                                      fr, rw, h, c, bm, bv)
        np.testing.assert_allclose(ph[0].cpu().numpy(), g8["ent_probs"][q], rtol=0, atol=2e-2)


@pytest.mark.parametrize("fp16,pairs", [(False, False), (True, False), (True, True)])
def test_lane_novelty_matches_oracle(mods, fp16, pairs):
    """Novelty of every perturbed lane against an archive (worker/worker.py:53 -> strategy_handler.py:25-30,
    categorical_tvd) == the oracle's per-lane get_strategy + TVD min, 66 probe obs, antithetic lanes.  pairs: the
    fp16 recurrence in the rollout's pair form (core_kernel_hpm2<1, kStrategy> + xproj_pair_kernel: f16(theta) +
    s f16(sigma eps) instead of f16(theta')) -- same tolerance, and not the per-lane path's bits."""
    engine, ImpalaPolicy, StrategyHandler, mh = mods
    A, Z, sigma = 4, 66, 0.02
    torch.manual_seed(5)
    pol = ImpalaPolicy((64, 64, 3), A, device="cuda")
    theta = pol.get_trainable_flat().astype(np.float32)
    P = theta.size
    tab = np.random.RandomState(124).randn(2 ** 22).astype(np.float32)
    rs = np.random.RandomState(9)
    frames = rs.randint(0, 256, size=(Z, 3, 64, 64)).astype(np.float32)
    rewards = rs.choice([-1.0, 0.0, 1.0, 2.0], size=Z).astype(np.float32)
    idx = np.repeat(rs.randint(0, tab.size - P, size=2), 2).astype(np.int64)
    sign = np.array([1, -1, 1, -1], np.int8)
    archive = [theta + np.float32(0.05) * tab[1000 + k:1000 + k + P] for k in range(3)]
    h = StrategyHandler(pol, mh.categorical_tvd, max_history_size=8, fp16=fp16)
    h.points = [a.astype(np.float32) for a in archive]
    h.set_zeta({"frame": frames, "reward": rewards, "done": np.zeros(Z, bool)})
    tab_d = torch.as_tensor(tab, device="cuda")
    idx_d, sign_d = torch.as_tensor(idx, device="cuda"), torch.as_tensor(sign, device="cuda")
    got = h.lane_strategies(tab_d, idx_d, sign_d, sigma, pairs=pairs).cpu().numpy()
    nov = h.lane_novelty(tab_d, idx_d, sign_d, sigma, pairs=pairs).cpu().numpy()
    if pairs:
        per_lane = h.lane_strategies(tab_d, idx_d, sign_d, sigma).cpu().numpy()
        assert not np.array_equal(got, per_lane)
        np.testing.assert_allclose(got, per_lane, rtol=0, atol=2e-2)
    zero = np.zeros(oi.num_bn(), np.float32)
    one = np.ones(oi.num_bn(), np.float32)
    ref = oi.lane_strategies(theta, tab, idx, sign, sigma, A, frames, rewards, zero, one)
    arch = np.stack([oi.strategy(oi.unflatten(a, A), oi.split_bn(zero, one), frames, rewards)[0] for a in archive])
    tol = 2e-2 if fp16 else 2e-5
    np.testing.assert_allclose(got, ref, rtol=0, atol=tol)
    np.testing.assert_allclose(h.archive.cpu().numpy(), arch, rtol=0, atol=tol)
    ref_nov = np.array([min(float(mh.categorical_tvd(s, b)) for b in arch) for s in ref])
    np.testing.assert_allclose(nov, ref_nov, rtol=0, atol=(2e-2 if fp16 else 1e-5))
    # a +eps lane and its -eps partner are different policies
    assert np.abs(got[0] - got[1]).max() > 1e-6


def test_eval_states_and_zeta_frames(mods):
    """Worker.eval_states for an ImpalaPolicy: the frames / carried rewards of the recorded deterministic
    episode (fdr_impala_env_frames) == the oracle frame env over the kernel's own actions."""
    engine, ImpalaPolicy, _, _ = mods
    from envs import FrameEnv
    from utils import SharedNoiseTable
    from worker import Agent, Worker
    torch.manual_seed(3)
    pol = ImpalaPolicy((64, 64, 3), 5, device="cuda")
    env = FrameEnv(5, episode_len=12, envs_per_lane=1, env_seed=11)
    w = Worker(pol, Agent(pol, env, 3), SharedNoiseTable(1 << 22, pol.num_params, random_seed=1), None)
    st = w.eval_states(max_states=9)
    spec = engine.ImpalaSpec(5, 1, 12, entropy=False, env_seed=11)
    res = engine.impala_rollout(spec, engine.lanes_desc(pol.flat, 0, deterministic=torch.ones(1, dtype=torch.int8,
                                                                                               device="cuda")),
                                1, 0, jiggle=False, record=True)
    acts = res.actions[0].cpu().numpy()
    fr = st["frame"].cpu().numpy()
    assert fr.shape == (9, 3, 64, 64)
    for t in range(9):
        np.testing.assert_array_equal(fr[t], oi.frames(11, [0], t)[0].astype(np.float32))
    carried = [0.0] + [float(oi.rewards(11, [0], t, [acts[t]], 5)[0]) for t in range(8)]
    np.testing.assert_array_equal(st["reward"].cpu().numpy(), np.array(carried, np.float32))
    assert not st["done"].any()


def test_sequential_runner_impala_fp16_config5(mods):
    """BASELINE config 5 end to end at toy size: SequentialRunner on a Breakout-shaped frame env with
    ImpalaPolicy fp16 rollouts, 4 envs per perturbation, A = 4, the TVD novelty archive and AdaptiveOmega."""
    from run_sequential import SequentialRunner
    r = SequentialRunner(env_id="BreakoutNoFrameskip-v4", envs_per_lane=4, fp16=True, antithetic=True, batch_size=4,
                         episode_len=12, zeta_size=16, eval_prob=0.5, max_strategy_history_size=4, random_seed=3,
                         noise_table_size=1 << 22, device="cuda", verbose=False)
    assert r.policy.KIND == "impala" and r.env.act_dim == 4 and r.strategy_handler.fp16
    assert r.zeta["frame"].shape == (16, 3, 64, 64)
    r.train(4)
    assert len(r.history) == 4
    for rep in r.history:
        assert np.isfinite(rep["Noisy Reward"]) and np.isfinite(rep["Noisy Novelty"])
        assert rep["Update Magnitude"] > 0
        assert len(rep["rewards"]) == 4 * 2 * 4      # directions x antithetic x envs
    assert len(r.omega.reward_history) >= 1           # omega stepped on the eval epochs (run_sequential.py:149-151)
    # add_policy at start + once per epoch: the 5th submission meets a full archive (max 4) -> _replace_point
    assert len(r.strategy_handler.points) == 4
    assert r.strategy_handler.archive is not None and r.strategy_handler.archive.shape[1:] == (16, 4)
